// MFMA fragment traits shared by the GEMM and attention kernels.
//
// One abstraction for both compute dtypes: a lane of a 16x16 MFMA tile holds
// 8 consecutive K elements (k = 8*(lane>>4) + j, j = 0..7) of its A row and
// of its B column.
//   bf16: one v_mfma_f32_16x16x32_bf16 consumes the 8-element fragment.
//   f32 : eight v_mfma_f32_16x16x4_f32 (exact f32 FMA chains), instruction s
//         taking element s of every lane group, so together they cover the
//         same 32-wide K slice.  This keeps LDS layouts identical across
//         dtypes (8 contiguous K elements per lane = one or two 16-B reads).
// C/D layout of 16x16 MFMA: col = lane & 15, row = 4*(lane >> 4) + reg.
#pragma once
#include "sbk_common.h"

namespace sbk {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef uint16_t bf16_t;  // bf16 storage

template <typename T>
struct MT;

template <>
struct MT<bf16_t> {
  using frag = bf16x8;
  static constexpr int VEC = 8;  // elements per 16-byte chunk
  static constexpr int PAD = 8;  // LDS row padding (elements) = 16 bytes
  __device__ static __forceinline__ frag load(const bf16_t* p) { return *reinterpret_cast<const frag*>(p); }
  __device__ static __forceinline__ void mma(f32x4& c, const frag& a, const frag& b) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ frag zero() { return frag{}; }
  // elements 0..3 from p0, 4..7 from p1 (permuted-k fragments)
  __device__ static __forceinline__ frag load2x4(const bf16_t* p0, const bf16_t* p1) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const bf16x4 a = *reinterpret_cast<const bf16x4*>(p0);
    const bf16x4 b = *reinterpret_cast<const bf16x4*>(p1);
    return frag{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  }
  __device__ static __forceinline__ frag from8(const float* v) {
    frag f;
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = (__bf16)v[i];
    return f;
  }
  __device__ static __forceinline__ bf16_t from_f32(float v) { return f32_to_bf16(v); }
  __device__ static __forceinline__ float to_f32(bf16_t v) { return bf16_to_f32(v); }
};

template <>
struct MT<float> {
  using frag = f32x8;
  static constexpr int VEC = 4;
  static constexpr int PAD = 4;
  __device__ static __forceinline__ frag load(const float* p) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    frag v;
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    return v;
  }
  __device__ static __forceinline__ void mma(f32x4& c, const frag& a, const frag& b) {
#pragma unroll
    for (int s = 0; s < 8; ++s) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], c, 0, 0, 0);
  }
  __device__ static __forceinline__ frag zero() { return frag{}; }
  __device__ static __forceinline__ frag load2x4(const float* p0, const float* p1) {
    const float4 a = *reinterpret_cast<const float4*>(p0);
    const float4 b = *reinterpret_cast<const float4*>(p1);
    frag v;
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    return v;
  }
  __device__ static __forceinline__ frag from8(const float* v) {
    frag f;
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = v[i];
    return f;
  }
  __device__ static __forceinline__ float from_f32(float v) { return v; }
  __device__ static __forceinline__ float to_f32(float v) { return v; }
};

}  // namespace sbk
