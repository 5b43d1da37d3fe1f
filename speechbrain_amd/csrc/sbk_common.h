// Shared device helpers for the sbk (speechbrain-amd kernels) library.
// gfx950 / CDNA4 only: wave64, 160 KiB LDS per CU, fp32 + bf16 MFMA.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include <mutex>

#define SBK_API extern "C" __attribute__((visibility("default")))

#define SBK_CHECK_LAUNCH()                          \
  do {                                              \
    hipError_t _e = hipGetLastError();              \
    if (_e != hipSuccess) return (int)_e;           \
  } while (0)

#define SBK_ERR_ARG 1001  // invalid argument (shape/config) detected on host

// Timeline probes: s_memtime marks compiled only into the probe builds of
// scripts/probe_build.sh (-DSBK_PROBE_TL, never the product library, which
// the probe scripts then load in its place); in the product every
// SBK_PROBE(...) expands to nothing.
#ifdef SBK_PROBE_TL
#define SBK_PROBE(...) __VA_ARGS__
#else
#define SBK_PROBE(...)
#endif
// a device buffer of probe marks and its host read-back entry
#define SBK_PROBE_BUFFER(name, rows, cols) SBK_PROBE(__device__ unsigned long long name[rows][cols];)
#define SBK_PROBE_EXPORT(fn, name)                                                                     \
  SBK_PROBE(SBK_API int fn(unsigned long long* out) {                                                  \
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(name), sizeof(name), 0, hipMemcpyDeviceToHost);    \
  })

namespace sbk {

constexpr int kWave = 64;

// Opt a kernel into `bytes` of dynamic LDS (> 64 KB needs it) on the current
// device.  hipFuncSetAttribute is per device, so the record is per (kernel,
// device), and it keeps the largest size set so far: a later launch asking
// for more sets the attribute again.  Thread-safe; host only.
inline hipError_t lds_optin(const void* kern, size_t bytes) {
  struct Entry {
    const void* kern;
    int dev;
    size_t bytes;
  };
  static std::mutex mu;
  static Entry table[512];
  static int n = 0;
  int dev = 0;
  if (hipError_t e = hipGetDevice(&dev)) return e;
  std::lock_guard<std::mutex> lock(mu);
  int i = 0;
  while (i < n && !(table[i].kern == kern && table[i].dev == dev)) ++i;
  if (i < n && table[i].bytes >= bytes) return hipSuccess;
  if (hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes)) return e;
  if (i < n) table[i].bytes = bytes;
  else if (n < 512) table[n++] = Entry{kern, dev, bytes};
  return hipSuccess;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// VALU-only cross-lane reductions (gfx950).  __shfl_xor lowers to
// ds_bpermute_b32: each step is an LDS-pipe round trip (~50+ cycles) behind a
// full lgkmcnt wait.  These use DPP row permutes and the gfx950
// v_permlane32_swap / v_permlane16_swap half-swaps instead.  Every step adds
// the same two operands in both partner lanes (involutive permutes), so all
// lanes of the reduced group end with the identical value.
//
// sum / max over the 4 lanes {l, l^16, l^32, l^48}: one column of a 16x16
// MFMA tile
__device__ __forceinline__ float col4_sum(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ float col4_max(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// whole-wave sum: row_mirror, row_half_mirror, quad_perm [2,3,0,1] and
// [1,0,3,2] inside each 16-lane row, then col4_sum across the rows
__device__ __forceinline__ float wave_sum_v(float v) {
  v += dpp_f32<0x140>(v);
  v += dpp_f32<0x141>(v);
  v += dpp_f32<0x4E>(v);
  v += dpp_f32<0xB1>(v);
  return col4_sum(v);
}

// Monotone float <-> int32 key so that atomicMax on the key orders floats.
__device__ __forceinline__ int float_to_key(float f) {
  int i = __float_as_int(f);
  return i >= 0 ? i : (i ^ 0x7FFFFFFF);
}
__device__ __forceinline__ float key_to_float(int k) {
  return __int_as_float(k >= 0 ? k : (k ^ 0x7FFFFFFF));
}

__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
// Round-to-nearest-even f32 -> bf16 (NaN handled by the hardware cvt path
// where the compiler emits v_cvt_pk_bf16_f32).
// fp32 -> bf16, round to nearest even, on the gfx950 conversion instruction
// (v_cvt_pk_bf16_f32: one VALU op; the software rounding of __float2bfloat16
// was ~5 and sat in the VALU-bound epilogues of the fused kernels).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}
// two values packed (lo in bits 0-15): one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2_t{lo, hi}, b2_t));
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024). `red` >= 16 floats.
// Block-wide max (all threads get the result); red: >= blockDim/64 floats.
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float m = red[0];
  for (int i = 1; i < nw; ++i) m = fmaxf(m, red[i]);
  return m;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

}  // namespace sbk
