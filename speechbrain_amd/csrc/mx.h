// MXFP8 (OCP microscaling, e4m3 elements + one E8M0 exponent per 32
// consecutive elements along the contraction dimension) helpers for gfx950.
//
// Producers quantise with the smallest power-of-two scale that keeps the
// block inside the e4m3 range (|q| <= 448): E = ceil(log2(amax / 448)),
// q = x * 2^-E rounded to nearest even by v_cvt_pk_fp8_f32 (OCP e4m3fn on
// gfx950, not the MI300 fnuz encoding), scale byte = E + 127.  The consumer
// GEMM hands the scale bytes to v_mfma_scale_f32_32x32x64_f8f6f4, which
// applies 2^(Ea-127) * 2^(Eb-127) in hardware: no dequantisation pass and no
// global amax reduction anywhere.
#pragma once
#include "sbk_common.h"

namespace sbk {

constexpr float kE4M3Max = 448.f;

// Biased E8M0 exponent (0..254) for a block whose largest magnitude is amax.
// E = ceil(log2(amax / 448)) without the division: with amax = ma * 2^ea
// (ma in [0.5, 1)) and 448 = 0.875 * 2^9, amax / 448 = (ma / 0.875) *
// 2^(ea - 9), whose ceil-log2 is ea - 9, plus 1 when ma > 0.875 — equal to
// frexp(amax / 448)'s rule (m == 0.5 ? e - 1 : e) for every finite amax (the
// correctly rounded quotient never lands on a power of two the exact one
// misses), at a frexp and a compare instead of an IEEE divide (~15 VALU
// instructions in the epilogues that quantise every 32 outputs)
__device__ __forceinline__ int mx_scale_byte(float amax) {
  if (!(amax > 0.f)) return 0;  // all-zero block: 2^-127
  int ea;
  const float ma = frexpf(amax, &ea);
  int E = ea - 9 + (ma > 0.875f ? 1 : 0);
  E = E < -127 ? -127 : (E > 127 ? 127 : E);
  return E + 127;
}

__device__ __forceinline__ float mx_inv_scale(int byte) { return ldexpf(1.f, 127 - byte); }

__device__ __forceinline__ float clamp_e4m3(float q) { return __builtin_amdgcn_fmed3f(q, -kE4M3Max, kE4M3Max); }

// four floats (already scaled) -> four e4m3 bytes, little-endian in a dword
__device__ __forceinline__ uint32_t pack4_e4m3(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(clamp_e4m3(a), clamp_e4m3(b), 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(clamp_e4m3(c), clamp_e4m3(d), v, true);
  return (uint32_t)v;
}

// e4m3 byte -> float (used by the reference-check paths only)
__device__ __forceinline__ float e4m3_to_f32(uint32_t byte) {
  const uint32_t s = (byte >> 7) & 1, e = (byte >> 3) & 15, m = byte & 7;
  float v;
  if (e == 0)
    v = ldexpf((float)m, -9);  // subnormal: m/8 * 2^-6
  else if (e == 15 && m == 7)
    v = __builtin_nanf("");
  else
    v = ldexpf(1.f + (float)m / 8.f, (int)e - 7);
  return s ? -v : v;
}

// max over aligned groups of G consecutive lanes (G = 1, 2, ..., 32), VALU
// only: DPP row_mirror / row_half_mirror / quad permutes inside 16-lane rows
// (involutive, so every lane of a group ends with the group max), then
// v_permlane16_swap to pair rows 0-1 and 2-3 for G = 32.
template <int G>
__device__ __forceinline__ float group_max(float v) {
  static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16 || G == 32, "group size");
  if (G == 1) return v;
  if (G >= 16) v = fmaxf(v, dpp_f32<0x140>(v));
  if (G >= 8) v = fmaxf(v, dpp_f32<0x141>(v));
  if (G >= 4) v = fmaxf(v, dpp_f32<0x4E>(v));
  v = fmaxf(v, dpp_f32<0xB1>(v));
  if (G == 32) {
    const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
  }
  return v;
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

}  // namespace sbk
