// Internal interface of the 256 x 256-tile bf16 GEMM (gemm256.hip), used by
// sbk_gemm's dispatch in gemm.hip.  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct Gemm256Epi {
  const float* bias;       // [N] or null
  int act;                 // 0 none, 1 Swish, 3 LeakyReLU, 4 GELU (GLU not supported)
  float slope;
  const float* res;        // [M, ldr] fp32 or null
  int ldr;
  float alpha;
  const uint8_t* rowmask;  // [M]: nonzero -> value 0 before the residual
  void* out;
  int ldc;
  int out_bf16;
};

// N % 256 == 0, K % 64 == 0, 16-B aligned bf16 operands with lda, ldw % 8 == 0,
// 16-B aligned bias / residual / out with ldr, ldc % 4 == 0.
bool gemm256_supported(int M, int N, int K, long long lda, long long ldw, const void* A, const void* W,
                       const Gemm256Epi& ep);
int gemm256_launch(const void* A, long long lda, const void* W, long long ldw, int M, int N, int K,
                   const Gemm256Epi& ep, hipStream_t s);

// MXFP8 form (sbk_mx_gemm's arguments; byte strides): K % 128 == 0,
// N % 256 == 0, 16-B aligned operand rows, 4-B aligned scale rows;
// out_mode 0 fp32, 1 bf16, 2 MXFP8 (+ out_scales).  Swish is not offered.
bool mx256_supported(int M, int N, int K, long long lda, long long ldsa, long long rpb, long long a_bs,
                     long long s_bs, long long ldw, long long ldsw, const void* A, const void* SA, const void* W,
                     const void* SW, const Gemm256Epi& ep, int out_mode, const void* out_scales);
int mx256_launch(const void* A, const void* SA, long long lda, long long ldsa, long long rpb, long long a_bs,
                 long long s_bs, const void* W, const void* SW, long long ldw, long long ldsw, int M, int N, int K,
                 const Gemm256Epi& ep, int out_mode, void* out_scales, long long ldso, hipStream_t s,
                 float* ws = nullptr, long long ws_floats = 0);
// fp32 workspace (floats) mx256_launch uses for its split-K tail at this
// shape (0: none; the launch runs whole tiles when ws is absent or smaller)
long long mx256_split_floats(int M, int N, int K, int out_mode);
