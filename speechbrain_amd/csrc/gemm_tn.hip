// Weight-gradient GEMM (bf16 MFMA, fp32 accumulation):
//
//   C[b] (+)= A[b]^T · B[b]      A (K, M), B (K, N) row-major, C (M, N) fp32
//
// the backward of every nn.Linear / 1x1 conv / im2col conv of the training
// path (dW = dY^T X: the contraction runs over the B*T token rows, which are
// the ROWS of both stored operands), and the batched products of the
// attention backward of the same shape.  Reference sites: the autograd of
// torch.nn.Linear under speechbrain/nnet/linear.py:15-76 and of the ConvBlock
// convolutions (speechbrain/lobes/models/convolution.py:112-175).
//
// Both operands are staged k-major exactly as stored ([64 k][128 + 16] bf16
// tiles, register-prefetched one step ahead) and read k-transposed for the
// MFMA with ds_read_b64_tr_b16, so no transpose pass over the (tokens x
// features) tensors exists.  128 x 128 or 64 x 64 output tiles, 4 waves as
// 2 x 2, and the K (token) range split over workgroups; partial tiles are
// added into C with fp32 atomics (C is initialised by the caller), columns /
// rows past M / N never stored.  The split count is bounded by the total
// atomic traffic, which dominated the first version (32-way splits).
#include "mfma.h"

using namespace sbk;

namespace {

constexpr int TN_BK = 64, TN_LD = 144;

__device__ __forceinline__ bf16x8 frag_tr(const bf16_t* X, int k0, int dbase, int lane) {
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const bf16_t* a0 = X + (k0 + 4 * g + q) * TN_LD + dbase + 4 * p;
  const bf16_t* a1 = a0 + 16 * TN_LD;
  const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4_t*)(a0));
  const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4_t*)(a1));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

struct TnArgs {
  const bf16_t* A;
  const bf16_t* B;
  float* C;
  long long lda, ldb, ldc, sA, sB, sC;
  int M, N, K, kchunk, nsplit;
};

// BM x BN output tile (BM, BN in {64, 128}), 4 waves as 2 x 2, each wave
// (BM / 2) x (BN / 2) = MI x NI MFMA tiles of 16 x 16.
template <int BM, int BN>
__global__ void __launch_bounds__(256) gemm_tn_kernel(TnArgs a) {
  constexpr int MI = BM / 32, NI = BN / 32, CA = BM / 32, CB = BN / 32;  // MFMA tiles / 16-B chunks per thread
  __shared__ __attribute__((aligned(16))) bf16_t As[TN_BK * TN_LD];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[TN_BK * TN_LD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int bz = blockIdx.z / a.nsplit, sp = blockIdx.z - bz * a.nsplit;
  const int k0 = sp * a.kchunk, k1 = min(a.K, k0 + a.kchunk);
  const bf16_t* A = a.A + bz * a.sA;
  const bf16_t* B = a.B + bz * a.sB;
  float* C = a.C + bz * a.sC;
  // chunk c of a step: row c / (BM / 8), columns 8 (c % (BM / 8)).  DEPTH
  // register sets: the loads of step kt + DEPTH are issued right after step
  // kt's set is stored to LDS.  Measured: DEPTH 4 (64-tile) / 2 (128-tile)
  // is no faster than 1 (the step is bound by its store -> barrier -> read
  // -> MFMA -> barrier chain, not by the global loads) and costs VGPRs.  A
  // double-buffered LDS variant (one barrier per step) was no faster either
  // (t64: 117 vs 112 us at one split; profiles/r02_gemm_sweep*.log).
  constexpr int DEPTH = 1;
  uint4 ra[DEPTH][CA], rb[DEPTH][CB];
  auto gload = [&](uint4 (&xa)[CA], uint4 (&xb)[CB], int kb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int c = tid + i * 256, r = kb + c / (BM / 8), cc = (c % (BM / 8)) * 8;
      const bool rk = r < k1;
      xa[i] = rk && m0 + cc < a.M ? *reinterpret_cast<const uint4*>(A + (long long)(rk ? r : k0) * a.lda + m0 + cc)
                                  : uint4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = tid + i * 256, r = kb + c / (BN / 8), cc = (c % (BN / 8)) * 8;
      const bool rk = r < k1;
      xb[i] = rk && n0 + cc < a.N ? *reinterpret_cast<const uint4*>(B + (long long)(rk ? r : k0) * a.ldb + n0 + cc)
                                  : uint4{0u, 0u, 0u, 0u};
    }
  };
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (k1 - k0 + TN_BK - 1) / TN_BK;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (d < nk) gload(ra[d], rb[d], k0 + d * TN_BK);
  for (int kt0 = 0; kt0 < nk; kt0 += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int kt = kt0 + d;
      if (kt >= nk) break;  // uniform
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const int c = tid + i * 256;
        *reinterpret_cast<uint4*>(As + (c / (BM / 8)) * TN_LD + (c % (BM / 8)) * 8) = ra[d][i];
      }
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        const int c = tid + i * 256;
        *reinterpret_cast<uint4*>(Bs + (c / (BN / 8)) * TN_LD + (c % (BN / 8)) * 8) = rb[d][i];
      }
      __syncthreads();
      if (kt + DEPTH < nk) gload(ra[d], rb[d], k0 + (kt + DEPTH) * TN_BK);
#pragma unroll
      for (int kk = 0; kk < TN_BK / 32; ++kk) {
        bf16x8 fa[MI], fb[NI];
#pragma unroll
        for (int i = 0; i < MI; ++i) fa[i] = frag_tr(As, kk * 32, wm * (BM / 2) + i * 16, lane);
#pragma unroll
        for (int j = 0; j < NI; ++j) fb[j] = frag_tr(Bs, kk * 32, wn * (BN / 2) + j * 16, lane);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
      __syncthreads();
    }
  }
  // D[m][n]: lane holds rows m = 4g + r, column n = lane & 15 of each tile;
  // one split (nsplit == 1) stores, several add with fp32 atomics
  const int g = lane >> 4, fr = lane & 15;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * (BM / 2) + i * 16 + 4 * g + r;
      if (m >= a.M) continue;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int n = n0 + wn * (BN / 2) + j * 16 + fr;
        if (n < a.N) {
          float* cp = C + (long long)m * a.ldc + n;
          if (a.nsplit == 1) *cp += acc[i][j][r];
          else atomicAdd(cp, acc[i][j][r]);
        }
      }
    }
}


// Exact-fp32 variant (the fp32 parity mode of the training path): the same
// token-major staging with fp32 operands, 64 x 64 tiles, 32 k-rows per
// step, read for v_mfma_f32_16x16x4_f32 (lane l: row / column l & 15 of the
// tile, k-row l >> 4 of the 4-deep slice) — one ds_read_b32 per fragment,
// the 16 lanes of a k-row on consecutive banks (row stride 64 + 16 floats).
// Operands with M, N, lda or ldb not a multiple of 4 (or unaligned) load
// element-wise (`vec` false), so any shape is accepted.
constexpr int TF_BK = 32, TF_LD = 80;

__global__ void __launch_bounds__(256) gemm_tn_f32_kernel(const float* __restrict__ Ap, const float* __restrict__ Bp,
                                                          float* __restrict__ Cp, long long lda, long long ldb,
                                                          long long ldc, long long sA, long long sB, long long sC, int M,
                                                          int N, int K, int kchunk, int nsplit, int vec) {
  __shared__ __attribute__((aligned(16))) float As[TF_BK * TF_LD];
  __shared__ __attribute__((aligned(16))) float Bs[TF_BK * TF_LD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  const int bz = blockIdx.z / nsplit, sp = blockIdx.z - bz * nsplit;
  const int k0 = sp * kchunk, k1 = min(K, k0 + kchunk);
  const float* A = Ap + bz * sA;
  const float* B = Bp + bz * sB;
  float* C = Cp + bz * sC;
  // 32 k-rows x 64 columns = 512 float4 chunks per operand: 2 per thread
  float4 ra[2], rb[2];
  auto ld4 = [&](const float* X, long long ld, int r, int c, int lim) __attribute__((always_inline)) {
    const float* p = X + (long long)r * ld + c;
    if (vec) return c < lim ? *reinterpret_cast<const float4*>(p) : make_float4(0.f, 0.f, 0.f, 0.f);
    return make_float4(c < lim ? p[0] : 0.f, c + 1 < lim ? p[1] : 0.f, c + 2 < lim ? p[2] : 0.f,
                       c + 3 < lim ? p[3] : 0.f);
  };
  auto gload = [&](int kb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * 256, r = kb + (c >> 4), cc = (c & 15) * 4;
      const bool rk = r < k1;
      ra[i] = rk ? ld4(A, lda, r, m0 + cc, M) : make_float4(0.f, 0.f, 0.f, 0.f);
      rb[i] = rk ? ld4(B, ldb, r, n0 + cc, N) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (k1 - k0 + TF_BK - 1) / TF_BK;
  if (nk > 0) gload(k0);
  const int fr = lane & 15, g = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * 256;
      *reinterpret_cast<float4*>(As + (c >> 4) * TF_LD + (c & 15) * 4) = ra[i];
      *reinterpret_cast<float4*>(Bs + (c >> 4) * TF_LD + (c & 15) * 4) = rb[i];
    }
    __syncthreads();
    if (kt + 1 < nk) gload(k0 + (kt + 1) * TF_BK);
#pragma unroll
    for (int kk = 0; kk < TF_BK / 4; ++kk) {
      const int kr = (4 * kk + g) * TF_LD;
      float fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = As[kr + wm * 32 + i * 16 + fr];
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = Bs[kr + wn * 32 + j * 16 + fr];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * 32 + i * 16 + 4 * g + r;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn * 32 + j * 16 + fr;
        if (n < N) {
          float* cp = C + (long long)m * ldc + n;
          if (nsplit == 1) *cp += acc[i][j][r];
          else atomicAdd(cp, acc[i][j][r]);
        }
      }
    }
}

}  // namespace

// C[b] += A[b]^T B[b] for b < batch.  A (K, M) with row stride lda, B (K, N)
// row stride ldb, bf16; C (M, N) fp32 row stride ldc (caller-initialised);
// sA / sB / sC batch strides in elements.  M, N, lda, ldb multiples of 8
// and A, B 16-B aligned (16-B row chunks).
// tile 128 / 64 (square), nsplit >= 1 token-range splits (0 = choose)
SBK_API int sbk_gemm_tn_cfg(const void* A, long long lda, long long sA, const void* B, long long ldb, long long sB,
                            int M, int N, int K, int batch, float* C, long long ldc, long long sC, int tile, int nsplit,
                            void* stream) {
  if (!A || !B || !C || M <= 0 || N <= 0 || K < 0 || batch <= 0) return SBK_ERR_ARG;
  if ((M | N) % 8 || lda % 8 || ldb % 8 || lda < M || ldb < N || ldc < N) return SBK_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15 || (sA | sB) % 8) return SBK_ERR_ARG;
  if (K == 0) return 0;
  if (tile == 0) {
    // 128-wide tiles when they alone give >= 256 workgroups and neither side
    // is <= 64 (a half-empty tile), else 64
    const long long t128 = (long long)((M + 127) / 128) * ((N + 127) / 128) * batch;
    tile = t128 >= 256 && M > 64 && N > 64 ? 128 : 64;
  }
  if (tile != 64 && tile != 128) return SBK_ERR_ARG;
  const int tm = (M + tile - 1) / tile, tn = (N + tile - 1) / tile;
  const long long tiles = (long long)tm * tn * batch;
  if (nsplit <= 0) {
    // split the token range until ~1024 workgroups, >= 256 rows each, and at
    // most ~4M fp32 atomics in all (L2 atomic throughput, not the MFMA loop,
    // bounds a many-way split: 32 splits of a 1024 x 256 dW ran at 88-168 TF/s)
    nsplit = 1;
    while (tiles * nsplit * 2 <= 1024 && (long long)K / (nsplit * 2) >= 256 &&
           (long long)M * N * batch * nsplit * 2 <= (4LL << 20))
      nsplit *= 2;
  }
  const int kchunk = ((K + nsplit - 1) / nsplit + TN_BK - 1) / TN_BK * TN_BK;
  nsplit = (K + kchunk - 1) / kchunk;
  if ((long long)batch * nsplit > 65535) return SBK_ERR_ARG;
  TnArgs a{reinterpret_cast<const bf16_t*>(A), reinterpret_cast<const bf16_t*>(B), C, lda, ldb, ldc, sA, sB, sC,
           M, N, K, kchunk, nsplit};
  if (tile == 128)
    hipLaunchKernelGGL((gemm_tn_kernel<128, 128>), dim3(tm, tn, batch * nsplit), dim3(256), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL((gemm_tn_kernel<64, 64>), dim3(tm, tn, batch * nsplit), dim3(256), 0, (hipStream_t)stream, a);
  SBK_CHECK_LAUNCH();
  return 0;
}

// C[b] += A[b]^T B[b] for b < batch.  A (K, M) with row stride lda, B (K, N)
// row stride ldb, bf16; C (M, N) fp32 row stride ldc (caller-initialised);
// sA / sB / sC batch strides in elements.  M, N, lda, ldb multiples of 8
// and A, B 16-B aligned (16-B row chunks).
SBK_API int sbk_gemm_tn(const void* A, long long lda, long long sA, const void* B, long long ldb, long long sB,
                        int M, int N, int K, int batch, float* C, long long ldc, long long sC, void* stream) {
  return sbk_gemm_tn_cfg(A, lda, sA, B, ldb, sB, M, N, K, batch, C, ldc, sC, 0, 0, stream);
}

// fp32 operands (exact-f32 MFMA): C[b] += A[b]^T B[b], arguments as
// sbk_gemm_tn; any M, N, lda, ldb (element-wise loads unless all are
// multiples of 4 with 16-B aligned A, B and batch strides).  The weight
// gradient dW = dY^T X of the fp32 (parity) training path.  nsplit: token-
// range splits (0 = choose; 1 = plain stores, deterministic).
SBK_API int sbk_gemm_tn_f32(const float* A, long long lda, long long sA, const float* B, long long ldb, long long sB,
                            int M, int N, int K, int batch, float* C, long long ldc, long long sC, int nsplit,
                            void* stream) {
  if (!A || !B || !C || M <= 0 || N <= 0 || K < 0 || batch <= 0 || nsplit < 0) return SBK_ERR_ARG;
  if (lda < M || ldb < N || ldc < N) return SBK_ERR_ARG;
  if (K == 0) return 0;
  const int vec = ((M | N) % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && (sA | sB) % 4 == 0 &&
                   ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) == 0);
  const int tm = (M + 63) / 64, tn = (N + 63) / 64;
  const long long tiles = (long long)tm * tn * batch;
  if (nsplit == 0) {
    nsplit = 1;
    while (tiles * nsplit * 2 <= 1024 && (long long)K / (nsplit * 2) >= 256 &&
           (long long)M * N * batch * nsplit * 2 <= (4LL << 20))
      nsplit *= 2;
  }
  const int kchunk = ((K + nsplit - 1) / nsplit + TF_BK - 1) / TF_BK * TF_BK;
  nsplit = (K + kchunk - 1) / kchunk;
  if ((long long)batch * nsplit > 65535) return SBK_ERR_ARG;
  hipLaunchKernelGGL(gemm_tn_f32_kernel, dim3(tm, tn, batch * nsplit), dim3(256), 0, (hipStream_t)stream, A, B, C, lda,
                     ldb, ldc, sA, sB, sC, M, N, K, kchunk, nsplit, vec);
  SBK_CHECK_LAUNCH();
  return 0;
}
