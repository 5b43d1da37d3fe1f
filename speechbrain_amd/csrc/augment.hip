// SpecAugment kernels: bicubic / bilinear time warp, frequency/time masks, mean fill.
//
// Reference: speechbrain/lobes/augment.py:106-201 (SpecAugment.forward,
// time_warp, mask_along_axis).  The random draws (warp centre c and width w,
// mask lengths/positions) are made on the host with the CPU generator in the
// reference's order, so mask indices are bit-exact with the reference CPU
// path; the kernels only apply them.
//
// Data: x (N, T, F) fp32 (N = batch, or batch*channels for 4-D input).
//   warp kernel : y[n, t, :] = bicubic(x[n, 0:c, :] -> w rows)  for t <  w
//                              bicubic(x[n, c:T, :] -> T-w rows) for t >= w
//                 (align_corners=True, A=-0.75, border-clamped taps; the
//                  frequency axis keeps its size, where bicubic is the identity)
//                 + per-block partial sums for the mean fill.
//   apply kernel: x = time-masked ? mean2 : freq-masked ? mean1 : y
//                 (mean1 = mean after warp, mean2 = mean after freq masking,
//                  reduced in a fixed order from the partials -> deterministic)
// HBM traffic: read x, write y, read y, write x (the in-place contract needs
// the copy because warped rows move), or read+write x once without warp.
#include "sbk_common.h"

// No FMA contraction in this file: the warp weights and the source index are
// rounded op by op like the reference's float arithmetic (an fma of the
// index product shifts the bicubic phase by up to 1 ulp of the index).
#pragma clang fp contract(off)

using namespace sbk;

namespace {

__device__ __forceinline__ float cubic1(float x) {  // |x| <= 1
  const float A = -0.75f;
  return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f;
}
__device__ __forceinline__ float cubic2(float x) {  // 1 < |x| < 2
  const float A = -0.75f;
  return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A;
}

// Is frequency bin f of sequence n covered by one of its masks?
__device__ __forceinline__ bool in_masks(const int* m, int n, int nm, int i) {
  for (int k = 0; k < nm; ++k) {
    const int len = m[(n * nm + k) * 2 + 0], pos = m[(n * nm + k) * 2 + 1];
    if (pos <= i && i < pos + len) return true;
  }
  return false;
}

// number of (sequence, frequency) cells covered by a frequency mask
// (pos <= f < pos + len), over all sequences — reduced by the block.  The
// table is read through LDS (mlds, FM_LDS ints) when it fits: the checks of
// the (n, f) cells then cost no global round trip each.
constexpr int FM_LDS = 2048;
__device__ __forceinline__ long long fmask_cells(const int* fmask, int n_fmask, int N, int F, float* red, int* mlds,
                                                 bool prestaged = false) {
  const int nm = N * n_fmask * 2;
  const bool staged = nm <= FM_LDS;
  if (staged && !prestaged) {
    for (int i = threadIdx.x; i < nm; i += blockDim.x) mlds[i] = fmask[i];
    __syncthreads();
  }
  const int* m = staged ? mlds : fmask;
  float cnt = 0.f;  // exact: < 2^24 cells
  for (int i = threadIdx.x; i < N * F; i += blockDim.x) cnt += in_masks(m, i / F, n_fmask, i % F) ? 1.f : 0.f;
  return (long long)block_sum(cnt, red);
}

// One block per (n, tile of TT output rows); threads over F.  CUBIC: the
// bicubic resize (A = -0.75, border-clamped taps); else bilinear
// (time_warp_mode="bilinear": two taps, lambda0 = 1 - lambda1, the upper
// tap clamped to the last row) — torch's upsample_*2d with align_corners.
template <bool CUBIC>
__global__ void __launch_bounds__(256) warp_kernel(const float* __restrict__ x, float* __restrict__ y, int N, int T,
                                                   int F, int c, int w, int TT, const int* __restrict__ fmask,
                                                   int n_fmask, float* __restrict__ partial) {
  __shared__ float red[16];
  const int ntile = (T + TT - 1) / TT;
  const int n = blockIdx.x / ntile;
  const int t0 = (blockIdx.x - n * ntile) * TT;
  const int t1 = min(T, t0 + TT);
  const float* xn = x + (long long)n * T * F;
  float* yn = y + (long long)n * T * F;
  float s_all = 0.f, s_msk = 0.f;
  for (int t = t0; t < t1; ++t) {
    // segment: [0, w) <- x[0, c) ; [w, T) <- x[c, T)
    const bool left = t < w;
    const int in_rows = left ? c : T - c;
    const int out_rows = left ? w : T - w;
    const int src0 = left ? 0 : c;
    const int dst = left ? t : t - w;
    int idx[4];
    float wt[4];
    if (in_rows == out_rows) {
      idx[0] = idx[1] = idx[2] = idx[3] = dst;
      wt[0] = 0.f; wt[1] = 1.f; wt[2] = 0.f; wt[3] = 0.f;
    } else {
      // correctly rounded like the reference (a float divide may be 1 ulp off on the GPU)
      const float scale = out_rows > 1 ? (float)((double)(in_rows - 1) / (double)(out_rows - 1)) : 0.f;
      const float real = scale * (float)dst;
      const float fl = floorf(real);
      const float tt = real - fl;
      const int i0 = (int)fl;
      if (CUBIC) {
        wt[0] = cubic2(tt + 1.f);
        wt[1] = cubic1(tt);
        wt[2] = cubic1(1.f - tt);
        wt[3] = cubic2(2.f - tt);
#pragma unroll
        for (int k = 0; k < 4; ++k) idx[k] = min(max(i0 - 1 + k, 0), in_rows - 1);
      } else {
        const float l1 = fminf(fmaxf(tt, 0.f), 1.f);
        wt[0] = 1.f - l1;
        wt[1] = l1;
        wt[2] = wt[3] = 0.f;
        idx[0] = i0;
        idx[1] = i0 + (i0 < in_rows - 1 ? 1 : 0);
        idx[2] = idx[3] = i0;
      }
    }
    for (int f = threadIdx.x; f < F; f += blockDim.x) {
      float v;
      if (in_rows == out_rows) {
        v = xn[(long long)(src0 + dst) * F + f];
      } else {
        if (CUBIC) {
          v = 0.f;
#pragma unroll
          for (int k = 0; k < 4; ++k) v += wt[k] * xn[(long long)(src0 + idx[k]) * F + f];
        } else {
          v = wt[0] * xn[(long long)(src0 + idx[0]) * F + f] + wt[1] * xn[(long long)(src0 + idx[1]) * F + f];
        }
      }
      yn[(long long)t * F + f] = v;
      s_all += v;
      if (n_fmask && in_masks(fmask, n, n_fmask, f)) s_msk += v;
    }
  }
  if (partial) {
    const float a = block_sum(s_all, red);
    const float m = block_sum(s_msk, red);
    if (threadIdx.x == 0) {
      partial[2 * blockIdx.x] = a;
      partial[2 * blockIdx.x + 1] = m;
    }
  }
}

// Partial sums without a warp (mean fill on unwarped input).
__global__ void __launch_bounds__(256) sum_kernel(const float* __restrict__ x, int N, int T, int F, int TT,
                                                  const int* __restrict__ fmask, int n_fmask,
                                                  float* __restrict__ partial) {
  __shared__ float red[16];
  const int ntile = (T + TT - 1) / TT;
  const int n = blockIdx.x / ntile;
  const int t0 = (blockIdx.x - n * ntile) * TT;
  const int t1 = min(T, t0 + TT);
  const float* xn = x + (long long)n * T * F;
  float s_all = 0.f, s_msk = 0.f;
  for (int t = t0; t < t1; ++t)
    for (int f = threadIdx.x; f < F; f += blockDim.x) {
      const float v = xn[(long long)t * F + f];
      s_all += v;
      if (n_fmask && in_masks(fmask, n, n_fmask, f)) s_msk += v;
    }
  const float a = block_sum(s_all, red);
  const float m = block_sum(s_msk, red);
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = a;
    partial[2 * blockIdx.x + 1] = m;
  }
}

// x[n,t,f] = tmask ? fill_t : fmask ? fill_f : src[n,t,f]   (src may alias x)
__global__ void __launch_bounds__(256) apply_kernel(const float* src, float* x, int N, int T, int F, int TT,
                                                    const int* __restrict__ fmask, int n_fmask,
                                                    const int* __restrict__ tmask, int n_tmask,
                                                    const float* __restrict__ partial, int nparts,
                                                    long long n_fcells, int use_mean) {
  __shared__ float red[16];
  __shared__ float fills[2];
  __shared__ int mlds[FM_LDS];
  if (use_mean) {
    if (n_fcells < 0) n_fcells = n_fmask ? fmask_cells(fmask, n_fmask, N, F, red, mlds) * T : 0;
    // deterministic reduction of the per-block partial sums, same order in every block
    float a = 0.f, m = 0.f;
    for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
      a += partial[2 * i];
      m += partial[2 * i + 1];
    }
    a = block_sum(a, red);
    m = block_sum(m, red);
    if (threadIdx.x == 0) {
      const double total = (double)N * T * F;
      const float mean1 = (float)(a / total);
      fills[0] = mean1;
      fills[1] = (float)(((double)a - (double)m + (double)mean1 * (double)n_fcells) / total);
    }
  } else if (threadIdx.x == 0) {
    fills[0] = fills[1] = 0.f;
  }
  __syncthreads();
  const float fill_f = fills[0], fill_t = fills[1];
  const int ntile = (T + TT - 1) / TT;
  const int n = blockIdx.x / ntile;
  const int t0 = (blockIdx.x - n * ntile) * TT;
  const int t1 = min(T, t0 + TT);
  for (int t = t0; t < t1; ++t) {
    const bool tm = n_tmask && in_masks(tmask, n, n_tmask, t);
    for (int f = threadIdx.x; f < F; f += blockDim.x) {
      const long long i = ((long long)n * T + t) * F + f;
      float v;
      if (tm)
        v = fill_t;
      else if (n_fmask && in_masks(fmask, n, n_fmask, f))
        v = fill_f;
      else
        v = src[i];
      x[i] = v;
    }
  }
}

// ---- 4-wide path (F % 4 == 0, 16-B aligned x / scratch): the kernels
// above move one float per thread and every apply block re-reduced all the
// warp blocks' partial sums (3,008 blocks x 24 KB of L2 reads at config 2).
// Here a thread moves one float4 (its four frequency columns' mask bits
// computed once) for UR rows whose loads (all taps) are issued together, a
// block covers UR x (256 / (F/4)) rows (16 at F = 240: 3,008 blocks at
// config 2, ~12 per CU), and the two fills are reduced once by a one-block
// kernel.  (A first version walked 64 rows per block one row at a time:
// 752 blocks, each thread's 16 dependent-latency iterations; 104 us.)
constexpr int UR = 4;

__device__ __forceinline__ unsigned col_mask4(const int* m, int n, int nm, int f0) {
  unsigned cm = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (nm && in_masks(m, n, nm, f0 + e)) cm |= 1u << e;
  return cm;
}

__host__ __device__ __forceinline__ int rows_per_block4(int F) { return UR * (256 / (F >> 2)); }

// y = warp(x) (bicubic / bilinear as warp_kernel; c < 0: no warp, y unused)
// and the block's partial sums [all, freq-masked cells] of the warped values.
template <bool CUBIC, bool WARP>
__global__ void __launch_bounds__(256) warp4_kernel(const float* __restrict__ x, float* __restrict__ y, int N, int T,
                                                    int F, int c, int w, const int* __restrict__ fmask, int n_fmask,
                                                    float* __restrict__ partial) {
  constexpr int NTAP = WARP ? (CUBIC ? 4 : 2) : 1;
  __shared__ float red[16];
  const int F4 = F >> 2, rpp = 256 / F4, RB = UR * rpp;
  const int ntile = (T + RB - 1) / RB;
  const int n = blockIdx.x / ntile;
  const int t0 = (blockIdx.x - n * ntile) * RB;
  const int q = threadIdx.x % F4, tr = threadIdx.x / F4;
  const float* xn = x + (long long)n * T * F;
  float* yn = y + (long long)n * T * F;
  float s_all = 0.f, s_msk = 0.f;
  if (tr < rpp) {
    const unsigned cm = col_mask4(fmask, n, n_fmask, 4 * q);
    float4 a[UR][NTAP];
    float wt[UR][NTAP];
    bool ident[UR];
    // every tap of the UR rows first
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const int t = min(t0 + tr + u * rpp, T - 1);
      if constexpr (WARP) {
        const bool left = t < w;
        const int in_rows = left ? c : T - c, out_rows = left ? w : T - w;
        const int src0 = left ? 0 : c, dst = left ? t : t - w;
        ident[u] = in_rows == out_rows;
        const float scale = out_rows > 1 ? (float)((double)(in_rows - 1) / (double)(out_rows - 1)) : 0.f;
        const float real = scale * (float)dst;
        const float fl = floorf(real);
        const float tt = real - fl;
        const int i0 = (int)fl;
        if constexpr (CUBIC) {
          wt[u][0] = cubic2(tt + 1.f);
          wt[u][1] = cubic1(tt);
          wt[u][2] = cubic1(1.f - tt);
          wt[u][3] = cubic2(2.f - tt);
#pragma unroll
          for (int k = 0; k < NTAP; ++k) {
            const int r = ident[u] ? dst : min(max(i0 - 1 + k, 0), in_rows - 1);
            a[u][k] = *reinterpret_cast<const float4*>(xn + (long long)(src0 + r) * F + 4 * q);
          }
        } else {
          const float l1 = fminf(fmaxf(tt, 0.f), 1.f);
          wt[u][0] = 1.f - l1;
          wt[u][NTAP - 1] = l1;
          const int i1 = i0 + (i0 < in_rows - 1 ? 1 : 0);
          a[u][0] = *reinterpret_cast<const float4*>(xn + (long long)(src0 + (ident[u] ? dst : i0)) * F + 4 * q);
          a[u][NTAP - 1] = *reinterpret_cast<const float4*>(xn + (long long)(src0 + (ident[u] ? dst : i1)) * F + 4 * q);
        }
      } else {
        ident[u] = true;
        a[u][0] = *reinterpret_cast<const float4*>(xn + (long long)t * F + 4 * q);
      }
    }
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const int t = t0 + tr + u * rpp;
      if (t >= T) continue;
      float4 v;
      if (ident[u]) {
        v = a[u][WARP && CUBIC ? 1 : 0];
      } else {
        v = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (CUBIC) {
#pragma unroll
          for (int k = 0; k < NTAP; ++k) {
            v.x += wt[u][k] * a[u][k].x; v.y += wt[u][k] * a[u][k].y;
            v.z += wt[u][k] * a[u][k].z; v.w += wt[u][k] * a[u][k].w;
          }
        } else {
          const float l0 = wt[u][0], l1 = wt[u][NTAP - 1];
          const float4 a0 = a[u][0], a1 = a[u][NTAP - 1];
          v = make_float4(l0 * a0.x + l1 * a1.x, l0 * a0.y + l1 * a1.y, l0 * a0.z + l1 * a1.z, l0 * a0.w + l1 * a1.w);
        }
      }
      if (WARP) *reinterpret_cast<float4*>(yn + (long long)t * F + 4 * q) = v;
      s_all += v.x + v.y + v.z + v.w;
      s_msk += ((cm & 1) ? v.x : 0.f) + ((cm & 2) ? v.y : 0.f) + ((cm & 4) ? v.z : 0.f) + ((cm & 8) ? v.w : 0.f);
    }
  }
  if (partial) {
    const float a = block_sum(s_all, red);
    const float m = block_sum(s_msk, red);
    if (threadIdx.x == 0) {
      partial[2 * blockIdx.x] = a;
      partial[2 * blockIdx.x + 1] = m;
    }
  }
}

// ---- In place, 1R + ~1.1W (x read once, unmasked cells written once, the
// masked cells written by fixup4_kernel after the means are known).
// roll4_kernel: one workgroup per (utterance n, slab of J float4 columns),
// all T rows in order through a 1024-row LDS ring: window after window of WR
// = 512 output rows (32 KB of loads in flight per workgroup at J = 4, two or
// more workgroups per CU), each output row's taps (|p(t) - t| <= |c - w|, so rows
// t - H .. t + H with H = |c - w| + 3) read from the ring.  The next window's
// new input rows are loaded into registers while this window computes — they
// lie above every row this window writes — and stored into the ring after
// it, so an input row is read from HBM before the workgroup overwrites it and
// never again (the in-place hazard is confined to the workgroup that owns the
// column slab).  Per workgroup partials [sum, freq-masked sum, freq-masked
// columns of the slab] feed the means.
#ifndef SBK_RL_JMAX
#define SBK_RL_JMAX 2  // (probe builds vary the slab width: 2 measured 39.2-39.7 us, 4 41.3-41.4, 1 48.6-49.2 per call)
#endif
// Windows of 256 output rows in a 1024-row ring: 34.5-34.7 us per call at
// config 2 against 36.1-36.3 for 512 / 1024 (shorter first-window exposure,
// more windows to overlap; profiles/r05bh_sa_window_ab.log), with a halo of
// (1024 - 256) / 2 = 384 rows, up from 256
#ifndef SBK_RL_WR
#define SBK_RL_WR 256
#endif
#ifndef SBK_RL_RING
#define SBK_RL_RING 1024
#endif
constexpr int RL_WR = SBK_RL_WR, RL_RING = SBK_RL_RING, RL_HMAX = (RL_RING - RL_WR) / 2, RL_MAXM = 32,
              RL_JMAX = SBK_RL_JMAX;
static_assert((RL_RING & (RL_RING - 1)) == 0 && RL_WR < RL_RING && RL_WR * RL_JMAX % 256 == 0, "ring geometry");
template <bool CUBIC, bool WARP, bool MEAN>
__global__ void __launch_bounds__(256) roll4_kernel(float* __restrict__ x, int N, int T, int F, int J, int c, int w,
                                                    const int* __restrict__ fmask, int n_fmask,
                                                    const int* __restrict__ tmask, int n_tmask,
                                                    float* __restrict__ partial) {
  constexpr int NTAP = WARP ? (CUBIC ? 4 : 2) : 1;
  constexpr int PF = RL_WR * RL_JMAX / 256;  // prefetch float4 per thread at the widest slab
  // (HIP's float4 struct arrays stay in scratch; ext_vector_type ones are registers)
  typedef float v4f __attribute__((ext_vector_type(4)));
  extern __shared__ v4f ring[];         // RL_RING x J
  __shared__ float red[16];
  __shared__ int tms[2 * RL_MAXM];      // utterance n's time masks: no global load inside the row loop
  const int F4 = F >> 2, nslab = F4 / J;
  // XCD-aware bijective remap (workgroup i runs on XCD i % 8): the slabs of
  // an utterance — J * 16 B of every 128-B row line — go to one XCD, whose L2
  // then fetches each line once
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int slab = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int n = slab / nslab, j0 = (slab - n * nslab) * J;
  if ((int)threadIdx.x < 2 * n_tmask) tms[threadIdx.x] = tmask[2 * n * n_tmask + threadIdx.x];
  const int RP = 256 / J;               // rows per pass
  const int q = threadIdx.x % J, rp = threadIdx.x / J;
  const bool act = rp < RP;
  float* xn = x + (long long)n * T * F + 4 * (j0 + q);
  const int H = WARP ? abs(c - w) + 3 : 0;
  // the two segments' source scales (align_corners), once per workgroup
  float scl[2] = {0.f, 0.f};
  if constexpr (WARP) {
#pragma unroll
    for (int sg = 0; sg < 2; ++sg) {
      const int in_rows = sg == 0 ? c : T - c, out_rows = sg == 0 ? w : T - w;
      scl[sg] = out_rows > 1 ? (float)((double)(in_rows - 1) / (double)(out_rows - 1)) : 0.f;
    }
  }
  const unsigned cm = act ? col_mask4(fmask, n, n_fmask, 4 * (j0 + q)) : 0u;
  float s_all = 0.f, s_msk = 0.f;
  // rows [lo, hi) -> registers pf (row lo + rp + k * RP), then -> ring.
  // Unconditional loads (rows past the range clamp onto row T - 1 and are not
  // stashed): a conditional load per row compiled to a branch with a full
  // vmcnt wait after each, serialising the prefetch.
  v4f pf[PF];
#define RL_FETCH(lo)                                                                  \
  _Pragma("unroll") for (int k = 0; k < PF; ++k) {                                    \
    const int r_ = min((lo) + rp + k * RP, T - 1);                                    \
    pf[k] = *reinterpret_cast<const v4f*>(xn + (long long)r_ * F);                  \
  }
#define RL_STASH(lo, hi)                                                              \
  _Pragma("unroll") for (int k = 0; k < PF; ++k) {                                    \
    const int r_ = (lo) + rp + k * RP;                                                \
    if (act && r_ < (hi)) ring[(r_ & (RL_RING - 1)) * J + q] = pf[k];                 \
  }
  // rows [0, have) are staged; a window computes the output rows whose taps
  // are all staged, [t0, have - H) (all remaining rows once have = T), while
  // the next RL_WR input rows are in flight; a stash overwrites ring rows
  // below have - RL_RING + RL_WR <= have - 2H, which no later window reads
  int have = min(T, RL_WR);
  RL_FETCH(0);
  RL_STASH(0, have);
  __syncthreads();
  for (int t0 = 0; t0 < T;) {
    // (max: with H > RL_WR the first windows stage rows but complete none —
    // t1 must not fall below t0)
    const int t1 = have >= T ? T : max(t0, have - H);
    const int nlo = have, nhi = min(T, have + RL_WR);
    RL_FETCH(nlo);  // in flight under this window's compute
    if (act) {
      for (int t = t0 + rp; t < t1; t += RP) {
        v4f v;
        if constexpr (WARP) {
          const bool left = t < w;
          const int in_rows = left ? c : T - c, out_rows = left ? w : T - w;
          const int src0 = left ? 0 : c, dst = left ? t : t - w;
          if (in_rows == out_rows) {
            v = ring[((src0 + dst) & (RL_RING - 1)) * J + q];
          } else {
            const float real = scl[left ? 0 : 1] * (float)dst;
            const float fl = floorf(real);
            const float tt = real - fl;
            const int i0 = (int)fl;
            if constexpr (CUBIC) {
              const float wt[4] = {cubic2(tt + 1.f), cubic1(tt), cubic1(1.f - tt), cubic2(2.f - tt)};
              v = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
              for (int k = 0; k < NTAP; ++k) {
                const int r = src0 + min(max(i0 - 1 + k, 0), in_rows - 1);
                const v4f a = ring[(r & (RL_RING - 1)) * J + q];
                v.x += wt[k] * a.x; v.y += wt[k] * a.y; v.z += wt[k] * a.z; v.w += wt[k] * a.w;
              }
            } else {
              const float l1 = fminf(fmaxf(tt, 0.f), 1.f), l0 = 1.f - l1;
              const int i1 = i0 + (i0 < in_rows - 1 ? 1 : 0);
              const v4f a0 = ring[((src0 + i0) & (RL_RING - 1)) * J + q];
              const v4f a1 = ring[((src0 + i1) & (RL_RING - 1)) * J + q];
              v = v4f{l0 * a0.x + l1 * a1.x, l0 * a0.y + l1 * a1.y, l0 * a0.z + l1 * a1.z, l0 * a0.w + l1 * a1.w};
            }
          }
        } else {
          v = ring[(t & (RL_RING - 1)) * J + q];
        }
        if constexpr (MEAN) {
          s_all += v.x + v.y + v.z + v.w;
          s_msk += ((cm & 1) ? v.x : 0.f) + ((cm & 2) ? v.y : 0.f) + ((cm & 4) ? v.z : 0.f) + ((cm & 8) ? v.w : 0.f);
        }
        // masked cells are fixup4_kernel's: a time-masked row or a fully
        // frequency-masked float4 is not written here
        if (WARP && cm != 15u && !(n_tmask && in_masks(tms, 0, n_tmask, t)))
          *reinterpret_cast<v4f*>(xn + (long long)t * F) = v;
      }
    }
    __syncthreads();  // every read of the ring for this window is done
    RL_STASH(nlo, nhi);
    have = nhi;
    t0 = t1;
    __syncthreads();
  }
  if constexpr (MEAN) {
    const float sa = block_sum(s_all, red);
    const float sm = block_sum(s_msk, red);
    const float nc = block_sum(act && rp == 0 ? (float)__builtin_popcount(cm) : 0.f, red);
    if (threadIdx.x == 0) {
      partial[3 * slab] = sa;
      partial[3 * slab + 1] = sm;
      partial[3 * slab + 2] = nc;
    }
  }
#undef RL_FETCH
#undef RL_STASH
}

// The masked cells after roll4_kernel: time-masked rows -> fill_t, the
// frequency-masked cells of the other rows -> fill_f (0 without the mean
// fill).  One workgroup per (utterance, FX_TR rows): the utterance's masked
// columns are listed in LDS, then only masked cells are touched (a pass over
// every cell checking the masks measured 40 us at config 2).  Every workgroup
// reduces the roll partials in the same fixed order (deterministic, no
// cross-workgroup hand-off).
constexpr int FX_TR = 64, FX_FMAX = 1024;
__global__ void __launch_bounds__(256) fixup4_kernel(float* __restrict__ x, int N, int T, int F,
                                                     const int* __restrict__ fmask, int n_fmask,
                                                     const int* __restrict__ tmask, int n_tmask,
                                                     const float* __restrict__ partial, int nparts, int use_mean,
                                                     long long n_fcells) {
  __shared__ float fl[2];
  __shared__ int fms[2 * RL_MAXM], tms[2 * RL_MAXM];
  __shared__ short cols[FX_FMAX];    // masked columns of partly masked float4s (scalar stores)
  __shared__ short quads[FX_FMAX / 4];  // fully masked float4s (16-B stores)
  __shared__ unsigned char trow[FX_TR];
  __shared__ int ncol, nquad;
  const int ntile = (T + FX_TR - 1) / FX_TR;
  const int n = blockIdx.x / ntile, r0 = (blockIdx.x - n * ntile) * FX_TR;
  if ((int)threadIdx.x < 2 * n_fmask) fms[threadIdx.x] = fmask[2 * n * n_fmask + threadIdx.x];
  if ((int)threadIdx.x < 2 * n_tmask) tms[threadIdx.x] = tmask[2 * n * n_tmask + threadIdx.x];
  __syncthreads();  // the mask tables
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  if (wv == 0 && use_mean) {
    // the roll partials, one wave, fixed order (deterministic; every
    // workgroup computes the same fills)
    // eight triples in flight per lane (a loop of one dependent load round
    // per 64 triples paid ~10 us of L2 latency at config 2's 960 partials)
    float a = 0.f, m = 0.f, nc = 0.f;
    for (int i0 = ln; i0 < nparts; i0 += 64 * 8) {
      float pa[8], pm[8], pn[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = min(i0 + 64 * u, nparts - 1);
        pa[u] = partial[3 * i];
        pm[u] = partial[3 * i + 1];
        pn[u] = partial[3 * i + 2];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (i0 + 64 * u < nparts) {
          a += pa[u];
          m += pm[u];
          nc += pn[u];
        }
    }
    a = wave_sum_v(a);
    m = wave_sum_v(m);
    nc = wave_sum_v(nc);
    if (ln == 0) {
      const double total = (double)N * T * F;
      const double cells = n_fcells >= 0 ? (double)n_fcells : (double)nc * T;
      const float mean1 = (float)(a / total);
      fl[0] = mean1;
      fl[1] = (float)(((double)a - (double)m + (double)mean1 * cells) / total);
    }
  } else if (wv == 1) {
    // this utterance's masked float4s: fully masked ones (one 16-B store per
    // row) and the masked columns of partly masked ones (4-B stores); the
    // running counts stay in wave-uniform registers
    int b4 = 0, b1 = 0;
    const int F4 = F >> 2;
    for (int q0 = 0; q0 < F4; q0 += 64) {
      const int q = q0 + ln;
      const unsigned cm = q < F4 ? col_mask4(fms, 0, n_fmask, 4 * q) : 0u;
      const unsigned long long full = __ballot(cm == 15u);
      if (cm == 15u) quads[b4 + __builtin_popcountll(full & ((1ull << ln) - 1))] = (short)q;
      b4 += __builtin_popcountll(full);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool m = cm != 15u && (cm >> e & 1u);
        const unsigned long long bal = __ballot(m);
        if (m) cols[b1 + __builtin_popcountll(bal & ((1ull << ln) - 1))] = (short)(4 * q + e);
        b1 += __builtin_popcountll(bal);
      }
    }
    if (ln == 0) {
      ncol = b1;
      nquad = b4;
    }
  } else if (wv == 2) {
    for (int i = ln; i < FX_TR; i += 64)
      trow[i] = (unsigned char)(r0 + i < T && n_tmask && in_masks(tms, 0, n_tmask, r0 + i));
  }
  __syncthreads();
  const float fill_f = use_mean ? fl[0] : 0.f, fill_t = use_mean ? fl[1] : 0.f;
  const int F4 = F >> 2, nc = ncol, nq = nquad, nr = min(FX_TR, T - r0);
  float* xt = x + ((long long)n * T + r0) * F;
  // time-masked rows: whole rows
  for (int i = threadIdx.x; i < nr * F4; i += blockDim.x) {
    const int r = i / F4;
    if (trow[r]) *reinterpret_cast<float4*>(xt + (long long)r * F + 4 * (i - r * F4)) = make_float4(fill_t, fill_t, fill_t, fill_t);
  }
  // the frequency-masked cells of the other rows
  for (int i = threadIdx.x; i < nr * nq; i += blockDim.x) {
    const int r = i / nq;
    if (!trow[r])
      *reinterpret_cast<float4*>(xt + (long long)r * F + 4 * quads[i - r * nq]) = make_float4(fill_f, fill_f, fill_f, fill_f);
  }
  for (int i = threadIdx.x; i < nr * nc; i += blockDim.x) {
    const int r = i / nc;
    if (!trow[r]) xt[(long long)r * F + cols[i - r * nc]] = fill_f;
  }
}

// slab width (float4 columns) of roll4_kernel: the widest divisor of F4 up to
// RL_JMAX (the ring is RL_RING x J x 16 B of LDS: 64 KB at J = 4)
__host__ __forceinline__ int roll_slab(int N, int F4) {
  (void)N;
  for (int J = RL_JMAX; J >= 1; --J)
    if (F4 % J == 0) return J;
  return 0;
}

// the two fills from the partial sums, once (fixed order: deterministic);
// 1024 threads, four independent pair loads in flight per thread
__global__ void __launch_bounds__(1024) fills_kernel(const float* __restrict__ partial, int nparts, int N, int T,
                                                     int F, long long n_fcells, const int* __restrict__ fmask,
                                                     int n_fmask, float* __restrict__ fills) {
  __shared__ float red[16];
  __shared__ int mlds[FM_LDS];
  // n_fcells < 0: count the frequency-masked cells here from the device mask
  // table (no host pass over the draws); its loads go out ahead of the
  // partial sums'
  static_assert(FM_LDS == 2 * 1024, "two table entries per thread");
  const int nm = N * n_fmask * 2;
  const bool count = n_fcells < 0 && n_fmask > 0, staged = count && nm <= FM_LDS;
  int e0 = 0, e1 = 0;
  if (staged) {
    if ((int)threadIdx.x < nm) e0 = fmask[threadIdx.x];
    if ((int)threadIdx.x + 1024 < nm) e1 = fmask[threadIdx.x + 1024];
  }
  float a = 0.f, m = 0.f;
  for (int i0 = threadIdx.x; i0 < nparts; i0 += 4 * blockDim.x) {
    float2 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = i0 + k * blockDim.x;
      v[k] = i < nparts ? *reinterpret_cast<const float2*>(partial + 2 * i) : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a += v[k].x;
      m += v[k].y;
    }
  }
  a = block_sum(a, red);
  m = block_sum(m, red);
  if (staged) {
    mlds[threadIdx.x] = e0;
    mlds[threadIdx.x + 1024] = e1;
    __syncthreads();
  }
  if (n_fcells < 0) n_fcells = count ? fmask_cells(fmask, n_fmask, N, F, red, mlds, staged) * T : 0;
  if (threadIdx.x == 0) {
    const double total = (double)N * T * F;
    const float mean1 = (float)(a / total);
    fills[0] = mean1;
    fills[1] = (float)(((double)a - (double)m + (double)mean1 * (double)n_fcells) / total);
  }
}

// x = time-masked ? fill_t : freq-masked ? fill_f : src, one float4 per
// thread and row, UR rows per thread loaded together
__global__ void __launch_bounds__(256) apply4_kernel(const float* src, float* x, int N, int T, int F,
                                                     const int* __restrict__ fmask, int n_fmask,
                                                     const int* __restrict__ tmask, int n_tmask,
                                                     const float* __restrict__ fills) {
  const int F4 = F >> 2, rpp = 256 / F4, RB = UR * rpp;
  const int ntile = (T + RB - 1) / RB;
  const int n = blockIdx.x / ntile;
  const int t0 = (blockIdx.x - n * ntile) * RB;
  const int q = threadIdx.x % F4, tr = threadIdx.x / F4;
  if (tr >= rpp) return;
  const float fill_f = fills ? fills[0] : 0.f, fill_t = fills ? fills[1] : 0.f;
  const unsigned cm = col_mask4(fmask, n, n_fmask, 4 * q);
  float4 v[UR];
#pragma unroll
  for (int u = 0; u < UR; ++u) {
    const int t = min(t0 + tr + u * rpp, T - 1);
    v[u] = *reinterpret_cast<const float4*>(src + ((long long)n * T + t) * F + 4 * q);
  }
#pragma unroll
  for (int u = 0; u < UR; ++u) {
    const int t = t0 + tr + u * rpp;
    if (t >= T) continue;
    float4 o = v[u];
    if (n_tmask && in_masks(tmask, n, n_tmask, t)) {
      o = make_float4(fill_t, fill_t, fill_t, fill_t);
    } else if (cm) {
      if (cm & 1) o.x = fill_f;
      if (cm & 2) o.y = fill_f;
      if (cm & 4) o.z = fill_f;
      if (cm & 8) o.w = fill_f;
    }
    *reinterpret_cast<float4*>(x + ((long long)n * T + t) * F + 4 * q) = o;
  }
}

}  // namespace

// Full SpecAugment application on x (N, T, F) fp32, in place.
//   warp: c, w (warp skipped when c < 0), warp_mode 0 bicubic / 1 bilinear;
//   tmp: (N, T, F) scratch, required when warping;
//   fmask (N, n_fmask, 2) / tmask (N, n_tmask, 2) int32 [len, pos] device arrays (or n_* = 0);
//   use_mean: fill with the running means (replace_with_zero=False), else 0;
//   partial: scratch of 2 * N * ceil(T/4) + 2 floats (when use_mean);
//   n_fcells: number of frequency-masked cells (the second mean's count); < 0: counted on the device
//             from fmask.
namespace {
bool roll_route(int N, int F, int c, int w, int n_fmask, int n_tmask, bool x_aligned) {
  return F % 4 == 0 && F <= FX_FMAX && x_aligned && (c < 0 || abs(c - w) + 3 <= RL_HMAX) && roll_slab(N, F >> 2) > 0 &&
         n_fmask <= RL_MAXM && n_tmask <= RL_MAXM;
}
}  // namespace

// 1 when sbk_specaugment needs its `tmp` scratch for these arguments (the
// warp of the copy path), 0 when it runs in place without one
SBK_API int sbk_specaugment_needs_scratch(int N, int T, int F, int c, int w, int n_fmask, int n_tmask, int x_aligned) {
  (void)T;
  return c >= 0 && !roll_route(N, F, c, w, n_fmask, n_tmask, x_aligned != 0);
}

SBK_API int sbk_specaugment(float* x, int N, int T, int F, int c, int w, int warp_mode, float* tmp, const int* fmask,
                            int n_fmask,
                            const int* tmask, int n_tmask, int use_mean, float* partial, long long n_fcells,
                            void* stream) {
  if (N <= 0 || T <= 0 || F <= 0 || warp_mode < 0 || warp_mode > 1) return SBK_ERR_ARG;
  hipStream_t s4 = (hipStream_t)stream;
  if (roll_route(N, F, c, w, n_fmask, n_tmask, (reinterpret_cast<uintptr_t>(x) & 15) == 0)) {
    // in place: roll4_kernel (x read once, unmasked cells written once) +
    // fixup4_kernel (the masked cells); `partial`: 3 * N * (F/4) / J floats
    const int J = roll_slab(N, F >> 2), nblk = N * ((F >> 2) / J);
    if (c >= 0 && (c <= 0 || c >= T || w <= 0 || w >= T)) return SBK_ERR_ARG;
    if (use_mean && !partial) return SBK_ERR_ARG;
    const size_t lds = (size_t)RL_RING * J * 16;
    float* pp = use_mean ? partial : nullptr;
#define SBK_ROLL(CU, WA, ME)                                                                                        \
  do {                                                                                                              \
    /* > 64 KB of LDS with the static arrays: opted in per device, for the */                                      \
    /* widest slab any call can take (RL_JMAX)                             */                                      \
    if (hipError_t e = sbk::lds_optin(reinterpret_cast<const void*>(&roll4_kernel<CU, WA, ME>),                    \
                                      (size_t)RL_RING * RL_JMAX * 16))                                              \
      return (int)e;                                                                                                \
    hipLaunchKernelGGL((roll4_kernel<CU, WA, ME>), dim3(nblk), dim3(256), lds, s4, x, N, T, F, J, c, w, fmask,      \
                       n_fmask, tmask, n_tmask, pp);                                                                \
  } while (0)
    if (c >= 0) {
      if (warp_mode == 0) {
        if (use_mean) SBK_ROLL(true, true, true); else SBK_ROLL(true, true, false);
      } else {
        if (use_mean) SBK_ROLL(false, true, true); else SBK_ROLL(false, true, false);
      }
      SBK_CHECK_LAUNCH();
    } else if (use_mean) {
      SBK_ROLL(true, false, true);
      SBK_CHECK_LAUNCH();
    }
#undef SBK_ROLL
    if (n_fmask == 0 && n_tmask == 0) return 0;
    const int fblk = N * ((T + FX_TR - 1) / FX_TR);
    hipLaunchKernelGGL(fixup4_kernel, dim3(fblk), dim3(256), 0, s4, x, N, T, F, fmask, n_fmask, tmask, n_tmask,
                       pp, nblk, use_mean, n_fcells);
    SBK_CHECK_LAUNCH();
    return 0;
  }
  if (F % 4 == 0 && F <= 1024 &&
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(tmp) | reinterpret_cast<uintptr_t>(partial)) & 15) == 0) {
    // 4-wide path; `partial` must hold 2 * N * ceil(T/4) + 2 floats (the fills at its end)
    const int rb = rows_per_block4(F);  // >= UR = 4
    const int nblk4 = N * ((T + rb - 1) / rb);
    float* fills = use_mean ? partial + 2 * N * ((T + 3) / 4) : nullptr;
    const float* src = x;
    if (c >= 0) {
      if (!tmp || c <= 0 || c >= T || w <= 0 || w >= T) return SBK_ERR_ARG;
      if (warp_mode == 0)
        hipLaunchKernelGGL((warp4_kernel<true, true>), dim3(nblk4), dim3(256), 0, s4, x, tmp, N, T, F, c, w, fmask,
                           n_fmask, use_mean ? partial : nullptr);
      else
        hipLaunchKernelGGL((warp4_kernel<false, true>), dim3(nblk4), dim3(256), 0, s4, x, tmp, N, T, F, c, w, fmask,
                           n_fmask, use_mean ? partial : nullptr);
      SBK_CHECK_LAUNCH();
      src = tmp;
    } else if (use_mean) {
      hipLaunchKernelGGL((warp4_kernel<true, false>), dim3(nblk4), dim3(256), 0, s4, x, nullptr, N, T, F, c, w, fmask,
                         n_fmask, partial);
      SBK_CHECK_LAUNCH();
    }
    if (c < 0 && n_fmask == 0 && n_tmask == 0) return 0;
    if (use_mean) {
      hipLaunchKernelGGL(fills_kernel, dim3(1), dim3(1024), 0, s4, partial, nblk4, N, T, F, n_fcells, fmask, n_fmask,
                         fills);
      SBK_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(apply4_kernel, dim3(nblk4), dim3(256), 0, s4, src, x, N, T, F, fmask, n_fmask, tmask, n_tmask,
                       fills);
    SBK_CHECK_LAUNCH();
    return 0;
  }
  const int TT = 16;
  const int nblk = N * ((T + TT - 1) / TT);
  hipStream_t s = (hipStream_t)stream;
  const float* src = x;
  if (c >= 0) {
    if (!tmp || c <= 0 || c >= T || w <= 0 || w >= T) return SBK_ERR_ARG;
    if (warp_mode == 0)
      hipLaunchKernelGGL(warp_kernel<true>, dim3(nblk), dim3(256), 0, s, x, tmp, N, T, F, c, w, TT, fmask, n_fmask,
                         use_mean ? partial : nullptr);
    else
      hipLaunchKernelGGL(warp_kernel<false>, dim3(nblk), dim3(256), 0, s, x, tmp, N, T, F, c, w, TT, fmask, n_fmask,
                         use_mean ? partial : nullptr);
    SBK_CHECK_LAUNCH();
    src = tmp;
  } else if (use_mean) {
    hipLaunchKernelGGL(sum_kernel, dim3(nblk), dim3(256), 0, s, x, N, T, F, TT, fmask, n_fmask, partial);
    SBK_CHECK_LAUNCH();
  }
  if (c < 0 && n_fmask == 0 && n_tmask == 0) return 0;
  hipLaunchKernelGGL(apply_kernel, dim3(nblk), dim3(256), 0, s, src, x, N, T, F, TT, fmask, n_fmask, tmask, n_tmask,
                     partial, nblk, n_fcells, use_mean);
  SBK_CHECK_LAUNCH();
  return 0;
}
