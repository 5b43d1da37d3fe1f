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
SBK_API int sbk_specaugment(float* x, int N, int T, int F, int c, int w, int warp_mode, float* tmp, const int* fmask,
                            int n_fmask,
                            const int* tmask, int n_tmask, int use_mean, float* partial, long long n_fcells,
                            void* stream) {
  if (N <= 0 || T <= 0 || F <= 0 || warp_mode < 0 || warp_mode > 1) return SBK_ERR_ARG;
  hipStream_t s4 = (hipStream_t)stream;
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
