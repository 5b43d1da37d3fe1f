// InputNormalization (speechbrain/processing/features.py:940-1231) on HIP.
//
// The reference loops over the utterances of a batch on the host
// (:1014-1066): per utterance, the mean and unbiased std over its first
// round(len * T) frames (:1017-1024, :1120-1145), then sentence / batch /
// global / speaker normalisation.  Here:
//   sbk_inorm_partials  grid (B, S): each workgroup folds one of S frame
//                       slices of one utterance into per-feature Welford
//                       partials (count, mean, M2) in fp64, thread (f, r)
//                       striding the frames of the slice (coalesced rows);
//   sbk_inorm_stats     one thread per (b, f) merges the S partials (Chan),
//                       std = sqrt(M2 / (n - 1)) clamped to >= eps like the
//                       reference (NaN for n <= 1, as torch.std);
//                       optionally the batch means of the per-utterance
//                       mean / std and the global moving average
//                       (mode 1: set, 2: (1 - w) g + w cur) in place;
//   sbk_inorm_apply     y = (x - m) / s over (B, T, F), m / s per utterance
//                       or shared, in place allowed.
// Frames are counted with rintf(len * T) (torch.round: half to even), clamped
// to [0, T].  Every pass is HBM-bound: 2 reads + 1 write of the features.
#include "sbk_common.h"

#include <algorithm>

using namespace sbk;

namespace {

constexpr int IN_NT = 256;

struct Welford {
  double n, mean, m2;
};

__device__ __forceinline__ Welford wmerge(Welford a, Welford b) {
  if (b.n == 0.0) return a;
  if (a.n == 0.0) return b;
  const double n = a.n + b.n, d = b.mean - a.mean;
  return Welford{n, a.mean + d * (b.n / n), a.m2 + b.m2 + d * d * (a.n * b.n / n)};
}

__device__ __forceinline__ int frames_of(const float* len, int b, int T) {
  const int n = (int)rintf(len[b] * (float)T);
  return n < 0 ? 0 : (n > T ? T : n);
}

// part: (B, S, F) Welford triples as 3 doubles.
__global__ void __launch_bounds__(IN_NT) inorm_partials_kernel(const float* __restrict__ x, const float* __restrict__ len,
                                                              int T, int F, int S, double* __restrict__ part) {
  extern __shared__ double sw[];  // R x F x 3
  const int b = blockIdx.x, s = blockIdx.y;
  const int R = IN_NT / F;  // frame lanes per feature (F <= 256)
  const int f = threadIdx.x % F, r = threadIdx.x / F;
  const int n = frames_of(len, b, T);
  const int per = (n + S - 1) / S;
  const int t0 = s * per, t1 = min(n, t0 + per);
  Welford w{0.0, 0.0, 0.0};
  if (r < R) {
    const float* xb = x + (long long)b * T * F + f;
    for (int t = t0 + r; t < t1; t += R) {
      const double v = xb[(long long)t * F];
      w.n += 1.0;
      const double d = v - w.mean;
      w.mean += d / w.n;
      w.m2 += d * (v - w.mean);
    }
    double* o = sw + ((long long)r * F + f) * 3;
    o[0] = w.n;
    o[1] = w.mean;
    o[2] = w.m2;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < F; i += blockDim.x) {
    Welford acc{0.0, 0.0, 0.0};
    for (int rr = 0; rr < R; ++rr) {
      const double* o = sw + ((long long)rr * F + i) * 3;
      acc = wmerge(acc, Welford{o[0], o[1], o[2]});
    }
    double* p = part + (((long long)b * S + s) * F + i) * 3;
    p[0] = acc.n;
    p[1] = acc.mean;
    p[2] = acc.m2;
  }
}

// Per-utterance statistics (B, F) and, when cur_mean is given, their batch
// means; upd: 0 none, 1 glob = cur, 2 glob = (1 - w) glob + w cur.
__global__ void inorm_stats_kernel(const double* __restrict__ part, int B, int S, int F, int mean_norm, int std_norm,
                                   float eps, float* __restrict__ mean, float* __restrict__ std,
                                   float* __restrict__ cur_mean, float* __restrict__ cur_std, int upd, float keep,
                                   float wgt, float* __restrict__ glob_mean, float* __restrict__ glob_std) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  float sm = 0.f, ss = 0.f;
  for (int b = 0; b < B; ++b) {
    Welford acc{0.0, 0.0, 0.0};
    for (int s = 0; s < S; ++s) {
      const double* p = part + (((long long)b * S + s) * F + f) * 3;
      acc = wmerge(acc, Welford{p[0], p[1], p[2]});
    }
    // torch.mean over 0 frames is NaN; torch.std (unbiased) over <= 1 frame is NaN
    const float m = mean_norm ? (acc.n > 0.0 ? (float)acc.mean : __int_as_float(0x7fc00000)) : 0.f;
    float sd = 1.f;
    if (std_norm) sd = acc.n > 1.0 ? (float)sqrt(acc.m2 / (acc.n - 1.0)) : __int_as_float(0x7fc00000);
    sd = (sd != sd) ? sd : fmaxf(sd, eps);  // torch.max propagates NaN
    if (mean) mean[(long long)b * F + f] = m;
    if (std) std[(long long)b * F + f] = sd;
    sm += m;
    ss += sd;
  }
  if (cur_mean) {
    const float cm = sm / (float)B, cs = ss / (float)B;
    cur_mean[f] = cm;
    cur_std[f] = cs;
    if (upd == 1) {
      glob_mean[f] = cm;
      glob_std[f] = cs;
    } else if (upd == 2) {
      // keep = fp32(1 - w) as the reference's scalar; two products and a sum, no FMA contraction
      glob_mean[f] = __fadd_rn(__fmul_rn(keep, glob_mean[f]), __fmul_rn(wgt, cm));
      glob_std[f] = __fadd_rn(__fmul_rn(keep, glob_std[f]), __fmul_rn(wgt, cs));
    }
  }
}

__global__ void inorm_apply_kernel(const float* __restrict__ x, int B, int T, int F, const float* __restrict__ m,
                                   const float* __restrict__ s, int per_utt, float* __restrict__ y) {
  const long long n = (long long)B * T * F;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int f = (int)(i % F);
    const long long k = per_utt ? (i / ((long long)T * F)) * F + f : f;
    y[i] = (x[i] - m[k]) / s[k];
  }
}

}  // namespace

SBK_API int sbk_inorm_slices(int T) { return T >= 4096 ? 16 : (T >= 512 ? 8 : (T >= 64 ? 2 : 1)); }

SBK_API int sbk_inorm_partials(const float* x, const float* len, int B, int T, int F, double* part, void* stream) {
  if (B <= 0 || T <= 0 || F <= 0 || F > IN_NT) return SBK_ERR_ARG;
  const int S = sbk_inorm_slices(T);
  const int R = IN_NT / F;
  inorm_partials_kernel<<<dim3(B, S), IN_NT, (size_t)R * F * 3 * sizeof(double), (hipStream_t)stream>>>(x, len, T, F,
                                                                                                       S, part);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_inorm_stats(const double* part, int B, int T, int F, int mean_norm, int std_norm, float eps,
                            float* mean, float* std, float* cur_mean, float* cur_std, int upd, float keep,
                            float wgt, float* glob_mean, float* glob_std, void* stream) {
  if (B <= 0 || T <= 0 || F <= 0 || F > IN_NT || (upd && (!cur_mean || !glob_mean || !glob_std))) return SBK_ERR_ARG;
  if (cur_mean && !cur_std) return SBK_ERR_ARG;
  inorm_stats_kernel<<<(F + 127) / 128, 128, 0, (hipStream_t)stream>>>(part, B, sbk_inorm_slices(T), F, mean_norm,
                                                                       std_norm, eps, mean, std, cur_mean, cur_std,
                                                                       upd, keep, wgt, glob_mean, glob_std);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_inorm_apply(const float* x, int B, int T, int F, const float* mean, const float* std, int per_utt,
                            float* y, void* stream) {
  if (B <= 0 || T <= 0 || F <= 0 || !mean || !std) return SBK_ERR_ARG;
  const long long n = (long long)B * T * F;
  const int grid = (int)std::min<long long>((n + 255) / 256, 8192);
  inorm_apply_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(x, B, T, F, mean, std, per_utt, y);
  SBK_CHECK_LAUNCH();
  return 0;
}
