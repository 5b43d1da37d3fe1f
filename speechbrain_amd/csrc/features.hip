// Feature front-end kernels: STFT / power spectrum / Fbank (fused), standalone
// Filterbank, top_db clamp, spectral magnitude, DCT, Deltas, ContextWindow.
//
// Reference semantics (Sinica-SLAM/speechbrain 0.5.13):
//   STFT                 speechbrain/processing/features.py:101-188 (torch.stft)
//   spectral_magnitude   features.py:327-356
//   Filterbank           features.py:415-712 (matmul + _amplitude_to_DB)
//   DCT                  features.py:740-786
//   Deltas               features.py:806-852
//   ContextWindow        features.py:879-937
//   Fbank / MFCC         speechbrain/lobes/features.py:130-147, :260-281
//
// Design (MI355X): the STFT is a real FFT of n_fft points computed as an
// n_fft/2-point complex mixed-radix Stockham FFT in LDS (radices 8/5/4/3/2),
// FPB frames per 256-thread workgroup.  The workgroup stages the union of its
// FPB overlapping frames once (coalesced), so the waveform is read from HBM
// ~once.  The Fbank epilogue (|X|^2 -> sparse mel -> dB -> per-utterance max)
// runs out of LDS, so the only HBM traffic is wav in + mel out: the kernel is
// bandwidth/latency bound, not FLOP bound (~11 kFLOP per frame).
#include "sbk_common.h"

using namespace sbk;

namespace {

struct FftPlan {
  int nc;          // complex FFT size (n_fft / 2)
  int nstages;
  int radix[12];
};

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
// multiply by -i
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }
// multiply by +i
__device__ __forceinline__ float2 mul_pi(float2 a) { return make_float2(-a.y, a.x); }

template <int R>
__device__ __forceinline__ void dft_small(float2* v);

template <>
__device__ __forceinline__ void dft_small<2>(float2* v) {
  float2 a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}

template <>
__device__ __forceinline__ void dft_small<3>(float2* v) {
  const float s = 0.86602540378443864676f;  // sin(2pi/3)
  float2 t = cadd(v[1], v[2]);
  float2 d = csub(v[1], v[2]);
  float2 y0 = cadd(v[0], t);
  float2 m = make_float2(v[0].x - 0.5f * t.x, v[0].y - 0.5f * t.y);
  float2 sd = make_float2(s * d.x, s * d.y);
  v[0] = y0;
  v[1] = cadd(m, mul_mi(sd));
  v[2] = cadd(m, mul_pi(sd));
}

template <>
__device__ __forceinline__ void dft_small<4>(float2* v) {
  float2 a = cadd(v[0], v[2]), b = csub(v[0], v[2]);
  float2 c = cadd(v[1], v[3]), d = mul_mi(csub(v[1], v[3]));
  v[0] = cadd(a, c);
  v[2] = csub(a, c);
  v[1] = cadd(b, d);
  v[3] = csub(b, d);
}

template <>
__device__ __forceinline__ void dft_small<5>(float2* v) {
  const float c1 = 0.30901699437494742410f;   // cos(2pi/5)
  const float c2 = -0.80901699437494742410f;  // cos(4pi/5)
  const float s1 = 0.95105651629515357212f;   // sin(2pi/5)
  const float s2 = 0.58778525229247312917f;   // sin(4pi/5)
  float2 t1 = cadd(v[1], v[4]), t2 = cadd(v[2], v[3]);
  float2 t3 = csub(v[1], v[4]), t4 = csub(v[2], v[3]);
  float2 y0 = cadd(v[0], cadd(t1, t2));
  float2 a = make_float2(v[0].x + c1 * t1.x + c2 * t2.x, v[0].y + c1 * t1.y + c2 * t2.y);
  float2 b = make_float2(v[0].x + c2 * t1.x + c1 * t2.x, v[0].y + c2 * t1.y + c1 * t2.y);
  float2 p = make_float2(s1 * t3.x + s2 * t4.x, s1 * t3.y + s2 * t4.y);
  float2 q = make_float2(s2 * t3.x - s1 * t4.x, s2 * t3.y - s1 * t4.y);
  v[0] = y0;
  v[1] = cadd(a, mul_mi(p));
  v[4] = cadd(a, mul_pi(p));
  v[2] = cadd(b, mul_mi(q));
  v[3] = cadd(b, mul_pi(q));
}

template <>
__device__ __forceinline__ void dft_small<8>(float2* v) {
  const float r = 0.70710678118654752440f;
  // DIF first stage: a_r = v_r + v_{r+4}; b_r = (v_r - v_{r+4}) * W8^r
  float2 a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = cadd(v[i], v[i + 4]);
    b[i] = csub(v[i], v[i + 4]);
  }
  b[1] = make_float2(r * (b[1].x + b[1].y), r * (b[1].y - b[1].x));     // * (r, -r)
  b[2] = mul_mi(b[2]);                                                  // * -i
  b[3] = make_float2(r * (-b[3].x + b[3].y), r * (-b[3].y - b[3].x));   // * (-r, -r)
  dft_small<4>(a);
  dft_small<4>(b);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = a[i];
    v[2 * i + 1] = b[i];
  }
}

// One Stockham autosort stage of radix R over FPB frames held in LDS.
template <int R>
__device__ __forceinline__ void stockham_stage(const float2* __restrict__ src, float2* __restrict__ dst,
                                               int nc, int Ns, const float2* __restrict__ tw, int nframes) {
  const int nb = nc / R;
  const int step = nc / (Ns * R);
  for (int task = threadIdx.x; task < nframes * nb; task += blockDim.x) {
    const int f = task / nb;
    const int j = task - f * nb;
    const float2* s = src + f * nc;
    float2* d = dst + f * nc;
    const int k = j % Ns;
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = s[j + r * nb];
#pragma unroll
    for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw[r * k * step]);
    dft_small<R>(v);
    const int idxD = (j / Ns) * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) d[idxD + r * Ns] = v[r];
  }
}

// Runs the whole complex FFT; returns the buffer holding the result.
__device__ float2* run_fft(float2* bufA, float2* bufB, const FftPlan& plan, const float2* tw, int nframes) {
  float2* src = bufA;
  float2* dst = bufB;
  int Ns = 1;
  for (int s = 0; s < plan.nstages; ++s) {
    __syncthreads();
    switch (plan.radix[s]) {
      case 8: stockham_stage<8>(src, dst, plan.nc, Ns, tw, nframes); break;
      case 5: stockham_stage<5>(src, dst, plan.nc, Ns, tw, nframes); break;
      case 4: stockham_stage<4>(src, dst, plan.nc, Ns, tw, nframes); break;
      case 3: stockham_stage<3>(src, dst, plan.nc, Ns, tw, nframes); break;
      default: stockham_stage<2>(src, dst, plan.nc, Ns, tw, nframes); break;
    }
    Ns *= plan.radix[s];
    float2* t = src;
    src = dst;
    dst = t;
  }
  __syncthreads();
  return src;
}

// Position mapping for torch.stft(center=True) padding modes.
__device__ __forceinline__ int map_pos(int p, int S, int mode, bool* valid) {
  *valid = true;
  if (p >= 0 && p < S) return p;
  switch (mode) {
    case 0: *valid = false; return 0;  // constant (zeros)
    case 1: {                          // reflect (no edge repeat)
      if (S == 1) return 0;
      int period = 2 * (S - 1);
      int q = p % period;
      if (q < 0) q += period;
      return q < S ? q : period - q;
    }
    case 2: return p < 0 ? 0 : S - 1;  // replicate
    default: {                         // circular
      int q = p % S;
      return q < 0 ? q + S : q;
    }
  }
}

struct SpecArgs {
  const float* wav;  // (Bo, S, C) contiguous; folded row b' = bo*C + c
  int S, C, Bfold;   // Bfold = Bo*C
  int n_fft, hop, center, pad_mode, T;
  const float* window;  // n_fft floats (win centred, zero padded)
  const float2* tw;     // W_nc^m, m in [0, nc)
  const float2* tw2;    // W_nfft^k, k in [0, nc]
  int fpb;              // frames per block
  // spectral_magnitude
  float power, eps;
  int log_mag;
  // STFT output strides (elements): bo, c, t, k, ri
  long long os_b, os_c, os_t, os_k, os_ri;
  int onesided;
  float norm_scale;
  // mel / dB (FBANK mode)
  const int* mel_start;   // (M,)
  const int* mel_len;     // (M,)
  const int* mel_off;     // (M,) offset into mel_w
  const float* mel_w;
  int M, log_mel, n_melw;
  float multiplier, db_offset, amin, amin_db;
  float* out;
  int* maxkey;  // (Bfold,) per-sequence max dB key
};

enum { MODE_STFT = 0, MODE_POWER = 1, MODE_FBANK = 2 };

template <int MODE>
__global__ void __launch_bounds__(256) spec_kernel(SpecArgs a, FftPlan plan) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int nc = plan.nc;
  const int nblk_t = (a.T + a.fpb - 1) / a.fpb;
  const int bf = blockIdx.x / nblk_t;
  const int t0 = (blockIdx.x - bf * nblk_t) * a.fpb;
  const int nf = min(a.fpb, a.T - t0);
  const int bo = bf / a.C, ch = bf - bo * a.C;
  const float* wrow = a.wav + (long long)bo * a.S * a.C + ch;

  float2* bufA = reinterpret_cast<float2*>(smem);
  float2* bufB = bufA + a.fpb * nc;
  float2* tw = bufB + a.fpb * nc;           // W_nc^m, staged once per block
  float2* tw2 = tw + nc;                    // W_nfft^k, k <= nc
  int* mstart = reinterpret_cast<int*>(tw2 + nc + 1);
  int* mlen = mstart + a.M;
  int* moff = mlen + a.M;
  float* mw = reinterpret_cast<float*>(moff + a.M);
  float* win = mw + (MODE == MODE_FBANK ? a.n_melw : 0);
  float* smp = win + a.n_fft;
  for (int i = threadIdx.x; i < a.n_fft; i += blockDim.x) win[i] = a.window[i];
  for (int i = threadIdx.x; i < nc; i += blockDim.x) tw[i] = a.tw[i];
  for (int i = threadIdx.x; i <= nc; i += blockDim.x) tw2[i] = a.tw2[i];
  if (MODE == MODE_FBANK) {
    for (int i = threadIdx.x; i < a.M; i += blockDim.x) {
      mstart[i] = a.mel_start[i];
      mlen[i] = a.mel_len[i];
      moff[i] = a.mel_off[i];
    }
    for (int i = threadIdx.x; i < a.n_melw; i += blockDim.x) mw[i] = a.mel_w[i];
  }

  // 1) stage the samples spanned by this block's frames
  const int pad = a.center ? a.n_fft / 2 : 0;
  const int base = t0 * a.hop - pad;
  const int span = (nf - 1) * a.hop + a.n_fft;
  for (int q = threadIdx.x; q < span; q += blockDim.x) {
    bool ok;
    int p = map_pos(base + q, a.S, a.pad_mode, &ok);
    smp[q] = ok ? wrow[(long long)p * a.C] : 0.f;
  }
  __syncthreads();
  // 2) window + pack real frame into nc complex values
  for (int i = threadIdx.x; i < nf * nc; i += blockDim.x) {
    const int f = i / nc, m = i - f * nc;
    const float* fr = smp + f * a.hop;
    bufA[f * nc + m] = make_float2(fr[2 * m] * win[2 * m], fr[2 * m + 1] * win[2 * m + 1]);
  }
  // 3) complex FFT of size nc
  float2* Z = run_fft(bufA, bufB, plan, tw, nf);
  float2* other = (Z == bufA) ? bufB : bufA;

  // 4) split into the real-input spectrum X[k], k = 0..nc
  const int nbins = nc + 1;
  if (MODE == MODE_STFT) {
    const int nout = a.onesided ? nbins : a.n_fft;
    for (int i = threadIdx.x; i < nf * nout; i += blockDim.x) {
      const int f = i / nout, kk = i - f * nout;
      const bool mirror = kk > nc;
      const int k = mirror ? a.n_fft - kk : kk;
      const float2 zk = Z[f * nc + (k % nc)];
      const float2 zr = Z[f * nc + ((nc - k) % nc)];
      const float2 zc = make_float2(zr.x, -zr.y);
      const float2 E = make_float2(0.5f * (zk.x + zc.x), 0.5f * (zk.y + zc.y));
      const float2 O = mul_mi(make_float2(0.5f * (zk.x - zc.x), 0.5f * (zk.y - zc.y)));
      float2 X = cadd(E, cmul(tw2[k], O));
      if (mirror) X.y = -X.y;
      float* o = a.out + bo * a.os_b + ch * a.os_c + (long long)(t0 + f) * a.os_t + kk * a.os_k;
      o[0] = X.x * a.norm_scale;
      o[a.os_ri] = X.y * a.norm_scale;
    }
    return;
  }
  float* P = reinterpret_cast<float*>(other);  // (nf, nbins) power
  for (int i = threadIdx.x; i < nf * nbins; i += blockDim.x) {
    const int f = i / nbins, k = i - f * nbins;
    const float2 zk = Z[f * nc + (k % nc)];
    const float2 zr = Z[f * nc + ((nc - k) % nc)];
    const float2 zc = make_float2(zr.x, -zr.y);
    const float2 E = make_float2(0.5f * (zk.x + zc.x), 0.5f * (zk.y + zc.y));
    const float2 O = mul_mi(make_float2(0.5f * (zk.x - zc.x), 0.5f * (zk.y - zc.y)));
    float2 X = cadd(E, cmul(tw2[k], O));
    X.x *= a.norm_scale;
    X.y *= a.norm_scale;
    float s = X.x * X.x + X.y * X.y;
    if (a.power != 1.0f) {
      if (a.power < 1.0f) s += a.eps;
      s = powf(s, a.power);
    }
    if (MODE == MODE_POWER) {
      if (a.log_mag) s = logf(s + a.eps);
      a.out[bo * a.os_b + ch * a.os_c + (long long)(t0 + f) * a.os_t + k * a.os_k] = s;
    } else {
      P[i] = s;
    }
  }
  if (MODE == MODE_POWER) return;
  __syncthreads();
  // 5) sparse mel projection + dB + running max
  float lmax = -INFINITY;
  float* orow = a.out + ((long long)bf * a.T + t0) * a.M;
  for (int i = threadIdx.x; i < nf * a.M; i += blockDim.x) {
    const int f = i / a.M, j = i - f * a.M;
    const float* pf = P + f * nbins + mstart[j];
    const float* w = mw + moff[j];
    const int L = mlen[j];
    float acc = 0.f;
    for (int q = 0; q < L; ++q) acc = fmaf(pf[q], w[q], acc);
    if (a.log_mel) {
      // clamp(x, amin) -> the host-rounded dB of amin exactly (-100 for 1e-10)
      acc = acc <= a.amin ? a.amin_db : a.multiplier * log10f(acc) - a.db_offset;
      lmax = fmaxf(lmax, acc);
    }
    orow[i] = acc;
  }
  if (a.log_mel) {
    lmax = wave_max(lmax);
    if ((threadIdx.x & 63) == 0 && lmax > -INFINITY) atomicMax(a.maxkey + bf, float_to_key(lmax));
  }
}

// Standalone Filterbank over a given spectrogram (N, T, F) -> (N, T, M).
struct FbArgs {
  const float* spec;
  int N, T, F;
  const int* mel_start;
  const int* mel_len;
  const int* mel_off;
  const float* mel_w;
  const float* dense;  // optional dense (F, M) matrix (learnable filters); null -> sparse
  int M, log_mel, rows_per_block;
  float multiplier, db_offset, amin, amin_db;
  float* out;
  int* maxkey;
};

__global__ void __launch_bounds__(256) filterbank_kernel(FbArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* rowbuf = reinterpret_cast<float*>(smem);
  const long long nrows = (long long)a.N * a.T;
  const long long r0 = (long long)blockIdx.x * a.rows_per_block;
  const int nr = (int)min((long long)a.rows_per_block, nrows - r0);
  for (int i = threadIdx.x; i < nr * a.F; i += blockDim.x) rowbuf[i] = a.spec[r0 * a.F + i];
  __syncthreads();
  float lmax = -INFINITY;
  int cur_n = -1;
  for (int i = threadIdx.x; i < nr * a.M; i += blockDim.x) {
    const int rr = i / a.M, j = i - rr * a.M;
    const float* pf = rowbuf + rr * a.F;
    float acc = 0.f;
    if (a.dense) {
      for (int q = 0; q < a.F; ++q) acc = fmaf(pf[q], a.dense[q * a.M + j], acc);
    } else {
      const float* w = a.mel_w + a.mel_off[j];
      const int L = a.mel_len[j];
      pf += a.mel_start[j];
      for (int q = 0; q < L; ++q) acc = fmaf(pf[q], w[q], acc);
    }
    if (a.log_mel) {
      acc = acc <= a.amin ? a.amin_db : a.multiplier * log10f(acc) - a.db_offset;
      const int n = (int)((r0 + rr) / a.T);
      // rows of one block may straddle two sequences: flush per sequence
      if (n != cur_n) {
        if (cur_n >= 0 && lmax > -INFINITY) atomicMax(a.maxkey + cur_n, float_to_key(lmax));
        cur_n = n;
        lmax = -INFINITY;
      }
      lmax = fmaxf(lmax, acc);
    }
    a.out[(r0 + rr) * a.M + j] = acc;
  }
  if (a.log_mel && cur_n >= 0 && lmax > -INFINITY) atomicMax(a.maxkey + cur_n, float_to_key(lmax));
}

// x[n, :] = max(x[n, :], max_n - top_db), per sequence n of `per_seq` floats.
__global__ void topdb_clamp_kernel(float* __restrict__ x, const int* __restrict__ maxkey,
                                   long long per_seq, int nseq, float top_db) {
  const long long total = per_seq * nseq;
  for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < total;
       i += (long long)gridDim.x * blockDim.x * 4) {
    if (i + 3 < total && (per_seq % 4) == 0) {
      const int n = (int)(i / per_seq);
      const float fl = key_to_float(maxkey[n]) - top_db;
      float4 v = *reinterpret_cast<float4*>(x + i);
      v.x = fmaxf(v.x, fl);
      v.y = fmaxf(v.y, fl);
      v.z = fmaxf(v.z, fl);
      v.w = fmaxf(v.w, fl);
      *reinterpret_cast<float4*>(x + i) = v;
    } else {
      for (long long e = i; e < min(i + 4, total); ++e) {
        const int n = (int)(e / per_seq);
        x[e] = fmaxf(x[e], key_to_float(maxkey[n]) - top_db);
      }
    }
  }
}

// spectral_magnitude on an arbitrary tensor: reduce the last axis (size L).
__global__ void magnitude_kernel(const float* __restrict__ x, float* __restrict__ y, long long n, int L,
                                 float power, float eps, int log_mag) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < L; ++q) {
      const float v = x[i * L + q];
      s = fmaf(v, v, s);
    }
    if (power < 1.0f) s += eps;
    if (power != 1.0f) s = powf(s, power);
    if (log_mag) s = logf(s + eps);
    y[i] = s;
  }
}

// DCT: y[r, j] = sum_i x[r, i] * D[i, j]   (D is (n_in, n_out)).
__global__ void __launch_bounds__(256) dct_kernel(const float* __restrict__ x, const float* __restrict__ D,
                                                  float* __restrict__ y, long long rows, int n_in, int n_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* Ds = reinterpret_cast<float*>(smem);
  for (int i = threadIdx.x; i < n_in * n_out; i += blockDim.x) Ds[i] = D[i];
  __syncthreads();
  const long long total = rows * n_out;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const long long r = e / n_out;
    const int j = (int)(e - r * n_out);
    const float* xr = x + r * n_in;
    float acc = 0.f;
    for (int i = 0; i < n_in; ++i) acc = fmaf(xr[i], Ds[i * n_out + j], acc);
    y[e] = acc;
  }
}

// Deltas along time of (N, T, F): one output, or fused [x | d1 | d2] concat.
//   d[t] = sum_{k=1..n} k * (x[clamp(t+k)] - x[clamp(t-k)]) / denom
template <bool CONCAT>
__global__ void __launch_bounds__(256) deltas_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                     int N, int T, int F, int n, float denom, int ttile) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // tile of rows [t0 - halo, t0 + ttile + halo) x F
  const int halo = CONCAT ? 2 * n : n;
  const int ntile = (T + ttile - 1) / ttile;
  const int b = blockIdx.x / ntile;
  const int t0 = (blockIdx.x - b * ntile) * ttile;
  const int nt = min(ttile, T - t0);
  const int rows = nt + 2 * halo;
  float* xs = reinterpret_cast<float*>(smem);
  float* d1s = xs + rows * F;
  const float* xb = x + (long long)b * T * F;
  for (int i = threadIdx.x; i < rows * F; i += blockDim.x) {
    const int r = i / F, f = i - r * F;
    int t = t0 - halo + r;
    t = t < 0 ? 0 : (t >= T ? T - 1 : t);
    xs[i] = xb[(long long)t * F + f];
  }
  __syncthreads();
  if (!CONCAT) {
    for (int i = threadIdx.x; i < nt * F; i += blockDim.x) {
      const int r = i / F + halo, f = i % F;
      float acc = 0.f;
      for (int k = 1; k <= n; ++k) acc = fmaf((float)k, xs[(r + k) * F + f] - xs[(r - k) * F + f], acc);
      y[((long long)b * T + t0) * F + i] = acc / denom;
    }
    return;
  }
  // d1 over rows [halo - n, halo + nt + n) with replicate padding at the
  // sequence ends applied to d1 itself (the second Deltas call pads d1).
  const int r1lo = halo - n, r1hi = halo + nt + n;
  for (int i = threadIdx.x; i < (r1hi - r1lo) * F; i += blockDim.x) {
    const int rr = i / F + r1lo, f = i % F;
    int t = t0 - halo + rr;
    t = t < 0 ? 0 : (t >= T ? T - 1 : t);
    float acc = 0.f;
    for (int k = 1; k <= n; ++k) {
      int tp = min(t + k, T - 1) - (t0 - halo);
      int tm = max(t - k, 0) - (t0 - halo);
      acc = fmaf((float)k, xs[tp * F + f] - xs[tm * F + f], acc);
    }
    d1s[rr * F + f] = acc / denom;
  }
  __syncthreads();
  float* yb = y + ((long long)b * T + t0) * 3 * F;
  for (int i = threadIdx.x; i < nt * F; i += blockDim.x) {
    const int lr = i / F, f = i - lr * F;
    const int r = lr + halo;
    float acc = 0.f;
    for (int k = 1; k <= n; ++k) acc = fmaf((float)k, d1s[(r + k) * F + f] - d1s[(r - k) * F + f], acc);
    float* o = yb + (long long)lr * 3 * F;
    o[f] = xs[r * F + f];
    o[F + f] = d1s[r * F + f];
    o[2 * F + f] = acc / denom;
  }
}

// ContextWindow: y[b, t, c*L + k] = x[b, t + k - left, c] (zero outside).
__global__ void context_kernel(const float* __restrict__ x, float* __restrict__ y, int N, int T, int F,
                               int left, int L) {
  const long long total = (long long)N * T * F * L;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(e % L);
    long long r = e / L;
    const int c = (int)(r % F);
    r /= F;
    const int t = (int)(r % T);
    const long long b = r / T;
    const int ts = t + k - left;
    y[e] = (ts >= 0 && ts < T) ? x[(b * T + ts) * F + c] : 0.f;
  }
}

int fill_plan(FftPlan* p, int nc) {
  p->nc = nc;
  p->nstages = 0;
  int rem = nc;
  const int radices[5] = {8, 5, 4, 3, 2};
  while (rem > 1) {
    bool found = false;
    for (int r : radices) {
      if (rem % r == 0) {
        if (p->nstages >= 12) return SBK_ERR_ARG;
        p->radix[p->nstages++] = r;
        rem /= r;
        found = true;
        break;
      }
    }
    if (!found) return SBK_ERR_ARG;
  }
  return 0;
}

inline int grid_for(long long n, int block) {
  long long g = (n + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI (declared in include/sbk.h)
// ---------------------------------------------------------------------------

SBK_API int sbk_fft_supported(int n_fft) {
  FftPlan p;
  if (n_fft < 4 || (n_fft & 1)) return 0;
  return fill_plan(&p, n_fft / 2) == 0 ? 1 : 0;
}

// mode 0: STFT (complex), 1: power spectrum, 2: fused Fbank (mel + dB, pre-top_db)
SBK_API int sbk_spectrum(int mode, const float* wav, int Bo, int S, int C, int n_fft, int hop, int center,
                         int pad_mode, int T, const float* window, const float* twiddle_nc,
                         const float* twiddle_nfft, int onesided, float norm_scale, float power, float eps,
                         int log_mag, const long long* out_strides, const int* mel_start, const int* mel_len,
                         const int* mel_off, const float* mel_w, int n_melw, int M, int log_mel,
                         float multiplier, float db_offset, float amin, float* out, int* maxkey, void* stream) {
  if (Bo <= 0 || T <= 0 || S <= 0 || C <= 0) return SBK_ERR_ARG;
  FftPlan plan;
  if ((n_fft & 1) || fill_plan(&plan, n_fft / 2)) return SBK_ERR_ARG;
  SpecArgs a;
  a.wav = wav; a.S = S; a.C = C; a.Bfold = Bo * C;
  a.n_fft = n_fft; a.hop = hop; a.center = center; a.pad_mode = pad_mode; a.T = T;
  a.window = window;
  a.tw = reinterpret_cast<const float2*>(twiddle_nc);
  a.tw2 = reinterpret_cast<const float2*>(twiddle_nfft);
  a.power = power; a.eps = eps; a.log_mag = log_mag;
  a.os_b = out_strides ? out_strides[0] : 0;
  a.os_c = out_strides ? out_strides[1] : 0;
  a.os_t = out_strides ? out_strides[2] : 0;
  a.os_k = out_strides ? out_strides[3] : 0;
  a.os_ri = out_strides ? out_strides[4] : 0;
  a.onesided = onesided; a.norm_scale = norm_scale;
  a.mel_start = mel_start; a.mel_len = mel_len; a.mel_off = mel_off; a.mel_w = mel_w;
  a.M = M; a.log_mel = log_mel; a.multiplier = multiplier; a.db_offset = db_offset; a.amin = amin;
  a.out = out; a.maxkey = maxkey;
  const int nc = n_fft / 2;
  a.n_melw = mode == MODE_FBANK ? n_melw : 0;
  a.amin_db = multiplier * (float)log10((double)amin) - db_offset;
  if (mode != MODE_FBANK) a.M = 0;
  int fpb = 16;
  auto lds_bytes = [&](int f) {
    return (size_t)2 * f * nc * sizeof(float2) + (size_t)(2 * nc + 1) * sizeof(float2) +
           (size_t)(3 * a.M + a.n_melw + n_fft) * 4 + (size_t)((f - 1) * hop + n_fft) * sizeof(float);
  };
  while (fpb > 1 && lds_bytes(fpb) > 72 * 1024) fpb >>= 1;
  if (lds_bytes(fpb) > 160 * 1024) return SBK_ERR_ARG;
  a.fpb = fpb;
  const int nblk = a.Bfold * ((T + fpb - 1) / fpb);
  hipStream_t s = (hipStream_t)stream;
  if (mode == MODE_FBANK && log_mel) {
    if (C != 1) return SBK_ERR_ARG;
    hipError_t e = hipMemsetD32Async((hipDeviceptr_t)maxkey, (int)0x80000000, a.Bfold, s);
    if (e != hipSuccess) return (int)e;
  }
  switch (mode) {
    case MODE_STFT: hipLaunchKernelGGL(spec_kernel<MODE_STFT>, dim3(nblk), dim3(256), lds_bytes(fpb), s, a, plan); break;
    case MODE_POWER: hipLaunchKernelGGL(spec_kernel<MODE_POWER>, dim3(nblk), dim3(256), lds_bytes(fpb), s, a, plan); break;
    case MODE_FBANK: hipLaunchKernelGGL(spec_kernel<MODE_FBANK>, dim3(nblk), dim3(256), lds_bytes(fpb), s, a, plan); break;
    default: return SBK_ERR_ARG;
  }
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_filterbank(const float* spec, int N, int T, int F, const int* mel_start, const int* mel_len,
                           const int* mel_off, const float* mel_w, const float* dense, int M, int log_mel,
                           float multiplier, float db_offset, float amin, float* out, int* maxkey, void* stream) {
  if (N <= 0 || T <= 0 || F <= 0 || M <= 0) return SBK_ERR_ARG;
  FbArgs a;
  a.spec = spec; a.N = N; a.T = T; a.F = F;
  a.mel_start = mel_start; a.mel_len = mel_len; a.mel_off = mel_off; a.mel_w = mel_w; a.dense = dense;
  a.M = M; a.log_mel = log_mel; a.multiplier = multiplier; a.db_offset = db_offset; a.amin = amin;
  a.amin_db = multiplier * (float)log10((double)amin) - db_offset;
  a.out = out; a.maxkey = maxkey;
  int rpb = 8;
  while (rpb > 1 && (size_t)rpb * F * 4 > 48 * 1024) rpb >>= 1;
  if ((size_t)F * 4 > 160 * 1024) return SBK_ERR_ARG;
  a.rows_per_block = rpb;
  const long long nrows = (long long)N * T;
  hipStream_t s = (hipStream_t)stream;
  if (log_mel) {
    hipError_t e = hipMemsetD32Async((hipDeviceptr_t)maxkey, (int)0x80000000, N, s);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(filterbank_kernel, dim3((unsigned)((nrows + rpb - 1) / rpb)), dim3(256),
                     (size_t)rpb * F * 4, s, a);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_topdb_clamp(float* x, const int* maxkey, long long per_seq, int nseq, float top_db, void* stream) {
  if (per_seq <= 0 || nseq <= 0) return SBK_ERR_ARG;
  hipLaunchKernelGGL(topdb_clamp_kernel, dim3(grid_for(per_seq * nseq / 4 + 1, 256)), dim3(256), 0,
                     (hipStream_t)stream, x, maxkey, per_seq, nseq, top_db);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_magnitude(const float* x, float* y, long long n, int L, float power, float eps, int log_mag,
                          void* stream) {
  if (n <= 0 || L <= 0) return SBK_ERR_ARG;
  hipLaunchKernelGGL(magnitude_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, x, y, n, L,
                     power, eps, log_mag);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_dct(const float* x, const float* D, float* y, long long rows, int n_in, int n_out, void* stream) {
  if (rows <= 0 || n_in <= 0 || n_out <= 0) return SBK_ERR_ARG;
  if ((size_t)n_in * n_out * 4 > 64 * 1024) return SBK_ERR_ARG;
  hipLaunchKernelGGL(dct_kernel, dim3(grid_for(rows * n_out, 256)), dim3(256), (size_t)n_in * n_out * 4,
                     (hipStream_t)stream, x, D, y, rows, n_in, n_out);
  SBK_CHECK_LAUNCH();
  return 0;
}

// concat=0: y = deltas(x) (N,T,F); concat=1: y = [x | d1 | d2] (N,T,3F)
SBK_API int sbk_deltas(const float* x, float* y, int N, int T, int F, int window_length, int concat, void* stream) {
  if (N <= 0 || T <= 0 || F <= 0 || window_length < 3) return SBK_ERR_ARG;
  const int n = (window_length - 1) / 2;
  const float denom = (float)(n * (n + 1) * (2 * n + 1)) / 3.0f;
  int ttile = 64;
  const int halo = concat ? 2 * n : n;
  auto lds = [&](int tt) { return (size_t)(tt + 2 * halo) * F * 4 * (concat ? 2 : 1); };
  while (ttile > 4 && lds(ttile) > 64 * 1024) ttile >>= 1;
  if (lds(ttile) > 160 * 1024) return SBK_ERR_ARG;
  const int nblk = N * ((T + ttile - 1) / ttile);
  if (concat)
    hipLaunchKernelGGL(deltas_kernel<true>, dim3(nblk), dim3(256), lds(ttile), (hipStream_t)stream, x, y, N, T, F,
                       n, denom, ttile);
  else
    hipLaunchKernelGGL(deltas_kernel<false>, dim3(nblk), dim3(256), lds(ttile), (hipStream_t)stream, x, y, N, T, F,
                       n, denom, ttile);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_context_window(const float* x, float* y, int N, int T, int F, int left, int right, void* stream) {
  if (N <= 0 || T <= 0 || F <= 0 || left < 0 || right < 0) return SBK_ERR_ARG;
  const int L = left + right + 1;
  hipLaunchKernelGGL(context_kernel, dim3(grid_for((long long)N * T * F * L, 256)), dim3(256), 0,
                     (hipStream_t)stream, x, y, N, T, F, left, L);
  SBK_CHECK_LAUNCH();
  return 0;
}
