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

// Filterbank._amplitude_to_DB before the top_db clamp (features.py:701-702):
// multiplier·log10(clamp(x, amin)) − multiplier·db_multiplier, with x ≤ amin
// mapped to the host-rounded dB of amin (exactly −100 for 1e-10).  One
// definition shared by the forward kernels and the backward's recompute, so
// the backward sees bit-identical dB values (tie detection against top_db).
__device__ __forceinline__ float to_db(float x, float amin, float amin_db, float mult, float off) {
  return x <= amin ? amin_db : mult * log10f(x) - off;
}


struct FftPlan {
  int nc;          // complex FFT size (n_fft / 2)
  int nstages;
  int radix[12];
};

// Complex arithmetic on packed fp32 pairs (v_pk_add/mul/fma_f32: one VALU op
// per complex add, two per complex multiply); the spectrum kernel is
// VALU-issue bound.
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2f tv(float2 a) { return v2f{a.x, a.y}; }
__device__ __forceinline__ float2 fv(v2f a) { return make_float2(a[0], a[1]); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  // (a.x b.x - a.y b.y, a.x b.y + a.y b.x)
  return fv(__builtin_elementwise_fma(v2f{-a.y, a.y}, v2f{b.y, b.x}, v2f{a.x, a.x} * tv(b)));
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return fv(tv(a) + tv(b)); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return fv(tv(a) - tv(b)); }
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
  float2 m = fv(tv(v[0]) - 0.5f * tv(t));
  float2 sd = fv(s * tv(d));
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
  float2 a = fv(tv(v[0]) + c1 * tv(t1) + c2 * tv(t2));
  float2 b = fv(tv(v[0]) + c2 * tv(t1) + c1 * tv(t2));
  float2 p = fv(s1 * tv(t3) + s2 * tv(t4));
  float2 q = fv(s2 * tv(t3) - s1 * tv(t4));
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
  b[1] = fv(r * (v2f{b[1].x, b[1].y} + v2f{b[1].y, -b[1].x}));          // * (r, -r)
  b[2] = mul_mi(b[2]);                                                  // * -i
  b[3] = fv(r * (v2f{-b[3].x, -b[3].y} + v2f{b[3].y, -b[3].x}));        // * (-r, -r)
  dft_small<4>(a);
  dft_small<4>(b);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = a[i];
    v[2 * i + 1] = b[i];
  }
}

// LDS layout of a frame's complex buffer: one float2 of padding every 8, so
// the radix-8 first stage's stride-8 writes (and the later stages' strided
// writes) hit distinct 64-bit bank pairs; frames are NCP float2 apart with
// NCP odd so neighbouring frames do not alias either.
__host__ __device__ constexpr int fpad(int i) { return i + (i >> 3); }
__host__ __device__ constexpr int frame_stride(int nc) { return (fpad(nc - 1) + 1) | 1; }
__host__ __device__ constexpr int first_radix(int n) {
  return n % 8 == 0 ? 8 : n % 5 == 0 ? 5 : n % 4 == 0 ? 4 : n % 3 == 0 ? 3 : n % 2 == 0 ? 2 : 0;
}

template <int R>
__device__ __forceinline__ void stockham_task(const float2* __restrict__ s, float2* __restrict__ d, int j, int nb,
                                              int Ns, int k, int step, const float2* __restrict__ tw) {
  float2 v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) v[r] = s[fpad(j + r * nb)];
#pragma unroll
  for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw[r * k * step]);
  dft_small<R>(v);
  const int idxD = (j - k) * R + k;  // (j / Ns) * Ns * R + k
#pragma unroll
  for (int r = 0; r < R; ++r) d[fpad(idxD + r * Ns)] = v[r];
}

// One Stockham autosort stage of radix R over the block's frames (runtime size).
template <int R>
__device__ __forceinline__ void stockham_stage(const float2* __restrict__ src, float2* __restrict__ dst,
                                               int nc, int ncp, int Ns, const float2* __restrict__ tw, int nframes) {
  const int nb = nc / R;
  const int step = nc / (Ns * R);
  int f = 0, j = threadIdx.x;
  while (j >= nb) { j -= nb; ++f; }
  while (f < nframes) {
    stockham_task<R>(src + f * ncp, dst + f * ncp, j, nb, Ns, j % Ns, step, tw);
    j += blockDim.x;
    while (j >= nb) { j -= nb; ++f; }
  }
}

// Runs the whole complex FFT (runtime plan); returns the buffer holding the result.
__device__ float2* run_fft(float2* bufA, float2* bufB, const FftPlan& plan, int ncp, const float2* tw, int nframes) {
  float2* src = bufA;
  float2* dst = bufB;
  int Ns = 1;
  for (int s = 0; s < plan.nstages; ++s) {
    __syncthreads();
    switch (plan.radix[s]) {
      case 8: stockham_stage<8>(src, dst, plan.nc, ncp, Ns, tw, nframes); break;
      case 5: stockham_stage<5>(src, dst, plan.nc, ncp, Ns, tw, nframes); break;
      case 4: stockham_stage<4>(src, dst, plan.nc, ncp, Ns, tw, nframes); break;
      case 3: stockham_stage<3>(src, dst, plan.nc, ncp, Ns, tw, nframes); break;
      default: stockham_stage<2>(src, dst, plan.nc, ncp, Ns, tw, nframes); break;
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
  int wav16;         // wav is 16-B aligned (the register-FFT kernel's LDS-DMA span staging needs it)
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
  float* slot_max;  // (Bfold, ceil(T / fpb)) per-block max dB (top_db reference)
};

enum { MODE_STFT = 0, MODE_POWER = 1, MODE_FBANK = 2 };

// Visits (f, j), f < nf, j < W, in the order of i = f*W + j strided by the
// block size, without a runtime division per element.
template <class Fn>
__device__ __forceinline__ void for_fj(int nf, int W, Fn&& fn) {
  int f = 0, j = threadIdx.x;
  while (j >= W) { j -= W; ++f; }
  while (f < nf) {
    fn(f, j);
    j += blockDim.x;
    while (j >= W) { j -= W; ++f; }
  }
}

// Runtime-plan spectrum kernel (any n_fft the radix set supports).
template <int MODE>
__global__ void __launch_bounds__(256) spec_kernel(SpecArgs a, FftPlan plan) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ float red[4];
  const int nc = plan.nc;
  const int ncp = frame_stride(nc);
  const int nblk_t = (a.T + a.fpb - 1) / a.fpb;
  const int bf = blockIdx.x / nblk_t;
  const int t0 = (blockIdx.x - bf * nblk_t) * a.fpb;
  const int nf = min(a.fpb, a.T - t0);
  const int bo = bf / a.C, ch = bf - bo * a.C;
  const float* wrow = a.wav + (long long)bo * a.S * a.C + ch;

  float2* bufA = reinterpret_cast<float2*>(smem);
  float2* bufB = bufA + a.fpb * ncp;
  float* tab = reinterpret_cast<float*>(bufB + a.fpb * ncp);  // tables, staged once per block
  float2* tw = reinterpret_cast<float2*>(tab);                // W_nc^m
  float2* tw2 = tw + nc;                                      // W_nfft^k, k <= nc
  int* mstart = reinterpret_cast<int*>(tw2 + nc + 1);
  int* mlen = mstart + a.M;
  int* moff = mlen + a.M;
  float* mw = reinterpret_cast<float*>(moff + a.M);
  // table segments: [tw | tw2 | mstart | mlen | moff | mw]
  const int b1 = 2 * nc, b2 = b1 + 2 * nc + 2, b3 = b2 + a.M, b4 = b3 + a.M, b5 = b4 + a.M;
  const int ntab = b5 + a.n_melw;

  // 1) prologue: every global load of a chunk (tables, frame samples, window)
  //    is issued before the first LDS store, so the block pays one memory
  //    latency instead of one per table / sample row.
  const int pad = a.center ? a.n_fft / 2 : 0;
  const int base = t0 * a.hop - pad;
  const int span = (nf - 1) * a.hop + a.n_fft;
  const bool interior = base >= 0 && base + span <= a.S;
  const bool vec2 = interior && a.C == 1 && ((a.hop | base | a.S) & 1) == 0;
  const int nfe = nf * nc;
  constexpr int KT = 8, KF = 8;
  for (int tb = 0, fb = 0; tb < ntab || fb < nfe; tb += KT * 256, fb += KF * 256) {
    float tv[KT];
    float2 fv[KF], wv[KF];
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      const int i = tb + (int)threadIdx.x + u * 256;
      float v = 0.f;
      if (i < b1) v = reinterpret_cast<const float*>(a.tw)[i];
      else if (i < b2) v = reinterpret_cast<const float*>(a.tw2)[i - b1];
      else if (i < b3) v = __int_as_float(a.mel_start[i - b2]);
      else if (i < b4) v = __int_as_float(a.mel_len[i - b3]);
      else if (i < b5) v = __int_as_float(a.mel_off[i - b4]);
      else if (i < ntab) v = a.mel_w[i - b5];
      tv[u] = v;
    }
#pragma unroll
    for (int u = 0; u < KF; ++u) {
      const int e = fb + (int)threadIdx.x + u * 256;
      fv[u] = wv[u] = make_float2(0.f, 0.f);
      if (e < nfe) {
        const int f = e / nc, m = e - f * nc;
        const int q = f * a.hop + 2 * m;
        wv[u] = *reinterpret_cast<const float2*>(a.window + 2 * m);
        if (vec2) {
          fv[u] = *reinterpret_cast<const float2*>(wrow + base + q);
        } else if (interior) {
          fv[u] = make_float2(wrow[(long long)(base + q) * a.C], wrow[(long long)(base + q + 1) * a.C]);
        } else {
          bool ok0, ok1;
          const int p0 = map_pos(base + q, a.S, a.pad_mode, &ok0);
          const int p1 = map_pos(base + q + 1, a.S, a.pad_mode, &ok1);
          fv[u] = make_float2(ok0 ? wrow[(long long)p0 * a.C] : 0.f, ok1 ? wrow[(long long)p1 * a.C] : 0.f);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      const int i = tb + (int)threadIdx.x + u * 256;
      if (i < ntab) tab[i] = tv[u];
    }
#pragma unroll
    for (int u = 0; u < KF; ++u) {
      const int e = fb + (int)threadIdx.x + u * 256;
      if (e < nfe) {
        const int f = e / nc, m = e - f * nc;
        bufA[f * ncp + fpad(m)] = make_float2(fv[u].x * wv[u].x, fv[u].y * wv[u].y);
      }
    }
  }
  // 3) complex FFT of size nc
  float2* Z = run_fft(bufA, bufB, plan, ncp, tw, nf);
  float2* other = (Z == bufA) ? bufB : bufA;

  // 4) split into the real-input spectrum X[k], k = 0..nc
  const int nbins = nc + 1;
  if (MODE == MODE_STFT) {
    const int nout = a.onesided ? nbins : a.n_fft;
    for_fj(nf, nout, [&](int f, int kk) {
      const bool mirror = kk > nc;
      const int k = mirror ? a.n_fft - kk : kk;
      const float2 zk = Z[f * ncp + fpad(k == nc ? 0 : k)];
      const float2 zr = Z[f * ncp + fpad(k == 0 ? 0 : nc - k)];
      const float2 zc = make_float2(zr.x, -zr.y);
      const float2 E = make_float2(0.5f * (zk.x + zc.x), 0.5f * (zk.y + zc.y));
      const float2 O = mul_mi(make_float2(0.5f * (zk.x - zc.x), 0.5f * (zk.y - zc.y)));
      float2 X = cadd(E, cmul(tw2[k], O));
      if (mirror) X.y = -X.y;
      float* o = a.out + bo * a.os_b + ch * a.os_c + (long long)(t0 + f) * a.os_t + kk * a.os_k;
      o[0] = X.x * a.norm_scale;
      o[a.os_ri] = X.y * a.norm_scale;
    });
    return;
  }
  float* P = reinterpret_cast<float*>(other);  // (nf, nbins) power
  for_fj(nf, nbins, [&](int f, int k) {
    const float2 zk = Z[f * ncp + fpad(k == nc ? 0 : k)];
    const float2 zr = Z[f * ncp + fpad(k == 0 ? 0 : nc - k)];
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
      P[f * nbins + k] = s;
    }
  });
  if (MODE == MODE_POWER) return;
  __syncthreads();
  // 5) sparse mel projection + dB + running max
  float lmax = -INFINITY;
  float* orow = a.out + ((long long)bf * a.T + t0) * a.M;
  for_fj(nf, a.M, [&](int f, int j) {
    const float* pf = P + f * nbins + mstart[j];
    const float* w = mw + moff[j];
    const int L = mlen[j];
    float acc = 0.f;
    for (int q = 0; q < L; ++q) acc = fmaf(pf[q], w[q], acc);
    if (a.log_mel) {
      // clamp(x, amin) -> the host-rounded dB of amin exactly (-100 for 1e-10)
      acc = to_db(acc, a.amin, a.amin_db, a.multiplier, a.db_offset);
      lmax = fmaxf(lmax, acc);
    }
    orow[f * a.M + j] = acc;
  });
  if (a.log_mel) {  // one partial max per block, reduced by the top_db kernel (no atomics)
    const float m = block_max(lmax, red);
    if (threadIdx.x == 0) a.slot_max[blockIdx.x] = m;
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
  float* slot_max;  // (N, ceil(T / rows_per_block)) per-block max dB
};

// One block per (sequence n, tile of rows_per_block frames).
__global__ void __launch_bounds__(256) filterbank_kernel(FbArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ float red[4];
  float* rowbuf = reinterpret_cast<float*>(smem);
  const int nblk_t = (a.T + a.rows_per_block - 1) / a.rows_per_block;
  const int n = blockIdx.x / nblk_t;
  const long long r0 = (long long)n * a.T + (long long)(blockIdx.x - n * nblk_t) * a.rows_per_block;
  const int nr = (int)min((long long)a.rows_per_block, (long long)(n + 1) * a.T - r0);
  for (int i = threadIdx.x; i < nr * a.F; i += blockDim.x) rowbuf[i] = a.spec[r0 * a.F + i];
  __syncthreads();
  float lmax = -INFINITY;
  for_fj(nr, a.M, [&](int rr, int j) {
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
      acc = to_db(acc, a.amin, a.amin_db, a.multiplier, a.db_offset);
      lmax = fmaxf(lmax, acc);
    }
    a.out[(r0 + rr) * a.M + j] = acc;
  });
  if (a.log_mel) {
    const float m = block_max(lmax, red);
    if (threadIdx.x == 0) a.slot_max[blockIdx.x] = m;
  }
}

// x[n, :] = max(x[n, :], max_n - top_db), per sequence n of `per_seq` floats;
// max_n is the max of the sequence's nslot per-block partial maxima.
// Grid (chunks, nseq): every block reduces its sequence's partials first.
__global__ void __launch_bounds__(256) topdb_clamp_kernel(float* __restrict__ x, const float* __restrict__ slot_max,
                                                          int nslot, long long per_seq, float top_db) {
  __shared__ float red[4];
  const int n = blockIdx.y;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < nslot; i += blockDim.x) m = fmaxf(m, slot_max[(long long)n * nslot + i]);
  const float fl = block_max(m, red) - top_db;
  float* xs = x + (long long)n * per_seq;
  const long long chunk = (long long)blockDim.x * 16;
  const long long c0 = (long long)blockIdx.x * chunk, c1 = min(per_seq, c0 + chunk);
  if ((per_seq & 3) == 0) {
    for (long long i = c0 + threadIdx.x * 4; i < c1; i += blockDim.x * 4) {
      float4 v = *reinterpret_cast<float4*>(xs + i);
      v.x = fmaxf(v.x, fl);
      v.y = fmaxf(v.y, fl);
      v.z = fmaxf(v.z, fl);
      v.w = fmaxf(v.w, fl);
      *reinterpret_cast<float4*>(xs + i) = v;
    }
  } else {
    for (long long i = c0 + threadIdx.x; i < c1; i += blockDim.x) xs[i] = fmaxf(xs[i], fl);
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

// The [x | d1 | d2] concat with float4 columns (F % 4 == 0, 16-B aligned):
// the scalar kernel above moved one float per thread with an integer divide
// per element (30.6 us at config 2, 2.0 TB/s).  Here each thread moves
// float4s, the tile load issues four independent loads per thread before
// any LDS store, and each output row leaves as 3 x F/4 float4 stores.  Same
// arithmetic order per element as deltas_kernel<true>.
// slot_max (optional): the fbank's per-workgroup maxima of sequence b
// (sbk_spectrum with the floor deferred): x is floored at max_b - top_db as
// it loads (features.py:706-711, the separate clamp pass folded in).
__global__ void __launch_bounds__(256) deltas4_concat_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                             int N, int T, int F, int n, float denom, int ttile,
                                                             const float* __restrict__ slot_max, int nslot,
                                                             float top_db) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ float red[4];
  const int F4 = F >> 2, halo = 2 * n;
  const int ntile = (T + ttile - 1) / ttile;
  const int b = blockIdx.x / ntile;
  const int t0 = (blockIdx.x - b * ntile) * ttile;
  const int nt = min(ttile, T - t0);
  const int rows = nt + 2 * halo;
  float4* xs = reinterpret_cast<float4*>(smem);
  float4* d1s = xs + rows * F4;
  const float4* xb = reinterpret_cast<const float4*>(x + (long long)b * T * F);
  const int nld = rows * F4;
  float fl = -INFINITY;
  if (slot_max) {
    float m = -INFINITY;
    for (int i = threadIdx.x; i < nslot; i += 256) m = fmaxf(m, slot_max[(long long)b * nslot + i]);
    fl = block_max(m, red) - top_db;
  }
  for (int base = threadIdx.x; base < nld; base += 4 * 256) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = min(base + u * 256, nld - 1), r = i / F4, q = i - r * F4;
      const int t = min(max(t0 - halo + r, 0), T - 1);
      v[u] = xb[(long long)t * F4 + q];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (base + u * 256 < nld) {
        float4 w = v[u];
        if (slot_max) w = make_float4(fmaxf(w.x, fl), fmaxf(w.y, fl), fmaxf(w.z, fl), fmaxf(w.w, fl));
        xs[base + u * 256] = w;
      }
  }
  __syncthreads();
  // d1 over rows [halo - n, halo + nt + n), replicate padding applied to d1
  const int r1lo = halo - n, r1hi = halo + nt + n;
  for (int i = threadIdx.x; i < (r1hi - r1lo) * F4; i += 256) {
    const int rr = i / F4 + r1lo, q = i % F4;
    const int t = min(max(t0 - halo + rr, 0), T - 1);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 1; k <= n; ++k) {
      const float4 p = xs[(min(t + k, T - 1) - (t0 - halo)) * F4 + q];
      const float4 m = xs[(max(t - k, 0) - (t0 - halo)) * F4 + q];
      const float kf = (float)k;
      acc.x = fmaf(kf, p.x - m.x, acc.x);
      acc.y = fmaf(kf, p.y - m.y, acc.y);
      acc.z = fmaf(kf, p.z - m.z, acc.z);
      acc.w = fmaf(kf, p.w - m.w, acc.w);
    }
    d1s[rr * F4 + q] = make_float4(acc.x / denom, acc.y / denom, acc.z / denom, acc.w / denom);
  }
  __syncthreads();
  float4* yb = reinterpret_cast<float4*>(y + ((long long)b * T + t0) * 3 * F);
  for (int i = threadIdx.x; i < nt * F4; i += 256) {
    const int lr = i / F4, q = i - lr * F4;
    const int r = lr + halo;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 1; k <= n; ++k) {
      const float4 p = d1s[(r + k) * F4 + q], m = d1s[(r - k) * F4 + q];
      const float kf = (float)k;
      acc.x = fmaf(kf, p.x - m.x, acc.x);
      acc.y = fmaf(kf, p.y - m.y, acc.y);
      acc.z = fmaf(kf, p.z - m.z, acc.z);
      acc.w = fmaf(kf, p.w - m.w, acc.w);
    }
    float4* o = yb + (long long)lr * 3 * F4;
    o[q] = xs[r * F4 + q];
    o[F4 + q] = d1s[r * F4 + q];
    o[2 * F4 + q] = make_float4(acc.x / denom, acc.y / denom, acc.z / denom, acc.w / denom);
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


// ---------------------------------------------------------------------------
// Static-plan spectrum kernel for the common FFT sizes (n_fft 400/512/1024/
// 2048).  NT threads own FPB frames; every stage's task -> thread map is a
// compile-time constant, so the per-element index arithmetic folds away and
// each thread runs a fixed, branch-free set of butterflies:
//   * stage 0 reads its radix-R0 inputs straight from the waveform (window
//     applied in registers), so the frames never pass through LDS raw;
//   * later stages run in place (read -> barrier -> write -> barrier) on one
//     padded LDS buffer per frame;
//   * the real-FFT split handles bins k and nc-k in one thread.
// For n_fft 400 (nc 200 = 8*5*5): FPB 8, NT 320 -> each radix-5 stage is
// exactly one task per thread.
// Round 2 (B = 32 x 15 s, Fbank incl. top_db 62.6 us): skipping the radix-5
// stages saves 9 us and the mel loop 4 us, so neither the FFT nor the
// filters set the time.  A wave-per-frame variant (three in-register
// Stockham stages, wave-private LDS exchanges, one block barrier) measured
// 81 us with global tables and 66 us with LDS tables: not kept.  Workgroups
// looping over G groups of 8 frames (tables staged once, one slot max per
// workgroup; the thread index made opaque per group to stop the compiler
// hoisting every stage's index math out of the loop): 70.6 / 61.7 / 60.9 /
// 59.7 / 94.5 us for G = 1 / 2 / 4 / 8 / 16 against 55.7 us: per-workgroup
// setup is not the cost either.
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int plan_nstages(int nc) {
  int n = 0;
  while (nc > 1) { nc /= first_radix(nc); ++n; }
  return n;
}
__host__ __device__ constexpr int plan_radix(int nc, int s) {
  for (int i = 0; i < s; ++i) nc /= first_radix(nc);
  return first_radix(nc);
}
__host__ __device__ constexpr int plan_ns(int nc, int s) {
  int ns = 1;
  for (int i = 0; i < s; ++i) { const int r = first_radix(nc); ns *= r; nc /= r; }
  return ns;
}

template <int NC, int FPB, int NT, int S>
__device__ __forceinline__ void static_stage(float2* __restrict__ buf, const float2* __restrict__ tw) {
  if constexpr (S < plan_nstages(NC)) {
    constexpr int R = plan_radix(NC, S), NS = plan_ns(NC, S), NB = NC / R;
    constexpr int STEP = NC / (NS * R), NCP = frame_stride(NC);
    constexpr int TASKS = FPB * NB, TPT = (TASKS + NT - 1) / NT;
    float2 v[TPT][R];
#pragma unroll
    for (int u = 0; u < TPT; ++u) {
      const int t = threadIdx.x + u * NT;
      if (TASKS % NT == 0 || t < TASKS) {
        const int f = t / NB, j = t - f * NB;
#pragma unroll
        for (int r = 0; r < R; ++r) v[u][r] = buf[f * NCP + fpad(j + r * NB)];
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < TPT; ++u) {
      const int t = threadIdx.x + u * NT;
      if (TASKS % NT == 0 || t < TASKS) {
        const int f = t / NB, j = t - f * NB, k = j % NS;
#pragma unroll
        for (int r = 1; r < R; ++r) v[u][r] = cmul(v[u][r], tw[r * k * STEP]);
        dft_small<R>(v[u]);
#pragma unroll
        for (int r = 0; r < R; ++r) buf[f * NCP + fpad((j - k) * R + k + r * NS)] = v[u][r];
      }
    }
    __syncthreads();
    static_stage<NC, FPB, NT, S + 1>(buf, tw);
  }
}

// s_memtime marks of wave 0 of every workgroup (probe builds only): start,
// stage 0 done, FFT done, split done, mel done, end, hardware / XCC id
SBK_PROBE_BUFFER(g_spec_tl, 8192, 8)
#define SPEC_TL(i) SBK_PROBE(if (threadIdx.x == 0 && blockIdx.x < 8192) g_spec_tl[blockIdx.x][i] = __builtin_amdgcn_s_memtime();)

template <int MODE, int NC, int FPB, int NT>
__global__ void __launch_bounds__(NT) spec_static_kernel(SpecArgs a) {
  SPEC_TL(0);
  SBK_PROBE(if (threadIdx.x == 0 && blockIdx.x < 8192) g_spec_tl[blockIdx.x][6] =
                (unsigned long long)__builtin_amdgcn_s_getreg(63492) |
                ((unsigned long long)__builtin_amdgcn_s_getreg(30740) << 32) | ((unsigned long long)blockIdx.x << 40);)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ float red[NT / 64];
  constexpr int NCP = frame_stride(NC), NBINS = NC + 1;
  const int tid = threadIdx.x;
  const int nblk_t = (a.T + FPB - 1) / FPB;
  const int bf = blockIdx.x / nblk_t;
  const int t0 = (blockIdx.x - bf * nblk_t) * FPB;
  const int nf = min(FPB, a.T - t0);
  const int bo = bf / a.C, ch = bf - bo * a.C;
  const float* wrow = a.wav + (long long)bo * a.S * a.C + ch;

  float2* buf = reinterpret_cast<float2*>(smem);                 // FPB x NCP complex
  float* P = reinterpret_cast<float*>(buf + FPB * NCP);           // FPB x NBINS power (FBANK)
  float* tab = P + (MODE == MODE_FBANK ? FPB * NBINS : 0);
  float2* tw = reinterpret_cast<float2*>(tab);                    // W_nc^m
  float2* tw2 = tw + NC;                                          // W_nfft^k
  int* mstart = reinterpret_cast<int*>(tw2 + NC + 1);
  int* mlen = mstart + a.M;
  int* moff = mlen + a.M;
  float* mw = reinterpret_cast<float*>(moff + a.M);
  // ---- tables: per-segment loads issued first, stored once the frame loads
  //      are in flight too (one memory latency for the whole prologue)
  constexpr int KW = (NC + NT - 1) / NT, KW2 = (NC + 1 + NT - 1) / NT, KMW = 4;
  float2 tv1[KW], tv2[KW2];
  float mwv[KMW];
  int ms = 0, ml = 0, mo = 0;
#pragma unroll
  for (int u = 0; u < KW; ++u) {
    const int i = tid + u * NT;
    tv1[u] = (NC % NT == 0 || i < NC) ? a.tw[i] : make_float2(0.f, 0.f);
  }
#pragma unroll
  for (int u = 0; u < KW2; ++u) {
    const int i = tid + u * NT;
    tv2[u] = i <= NC ? a.tw2[i] : make_float2(0.f, 0.f);
  }
  if constexpr (MODE == MODE_FBANK) {
    if (tid < a.M) {
      ms = a.mel_start[tid];
      ml = a.mel_len[tid];
      mo = a.mel_off[tid];
    }
#pragma unroll
    for (int u = 0; u < KMW; ++u) {
      const int i = tid + u * NT;
      mwv[u] = i < a.n_melw ? a.mel_w[i] : 0.f;
    }
  }

  // ---- stage 0 straight from the waveform: radix-R0 butterflies, Ns = 1
  {
    constexpr int R = first_radix(NC), NB = NC / R;
    constexpr int TASKS = FPB * NB, TPT = (TASKS + NT - 1) / NT;
    const int pad = a.center ? a.n_fft / 2 : 0;
    const int base = t0 * a.hop - pad;
    const int span = (nf - 1) * a.hop + a.n_fft;
    const bool interior = base >= 0 && base + span <= a.S;
    const bool vec2 = interior && a.C == 1 && ((a.hop | base | a.S) & 1) == 0;
    float2 v[TPT][R];
#pragma unroll
    for (int u = 0; u < TPT; ++u) {
      const int t = tid + u * NT;
      const int f = t / NB, j = t - f * NB;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int m = j + r * NB;
        float2 x = make_float2(0.f, 0.f);
        if ((TASKS % NT == 0 || t < TASKS) && f < nf) {
          const int q = base + f * a.hop + 2 * m;
          if (vec2) {  // row pointer once per task, constant offsets per r
            x = *reinterpret_cast<const float2*>(wrow + (base + f * a.hop + 2 * j) + 2 * r * NB);
          } else if (interior) {
            x = make_float2(wrow[(long long)q * a.C], wrow[(long long)(q + 1) * a.C]);
          } else {
            bool ok0, ok1;
            const int p0 = map_pos(q, a.S, a.pad_mode, &ok0);
            const int p1 = map_pos(q + 1, a.S, a.pad_mode, &ok1);
            x = make_float2(ok0 ? wrow[(long long)p0 * a.C] : 0.f, ok1 ? wrow[(long long)p1 * a.C] : 0.f);
          }
          const float2 w = *reinterpret_cast<const float2*>(a.window + 2 * j + 2 * r * NB);
          x.x *= w.x;
          x.y *= w.y;
        }
        v[u][r] = x;
      }
    }
#pragma unroll
    for (int u = 0; u < KW; ++u) {
      const int i = tid + u * NT;
      if (NC % NT == 0 || i < NC) tw[i] = tv1[u];
    }
#pragma unroll
    for (int u = 0; u < KW2; ++u) {
      const int i = tid + u * NT;
      if (i <= NC) tw2[i] = tv2[u];
    }
    if constexpr (MODE == MODE_FBANK) {
      if (tid < a.M) {
        mstart[tid] = ms;
        mlen[tid] = ml;
        moff[tid] = mo;
      }
      for (int i = tid + NT; i < a.M; i += NT) {  // M > NT (rare)
        mstart[i] = a.mel_start[i];
        mlen[i] = a.mel_len[i];
        moff[i] = a.mel_off[i];
      }
#pragma unroll
      for (int u = 0; u < KMW; ++u) {
        const int i = tid + u * NT;
        if (i < a.n_melw) mw[i] = mwv[u];
      }
      for (int i = tid + KMW * NT; i < a.n_melw; i += NT) mw[i] = a.mel_w[i];
    }
#pragma unroll
    for (int u = 0; u < TPT; ++u) {
      const int t = tid + u * NT;
      if (TASKS % NT == 0 || t < TASKS) {
        const int f = t / NB, j = t - f * NB;
        dft_small<R>(v[u]);
#pragma unroll
        for (int r = 0; r < R; ++r) buf[f * NCP + fpad(j * R + r)] = v[u][r];
      }
    }
    __syncthreads();
  }
  SPEC_TL(1);
  // ---- remaining stages in place
  static_stage<NC, FPB, NT, 1>(buf, tw);
  SPEC_TL(2);

  // ---- real split: bins k and NC-k per task
  constexpr int NPAIR = NC / 2 + 1, TASKS = FPB * NPAIR, TPT = (TASKS + NT - 1) / NT;
#pragma unroll
  for (int u = 0; u < TPT; ++u) {
    const int t = tid + u * NT;
    if (!(TASKS % NT == 0 || t < TASKS)) continue;
    const int f = t / NPAIR, k = t - f * NPAIR;
    if (f >= nf) continue;
    const float2 zk = buf[f * NCP + fpad(k)];
    const float2 zr = buf[f * NCP + fpad(k == 0 ? 0 : NC - k)];
    float2 X[2];
    int bins[2] = {k, NC - k};
    const int nb = (k == NC - k) ? 1 : 2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float2 za = h ? zr : zk, zb = h ? zk : zr;
      const float2 zc = make_float2(zb.x, -zb.y);
      const float2 E = make_float2(0.5f * (za.x + zc.x), 0.5f * (za.y + zc.y));
      const float2 O = mul_mi(make_float2(0.5f * (za.x - zc.x), 0.5f * (za.y - zc.y)));
      X[h] = cadd(E, cmul(tw2[bins[h]], O));
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h >= nb) break;
      const int kk = bins[h];
      float2 x = X[h];
      x.x *= a.norm_scale;
      x.y *= a.norm_scale;
      if (MODE == MODE_STFT) {
        float* o = a.out + bo * a.os_b + ch * a.os_c + (long long)(t0 + f) * a.os_t + kk * a.os_k;
        o[0] = x.x;
        o[a.os_ri] = x.y;
      } else {
        float p = x.x * x.x + x.y * x.y;
        if (a.power != 1.0f) {
          if (a.power < 1.0f) p += a.eps;
          p = powf(p, a.power);
        }
        if (MODE == MODE_POWER) {
          if (a.log_mag) p = logf(p + a.eps);
          a.out[bo * a.os_b + ch * a.os_c + (long long)(t0 + f) * a.os_t + kk * a.os_k] = p;
        } else {
          P[f * NBINS + kk] = p;
        }
      }
    }
  }
  SPEC_TL(3);
  if constexpr (MODE == MODE_FBANK) {
    __syncthreads();
    float lmax = -INFINITY;
    float* orow = a.out + ((long long)bf * a.T + t0) * a.M;
    // lane -> (mel j = t / FPB, frame f = t % FPB): a wave covers 64/FPB
    // neighbouring filters, whose lengths are nearly equal (little divergence)
    for (int t = tid; t < a.M * FPB; t += NT) {
      const int j = t / FPB, f = t - j * FPB;
      if (f >= nf) continue;
      const float* pf = P + f * NBINS + mstart[j];
      const float* w = mw + moff[j];
      const int L = mlen[j];
      float acc = 0.f;
      for (int q = 0; q < L; ++q) acc = fmaf(pf[q], w[q], acc);
      if (a.log_mel) {
        acc = to_db(acc, a.amin, a.amin_db, a.multiplier, a.db_offset);
        lmax = fmaxf(lmax, acc);
      }
      orow[f * a.M + j] = acc;
    }
    SPEC_TL(4);
    if (a.log_mel) {
      const float m = block_max(lmax, red);
      if (tid == 0) a.slot_max[blockIdx.x] = m;
    }
  }
  SPEC_TL(5);
}

// ---------------------------------------------------------------------------
// Register-FFT spectrum kernel, n_fft = 400 (nc = 200 = 8 x 25), mono, power
// spectrum or fused Fbank.  Eight lanes own one frame and a wave eight
// frames; the complex FFT is a 25 x 8 decomposition and a wave never waits
// on another after the table stage (persistent workgroups, tables once):
//   * the wave's 8 frames are one contiguous span of samples: LDS-DMA puts it
//     in the wave's frame regions (6 x 16 B per lane); lane n1 (0..7) then
//     reads z[8 n2 + n1], n2 = 0..24 (window from LDS) and runs a DFT-25
//     (5 x 5, compile-time twiddles) in registers;
//   * twiddle by W_200^(n1 k2), then a wave-private LDS transposition: lane
//     n1 writes Y[k2][n1]; each lane reads back the eight Y[k2][.] of a
//     unit {m, 25 - m} (m = 1..12, unit 0 = {0}) and runs two radix-8 DFTs,
//     which gives Z[k2 + 25 k1] for both k2 of the unit, k1 = 0..7 (two
//     passes of 13 / 12 rows, so a frame region is 848 B, not 1.6 KB);
//   * the real split X[k] = E + W_400^k O pairs bin k with 200 - k, which
//     lives in the same unit, so no second exchange: |X|^2 goes to the
//     frame's LDS region (over its consumed Y), then the mel filters as dense
//     16-B rows from each filter's aligned first bin (zero weights outside),
//     dB, and one partial max per wave (= per 8 frames: the slot layout of
//     the static kernel).
// Fbank at config 3: 53.2 us (static kernel, ~18k cycles per 8 frames, half
// of it behind its prologue loads, most of the rest at in-place stage
// barriers) -> 42.8 us.  Measured on the way: the first version (strided
// 8-B waveform loads, a 1.6 KB region per frame, 2 workgroups of 4 waves per
// CU) 42.9 us; window / twiddles read from their global tables per use
// 75 us (the vector-memory address rate); without the span staging 55.6 us;
// non-persistent 52.4 us.  s_memtime per wave (scripts/rf_tl.py): the load
// phase (all waves of a round fetching at once) and the mel phase dominate.
// ---------------------------------------------------------------------------
#ifndef SBK_RF_NW
#define SBK_RF_NW 4
#define SBK_RF_MINW 3
#endif
// 4 waves x 8 frames, three workgroups per CU (LDS), <= 168 VGPRs (no spills):
// 42.8 us against 45.9 us for 8-wave workgroups at 128 VGPRs (spills) and
// 44.3 us for one 8-wave workgroup per CU
constexpr int RF_NW = SBK_RF_NW, RF_NT = RF_NW * 64;
constexpr int RF_FS = 13 * 8 + 2;              // float2 per frame region (13 rows of Y[k2][8] / P[201]);
                                               // 212 floats = 20 mod 64 banks: frames on distinct banks
constexpr int RF_PAD = 24;                     // float2 of zeros after a wave's 8 regions
constexpr int RF_WS = 8 * RF_FS + RF_PAD;      // float2 per wave
constexpr int RF_SPAN = 1536;                  // staged samples per wave (6 KB: 8 frames at hop <= 162)
static_assert(RF_SPAN <= 2 * RF_WS, "the span fits the wave's regions");
constexpr int RF_LW = 36;                      // dense mel row: 16-B aligned start + up to 33 bins
typedef float rf4 __attribute__((ext_vector_type(4)));
#ifndef SBK_RF_WGS_PER_CU
#define SBK_RF_WGS_PER_CU 3                    // persistent grid: workgroups per CU (LDS: three fit)
#endif

// compile-time W_25^m for the DFT-25 (Taylor series in double, |x| <= pi)
__host__ __device__ constexpr double cx_sin(double x) {
  double t = x, s = x;
  for (int n = 1; n < 16; ++n) { t *= -x * x / ((2.0 * n) * (2.0 * n + 1.0)); s += t; }
  return s;
}
__host__ __device__ constexpr double cx_cos(double x) {
  double t = 1.0, s = 1.0;
  for (int n = 1; n < 16; ++n) { t *= -x * x / ((2.0 * n - 1.0) * (2.0 * n)); s += t; }
  return s;
}
struct Tw25 {
  float re[25], im[25];
};
__host__ __device__ constexpr Tw25 make_tw25() {
  Tw25 t{};
  for (int m = 0; m < 25; ++m) {
    double th = 2.0 * 3.14159265358979323846 * m / 25.0;
    if (th > 3.14159265358979323846) th -= 2.0 * 3.14159265358979323846;
    t.re[m] = (float)cx_cos(th);
    t.im[m] = (float)-cx_sin(th);
  }
  return t;
}
__device__ constexpr Tw25 kTw25 = make_tw25();

// DFT-25 in registers, natural order in and out: n = 5a + b, U_b = DFT5_a,
// U_b[c] *= W_25^(bc), X[c + 5d] = DFT5_b U_b[c]
__device__ __forceinline__ void dft25(float2 (&x)[25]) {
  float2 u[5][5];
#pragma unroll
  for (int b = 0; b < 5; ++b) {
#pragma unroll
    for (int a = 0; a < 5; ++a) u[b][a] = x[5 * a + b];
    dft_small<5>(u[b]);
  }
#pragma unroll
  for (int b = 1; b < 5; ++b)
#pragma unroll
    for (int c = 1; c < 5; ++c) {
      const int m = (b * c) % 25;
      u[b][c] = cmul(u[b][c], make_float2(kTw25.re[m], kTw25.im[m]));
    }
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    float2 t[5];
#pragma unroll
    for (int b = 0; b < 5; ++b) t[b] = u[b][c];
    dft_small<5>(t);
#pragma unroll
    for (int d = 0; d < 5; ++d) x[c + 5 * d] = t[d];
  }
}

// real-FFT split of bin k from Z[k] (za) and Z[nc - k] (zb), w = W_nfft^k
__device__ __forceinline__ float2 rsplit(float2 za, float2 zb, float2 w) {
  const float2 zc = make_float2(zb.x, -zb.y);
  const float2 E = make_float2(0.5f * (za.x + zc.x), 0.5f * (za.y + zc.y));
  const float2 O = mul_mi(make_float2(0.5f * (za.x - zc.x), 0.5f * (za.y - zc.y)));
  return cadd(E, cmul(w, O));
}

template <int MODE, bool GP>
__device__ __forceinline__ float rf_power(float2 x, const SpecArgs& a) {
  x.x *= a.norm_scale;
  x.y *= a.norm_scale;
  float p = x.x * x.x + x.y * x.y;
  if (GP && a.power != 1.0f) {
    if (a.power < 1.0f) p += a.eps;
    p = powf(p, a.power);
  }
  if (GP && MODE == MODE_POWER && a.log_mag) p = logf(p + a.eps);
  return p;
}

// one unit's 16 bins (m + 25 k1 and 200 - m - 25 k1, k1 = 0..7) from the
// radix-8 outputs A = Z[m + 25 .], B = Z[25 - m + 25 .]; unit 0 passes B =
// A rotated by one (Z[200 - 25 k1] = A[(8 - k1) % 8])
template <int MODE, bool GP>
__device__ __forceinline__ void rf_unit(int m, const float2 (&A)[8], const float2 (&B)[8], const float2* t2,
                                        const SpecArgs& a, float (&pw)[16]) {
#pragma unroll
  for (int k1 = 0; k1 < 8; ++k1) {
    const float2 wk = t2[m + 25 * k1];
    const float2 wr = make_float2(-wk.x, wk.y);  // W_400^(200-k) = -conj(W_400^k)
    pw[2 * k1] = rf_power<MODE, GP>(rsplit(A[k1], B[7 - k1], wk), a);
    pw[2 * k1 + 1] = rf_power<MODE, GP>(rsplit(B[7 - k1], A[k1], wr), a);
  }
}

// s_memtime marks of lane 0 of every wave (probe builds only): entry, tables,
// frames loaded, DFT-25 + twiddle, pass A, pass B, P written, end
SBK_PROBE_BUFFER(g_rf_tl, 16384, 8)
#define RF_TL(i) SBK_PROBE(if (lane == 0 && tl_row < 16384) g_rf_tl[tl_row][i] = __builtin_amdgcn_s_memtime();)

// GP: a power other than 1 or a log magnitude (the Fbank path has neither)
template <int MODE, bool GP>
__global__ void __launch_bounds__(RF_NT, SBK_RF_MINW) spec_reg_kernel(SpecArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NC = 200;
  float2* win = reinterpret_cast<float2*>(smem);  // (window[2n], window[2n+1]), n < 200
  float2* t1 = win + NC;                           // W_200^(n1 k2): [8][25]
  float2* t2 = t1 + NC;                            // W_400^k, k <= 200
  float2* fr = t2 + NC + 2;                        // per wave: 8 frame regions + a zero pad
  float* wd = reinterpret_cast<float*>(fr + RF_NW * RF_WS);   // mel weights, dense [M][RF_LW] from a 16-B aligned bin
  int* mstart = reinterpret_cast<int*>(wd + (MODE == MODE_FBANK ? a.M * RF_LW : 0));  // that aligned bin
  int* mlen_s = mstart + (MODE == MODE_FBANK ? a.M : 0);  // table stage only: mel_len, mel_off
  int* moff_s = mlen_s + (MODE == MODE_FBANK ? a.M : 0);
  __shared__ float lmax_w[RF_NW];  // table stage: per-wave max of (start & 3) + len
  __shared__ int trip_s[8];        // 16-B chunks per mel trip (16 filters; M <= 128)
  const int tid = threadIdx.x, lane = tid & 63;
  SBK_PROBE(int tl_row = blockIdx.x * RF_NW + (tid >> 6); unsigned long long tl0 = __builtin_amdgcn_s_memtime();)
  const int w = tid >> 6;
  const int nwb = (a.T + 7) >> 3;                   // 8-frame slots per utterance
  const int nblk_t = (nwb + RF_NW - 1) / RF_NW;
  const int pad = a.center ? NC : 0;
  // span of block bk for this wave: its first sample, or -1 (not staged:
  // utterance ends, other geometries, or no valid slot)
  auto span_of = [&](int bk) __attribute__((always_inline)) {
    const int bf_ = bk / nblk_t, sl = (bk - bf_ * nblk_t) * RF_NW + w;
    const int sp = sl * 8 * a.hop - pad;
    const bool ok = sl < nwb && sp >= 0 && sp + RF_SPAN <= a.S && 7 * a.hop + 2 * NC <= RF_SPAN &&
                    ((sp | a.S | a.hop) & 3) == 0 && a.wav16;
    return ok ? sp : -1;
  };
  auto fetch = [&](int bk, int sp) __attribute__((always_inline)) {
    const float* src = a.wav + (long long)(bk / nblk_t) * a.S + sp;
    float* stage = reinterpret_cast<float*>(fr + w * RF_WS);
#pragma unroll
    for (int c = 0; c < RF_SPAN / 256; ++c)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + c * 256 + lane * 4),
                                       (__attribute__((address_space(3))) void*)(stage + c * 256), 16, 0, 0);
  };
  // the first block's span is in flight under the table stage
  if (blockIdx.x < a.Bfold * nblk_t) {
    const int sp = span_of(blockIdx.x);
    if (sp >= 0) fetch(blockIdx.x, sp);
  }
  // ---- tables, once per workgroup (the only workgroup barriers; tables read
  // from global memory per use measured 75 against 47 us)
  if (tid < NC) {
    win[tid] = reinterpret_cast<const float2*>(a.window)[tid];
    const int n1 = tid / 25, k2 = tid - n1 * 25;
    t1[tid] = a.tw[n1 * k2];  // n1 k2 <= 168
  }
  for (int i = tid; i <= NC; i += RF_NT) t2[i] = a.tw2[i];
  int lw = 0;  // dense mel width (multiple of 4, <= RF_LW); 0 = a filter is wider (CSR loop from global)
  if constexpr (MODE == MODE_FBANK) {
    // Two global round trips, every load of each issued before its first use
    // (the loops that did this one dependent load at a time — the dense rows,
    // then 16 mel_start / mel_len pairs per trip from global — kept the first
    // block of every workgroup in the table stage for ~20k cycles,
    // profiles/r05am_fbank_timeline.log): the CSR arrays -> LDS with the
    // dense width as per-wave maxima (M <= 128 < RF_NT: one filter per
    // thread), then the dense rows' weights.
    static_assert(RF_NT >= 128, "one CSR entry per thread");
    {
      const int i0 = min(tid, a.M - 1);
      const int st = a.mel_start[i0], ln = a.mel_len[i0], of = a.mel_off[i0];
      if (tid < a.M) {
        mstart[tid] = st;
        mlen_s[tid] = ln;
        moff_s[tid] = of;
      }
      const float wm = wave_max(tid < a.M ? (float)((st & 3) + ln) : 0.f);
      if (lane == 0) lmax_w[tid >> 6] = wm;
    }
    __syncthreads();
    float lmf = lmax_w[0];
#pragma unroll
    for (int i = 1; i < RF_NW; ++i) lmf = fmaxf(lmf, lmax_w[i]);
    const int lm = (int)lmf;
    lw = lm <= RF_LW ? (lm + 3) & ~3 : 0;
    if (lw) {
      constexpr int UW = (128 * RF_LW + RF_NT - 1) / RF_NT;  // dense-row elements per thread (M <= 128)
      float wv[UW];
#pragma unroll
      for (int u = 0; u < UW; ++u) {  // unconditional loads (clamped index), selected after
        const int i = min(tid + u * RF_NT, a.M * RF_LW - 1);
        const int jm = i / RF_LW, c = i - jm * RF_LW, sh = mstart[jm] & 3;
        const bool in = c >= sh && c - sh < mlen_s[jm];
        const float v = a.mel_w[in ? moff_s[jm] + c - sh : 0];
        wv[u] = in ? v : 0.f;
      }
#pragma unroll
      for (int u = 0; u < UW; ++u)
        if (tid + u * RF_NT < a.M * RF_LW) wd[tid + u * RF_NT] = wv[u];
      // 16-B chunks per mel trip (filters 16 t .. 16 t + 15): the largest of
      // its filters' own counts, so a trip skips the trailing all-zero chunks
      // of the dense rows (wave-uniform), from the LDS copies
      if (tid < 8 && 16 * tid < a.M) {
        int c = 0;
        for (int jm = 16 * tid; jm < min(16 * tid + 16, a.M); ++jm) c = max(c, ((mstart[jm] & 3) + mlen_s[jm] + 3) >> 2);
        trip_s[tid] = c;
      }
    }
  }
  __syncthreads();
  SBK_PROBE(const unsigned long long tl1 = __builtin_amdgcn_s_memtime();)
  // persistent: workgroup-sized blocks of 64 frames strided over the grid
  // (the mel table is built once per workgroup)
  for (int blk = blockIdx.x; blk < a.Bfold * nblk_t; blk += gridDim.x) {
  const int bf = blk / nblk_t;
  const int slot = (blk - bf * nblk_t) * RF_NW + w;
  if (slot >= nwb) continue;
  // the lane's frame / column from an opaque lane id, per block: hoisted out
  // of the block loop, every lane-dependent LDS address would stay live
  // through it (spills)
  int ln;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
  const int q = ln >> 3, j = ln & 7;
  const int t0 = slot * 8;
  SBK_PROBE(tl_row = blk * RF_NW + w; if (lane == 0 && tl_row < 16384) { g_rf_tl[tl_row][0] = tl0; g_rf_tl[tl_row][1] = tl1; })
  SBK_PROBE(tl0 = __builtin_amdgcn_s_memtime();)
  const int tf = min(t0 + q, a.T - 1);              // frames past T recompute the last one
  const float* wrow = a.wav + (long long)bf * a.S;

  // ---- z[n2] = windowed (x[2n], x[2n+1]), n = 8 n2 + j
  float2 z[25];
  {
    const int s0 = tf * a.hop - pad + 2 * j;
    const int span0 = span_of(blk);  // first sample of the wave's 8 frames, or -1
    if (span0 >= 0) {
      // the wave's samples (one contiguous span) -> its frame regions by
      // LDS-DMA: RF_SPAN / 256 16-B pieces per lane instead of 25 strided
      // 8-B loads per lane (the vector-memory address rate, not HBM, set the
      // load phase); the frames then read their z pairs from LDS.  The first
      // block's span was issued before the table stage.
      const float* stage = reinterpret_cast<const float*>(fr + w * RF_WS);
      if (blk != blockIdx.x) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the last block's LDS reads are done
        fetch(blk, span0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const float2* src = reinterpret_cast<const float2*>(stage + (tf - t0) * a.hop + 2 * j);
#pragma unroll
      for (int n2 = 0; n2 < 25; ++n2) z[n2] = src[8 * n2];
    } else {  // utterance ends (padding), other geometries
#pragma unroll
      for (int n2 = 0; n2 < 25; ++n2) {
        bool ok0, ok1;
        const int p0 = map_pos(s0 + 16 * n2, a.S, a.pad_mode, &ok0);
        const int p1 = map_pos(s0 + 16 * n2 + 1, a.S, a.pad_mode, &ok1);
        z[n2] = make_float2(ok0 ? wrow[p0] : 0.f, ok1 ? wrow[p1] : 0.f);
      }
    }
#pragma unroll
    for (int n2 = 0; n2 < 25; ++n2) {
      const float2 wv = win[8 * n2 + j];
      z[n2] = make_float2(z[n2].x * wv.x, z[n2].y * wv.y);
    }
  }
  SBK_PROBE(asm volatile("s_waitcnt vmcnt(0)" ::: "memory");)
  RF_TL(2);
  dft25(z);
#pragma unroll
  for (int k2 = 1; k2 < 25; ++k2) z[k2] = cmul(z[k2], t1[j * 25 + k2]);
  RF_TL(3);

  // ---- transposition through the frame's LDS region in two passes of
  // 13 / 12 k2 rows: pass A holds k2 0..6 and 19..24 (units 0..6 on lanes
  // 0..6), pass B k2 7..18 (units 7..12 on lanes 0..5).  Each pass reads all
  // its rows before anything overwrites them; the powers wait in VGPRs.
  float2* reg = fr + w * RF_WS + q * RF_FS;
  float pa[16], pb[16];
  const int ma = min(j, 6), mb = 7 + min(j, 5);
  {
#pragma unroll
    for (int k2 = 0; k2 < 7; ++k2) reg[k2 * 8 + j] = z[k2];
#pragma unroll
    for (int k2 = 19; k2 < 25; ++k2) reg[(k2 - 12) * 8 + j] = z[k2];
    float2 A[8], B[8];
    const int rb = ma ? 13 - ma : 0;  // row of k2 = 25 - ma
#pragma unroll
    for (int n1 = 0; n1 < 8; ++n1) {
      A[n1] = reg[ma * 8 + n1];
      B[n1] = reg[rb * 8 + n1];
    }
    asm volatile("" ::: "memory");  // pass B's row writes stay behind these reads
    dft_small<8>(A);
    dft_small<8>(B);
    if (ma == 0) {
#pragma unroll
      for (int n = 0; n < 8; ++n) B[n] = A[(n + 1) & 7];
    }
    rf_unit<MODE, GP>(ma, A, B, t2, a, pa);
  }
  RF_TL(4);
  {
#pragma unroll
    for (int k2 = 7; k2 < 19; ++k2) reg[(k2 - 7) * 8 + j] = z[k2];
    float2 A[8], B[8];
#pragma unroll
    for (int n1 = 0; n1 < 8; ++n1) {
      A[n1] = reg[(mb - 7) * 8 + n1];
      B[n1] = reg[(18 - mb) * 8 + n1];
    }
    asm volatile("" ::: "memory");  // the P writes stay behind these reads
    dft_small<8>(A);
    dft_small<8>(B);
    rf_unit<MODE, GP>(mb, A, B, t2, a, pb);
  }
  RF_TL(5);
  const bool wa = j <= 6, wb = j <= 5;  // lanes with a unit of their own in pass A / B
  if constexpr (MODE == MODE_POWER) {
    if (t0 + q < a.T) {
      float* orow = a.out + bf * a.os_b + (long long)(t0 + q) * a.os_t;
#pragma unroll
      for (int k1 = 0; k1 < 8; ++k1) {
        if (wa) {
          orow[(ma + 25 * k1) * a.os_k] = pa[2 * k1];
          orow[(NC - ma - 25 * k1) * a.os_k] = pa[2 * k1 + 1];
        }
        if (wb) {
          orow[(mb + 25 * k1) * a.os_k] = pb[2 * k1];
          orow[(NC - mb - 25 * k1) * a.os_k] = pb[2 * k1 + 1];
        }
      }
    }
  } else {
    // |X|^2 -> P (the frame's region, over its consumed rows)
    float* P = reinterpret_cast<float*>(reg);
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) {
      if (wa) {
        P[ma + 25 * k1] = pa[2 * k1];
        P[NC - ma - 25 * k1] = pa[2 * k1 + 1];
      }
      if (wb) {
        P[mb + 25 * k1] = pb[2 * k1];
        P[NC - mb - 25 * k1] = pb[2 * k1 + 1];
      }
    }
    // the wave's pad (the dense mel reads run up to RF_LW - 1 bins past a
    // filter's start): finite zeros
    if (lane < 2 * RF_PAD) reinterpret_cast<float*>(fr + w * RF_WS + 8 * RF_FS)[lane] = 0.f;
    RF_TL(6);
    // ---- mel + dB: lane -> (filter jm, frame f) of this wave's frames
    float lmax = -INFINITY;
    const float* P0 = reinterpret_cast<const float*>(fr + w * RF_WS);
    float* obase = a.out + ((long long)bf * a.T + t0) * a.M;
    const int f = lane & 7;  // the lane's frame; filters jm = lane / 8 + 8 i
    auto mel = [&](int jm, int nch) __attribute__((always_inline)) {
      float acc = 0.f;
      if (lw) {
        // dense rows from the filter's 16-B aligned first bin, zero weights
        // outside it: 16-B reads of P and weights, lw / 4 of each
        const rf4* pf = reinterpret_cast<const rf4*>(P0 + f * (2 * RF_FS) + (mstart[jm] & ~3));
        const rf4* wq = reinterpret_cast<const rf4*>(wd + jm * RF_LW);
#pragma unroll
        for (int c = 0; c < RF_LW / 4; ++c) {
          if (c < nch) {
            const rf4 pv = pf[c], wv = wq[c];
            acc = fmaf(pv[0], wv[0], acc);
            acc = fmaf(pv[1], wv[1], acc);
            acc = fmaf(pv[2], wv[2], acc);
            acc = fmaf(pv[3], wv[3], acc);
          }
        }
      } else {
        const float* pf = P0 + f * (2 * RF_FS) + a.mel_start[jm];
        const float* wq = a.mel_w + a.mel_off[jm];
        const int L = a.mel_len[jm];
        for (int i = 0; i < L; ++i) acc = fmaf(pf[i], wq[i], acc);
      }
      return acc;
    };
    auto emit = [&](int jm, float acc) __attribute__((always_inline)) {
      if (t0 + f < a.T) {
        if (a.log_mel) {
          acc = to_db(acc, a.amin, a.amin_db, a.multiplier, a.db_offset);
          lmax = fmaxf(lmax, acc);
        }
        obase[f * a.M + jm] = acc;
      }
    };
    // two filters per trip: their LDS round trips overlap
    // (chunk count per trip from the table stage)
    auto trip_ch = [&](int t) __attribute__((always_inline)) {
      return lw ? __builtin_amdgcn_readfirstlane(trip_s[t]) : 0;
    };
    int jm = lane >> 3;
    for (; jm + 8 < a.M; jm += 16) {
      const int nch = trip_ch(jm >> 4);
      const float a0 = mel(jm, nch), a1 = mel(jm + 8, nch);
      emit(jm, a0);
      emit(jm + 8, a1);
    }
    if (jm < a.M) emit(jm, mel(jm, trip_ch(jm >> 4)));
    if (a.log_mel) {
      lmax = wave_max(lmax);
      if (lane == 0) a.slot_max[(long long)bf * nwb + slot] = lmax;
    }
  }
  SBK_PROBE(asm volatile("s_waitcnt vmcnt(0)" ::: "memory");)
  RF_TL(7);
  }  // blk
}

size_t reg_lds(int mode, int M) {
  return (size_t)(3 * 200 + 2 + RF_NW * RF_WS) * sizeof(float2) +
         (mode == MODE_FBANK ? (size_t)M * (RF_LW + 3) * 4 : 0);
}
// the register-FFT kernel takes n_fft 400 mono power / Fbank
bool use_reg(int nc, int mode, int C, int M) {
  return nc == 200 && C == 1 && (mode == MODE_POWER || (mode == MODE_FBANK && M <= 128));
}

template <int NC> struct StaticCfg;
template <> struct StaticCfg<200> { static constexpr int FPB = 8, NT = 320; };
template <> struct StaticCfg<256> { static constexpr int FPB = 8, NT = 256; };
template <> struct StaticCfg<512> { static constexpr int FPB = 4, NT = 256; };
template <> struct StaticCfg<1024> { static constexpr int FPB = 2, NT = 256; };

template <int NC>
size_t static_lds(int mode, int M, int n_melw) {
  constexpr int FPB = StaticCfg<NC>::FPB;
  return (size_t)FPB * frame_stride(NC) * sizeof(float2) + (mode == MODE_FBANK ? (size_t)FPB * (NC + 1) * 4 : 0) +
         (size_t)(4 * NC + 2 + 3 * M + n_melw) * 4;
}

template <int MODE, int NC>
void launch_static(int nblk_rows, hipStream_t s, const SpecArgs& a) {
  constexpr int FPB = StaticCfg<NC>::FPB, NT = StaticCfg<NC>::NT;
  const int nblk = nblk_rows * ((a.T + FPB - 1) / FPB);
  hipLaunchKernelGGL((spec_static_kernel<MODE, NC, FPB, NT>), dim3(nblk), dim3(NT),
                     static_lds<NC>(MODE, a.M, a.n_melw), s, a);
}

// Static-plan FFT sizes (n_fft 400 / 512 / 1024 / 2048); 0 = runtime plan.
int static_nc(int nc, int mode, int onesided) {
  if (mode == MODE_STFT && !onesided) return 0;
  return (nc == 200 || nc == 256 || nc == 512 || nc == 1024) ? nc : 0;
}
int static_fpb(int nc) {
  switch (nc) {
    case 200: return StaticCfg<200>::FPB;
    case 256: return StaticCfg<256>::FPB;
    case 512: return StaticCfg<512>::FPB;
    default: return StaticCfg<1024>::FPB;
  }
}
size_t static_lds_for(int nc, int mode, int M, int n_melw) {
  switch (nc) {
    case 200: return static_lds<200>(mode, M, n_melw);
    case 256: return static_lds<256>(mode, M, n_melw);
    case 512: return static_lds<512>(mode, M, n_melw);
    default: return static_lds<1024>(mode, M, n_melw);
  }
}

template <int MODE>
void launch_static_m(int nc, int rows, hipStream_t s, const SpecArgs& a) {
  switch (nc) {
    case 200: launch_static<MODE, 200>(rows, s, a); break;
    case 256: launch_static<MODE, 256>(rows, s, a); break;
    case 512: launch_static<MODE, 512>(rows, s, a); break;
    default: launch_static<MODE, 1024>(rows, s, a); break;
  }
}

int launch_spec(int mode, int nc, int rows, size_t lds, hipStream_t s, const SpecArgs& a, const FftPlan& plan) {
  if (use_reg(nc, mode, a.C, a.M)) {
    const int nwb = (a.T + 7) / 8;
    static int ncu = 0;
    if (!ncu) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        ncu = 256;
    }
    const dim3 grid(std::min(rows * ((nwb + RF_NW - 1) / RF_NW), SBK_RF_WGS_PER_CU * ncu));
    const size_t rl = reg_lds(mode, a.M);
    for (const void* k : {reinterpret_cast<const void*>(&spec_reg_kernel<MODE_POWER, true>),
                          reinterpret_cast<const void*>(&spec_reg_kernel<MODE_POWER, false>),
                          reinterpret_cast<const void*>(&spec_reg_kernel<MODE_FBANK, true>),
                          reinterpret_cast<const void*>(&spec_reg_kernel<MODE_FBANK, false>)})
      if (hipError_t e = sbk::lds_optin(k, rl)) return (int)e;  // > 64 KB of dynamic LDS
    const bool gp = a.power != 1.0f || (mode == MODE_POWER && a.log_mag);
    if (mode == MODE_POWER) {
      if (gp) hipLaunchKernelGGL((spec_reg_kernel<MODE_POWER, true>), grid, dim3(RF_NT), rl, s, a);
      else hipLaunchKernelGGL((spec_reg_kernel<MODE_POWER, false>), grid, dim3(RF_NT), rl, s, a);
    } else {
      if (gp) hipLaunchKernelGGL((spec_reg_kernel<MODE_FBANK, true>), grid, dim3(RF_NT), rl, s, a);
      else hipLaunchKernelGGL((spec_reg_kernel<MODE_FBANK, false>), grid, dim3(RF_NT), rl, s, a);
    }
    return 0;
  }
  const int snc = static_nc(nc, mode, a.onesided);
  if (snc) {
    if (mode == MODE_STFT) launch_static_m<MODE_STFT>(snc, rows, s, a);
    else if (mode == MODE_POWER) launch_static_m<MODE_POWER>(snc, rows, s, a);
    else launch_static_m<MODE_FBANK>(snc, rows, s, a);
    return 0;
  }
  const dim3 grid(rows * ((a.T + a.fpb - 1) / a.fpb));
  if (mode == MODE_STFT) hipLaunchKernelGGL(spec_kernel<MODE_STFT>, grid, dim3(256), lds, s, a, plan);
  else if (mode == MODE_POWER) hipLaunchKernelGGL(spec_kernel<MODE_POWER>, grid, dim3(256), lds, s, a, plan);
  else hipLaunchKernelGGL(spec_kernel<MODE_FBANK>, grid, dim3(256), lds, s, a, plan);
  return 0;
}

inline int grid_for(long long n, int block) {
  long long g = (n + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

SBK_PROBE_EXPORT(sbk_probe_spec_tl, g_spec_tl)
SBK_PROBE_EXPORT(sbk_probe_rf_tl, g_rf_tl)

// ---------------------------------------------------------------------------
// C ABI (declared in include/sbk.h)
// ---------------------------------------------------------------------------

SBK_API int sbk_fft_supported(int n_fft) {
  FftPlan p;
  if (n_fft < 4 || (n_fft & 1)) return 0;
  return fill_plan(&p, n_fft / 2) == 0 ? 1 : 0;
}

namespace {
// Frames per spectrum workgroup: as many as fit ~72 KB of LDS (<= 16).
// LDS of a spectrum workgroup: two padded frame buffers + the tables.
size_t spec_lds(int n_fft, int M, int n_melw, int fpb) {
  const int nc = n_fft / 2, ncp = frame_stride(nc);
  return (size_t)2 * fpb * ncp * sizeof(float2) + (size_t)(2 * nc + 1) * sizeof(float2) +
         (size_t)(3 * M + n_melw) * 4;
}
// Frames per workgroup: up to 8 while the LDS stays under ~40 KB (4
// workgroups per CU), fewer for long FFTs.
int spec_fpb(int n_fft, int hop, int M, int n_melw) {
  (void)hop;
  int fpb = 8;
  while (fpb > 1 && spec_lds(n_fft, M, n_melw, fpb) > 40 * 1024) fpb >>= 1;
  return spec_lds(n_fft, M, n_melw, fpb) > 160 * 1024 ? 0 : fpb;
}
int fb_rows_per_block(int F) {
  int rpb = 8;
  while (rpb > 1 && (size_t)rpb * F * 4 > 48 * 1024) rpb >>= 1;
  return rpb;
}
}  // namespace

SBK_API int sbk_spectrum_slots(int n_fft, int hop, int T, int M, int n_melw) {
  if (n_fft < 4 || (n_fft & 1) || T <= 0) return 0;
  const int snc = static_nc(n_fft / 2, MODE_FBANK, 1);
  const int fpb = snc ? static_fpb(snc) : spec_fpb(n_fft, hop, M, n_melw);
  return fpb ? (T + fpb - 1) / fpb : 0;
}

SBK_API int sbk_filterbank_slots(int T, int F) {
  if (T <= 0 || F <= 0) return 0;
  const int rpb = fb_rows_per_block(F);
  return (T + rpb - 1) / rpb;
}

// mode 0: STFT (complex), 1: power spectrum, 2: fused Fbank (mel + dB, pre-top_db)
SBK_API int sbk_spectrum(int mode, const float* wav, int Bo, int S, int C, int n_fft, int hop, int center,
                         int pad_mode, int T, const float* window, const float* twiddle_nc,
                         const float* twiddle_nfft, int onesided, float norm_scale, float power, float eps,
                         int log_mag, const long long* out_strides, const int* mel_start, const int* mel_len,
                         const int* mel_off, const float* mel_w, int n_melw, int M, int log_mel,
                         float multiplier, float db_offset, float amin, float* out, float* slot_max, void* stream) {
  if (Bo <= 0 || T <= 0 || S <= 0 || C <= 0) return SBK_ERR_ARG;
  if (mode < MODE_STFT || mode > MODE_FBANK) return SBK_ERR_ARG;
  FftPlan plan;
  if ((n_fft & 1) || fill_plan(&plan, n_fft / 2)) return SBK_ERR_ARG;
  SpecArgs a;
  a.wav = wav; a.S = S; a.C = C; a.Bfold = Bo * C;
  a.wav16 = (reinterpret_cast<uintptr_t>(wav) & 15) == 0;  // a view at a 4-B offset takes the unstaged path
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
  a.M = mode == MODE_FBANK ? M : 0;
  a.n_melw = mode == MODE_FBANK ? n_melw : 0;
  a.log_mel = log_mel; a.multiplier = multiplier; a.db_offset = db_offset; a.amin = amin;
  a.amin_db = multiplier * (float)log10((double)amin) - db_offset;
  a.out = out; a.slot_max = slot_max;
  if (mode == MODE_FBANK && log_mel && (C != 1 || !slot_max)) return SBK_ERR_ARG;
  const int snc = static_nc(n_fft / 2, mode, onesided);
  const int fpb = snc ? static_fpb(snc) : spec_fpb(n_fft, hop, a.M, a.n_melw);
  if (!fpb) return SBK_ERR_ARG;
  if (snc && static_lds_for(snc, mode, a.M, a.n_melw) > 64 * 1024) return SBK_ERR_ARG;
  a.fpb = fpb;
  if (int rc = launch_spec(mode, n_fft / 2, a.Bfold, spec_lds(n_fft, a.M, a.n_melw, fpb), (hipStream_t)stream, a,
                           plan))
    return rc;
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_filterbank(const float* spec, int N, int T, int F, const int* mel_start, const int* mel_len,
                           const int* mel_off, const float* mel_w, const float* dense, int M, int log_mel,
                           float multiplier, float db_offset, float amin, float* out, float* slot_max,
                           void* stream) {
  if (N <= 0 || T <= 0 || F <= 0 || M <= 0) return SBK_ERR_ARG;
  if ((size_t)F * 4 > 160 * 1024) return SBK_ERR_ARG;
  if (log_mel && !slot_max) return SBK_ERR_ARG;
  FbArgs a;
  a.spec = spec; a.N = N; a.T = T; a.F = F;
  a.mel_start = mel_start; a.mel_len = mel_len; a.mel_off = mel_off; a.mel_w = mel_w; a.dense = dense;
  a.M = M; a.log_mel = log_mel; a.multiplier = multiplier; a.db_offset = db_offset; a.amin = amin;
  a.amin_db = multiplier * (float)log10((double)amin) - db_offset;
  a.out = out; a.slot_max = slot_max;
  const int rpb = fb_rows_per_block(F);
  a.rows_per_block = rpb;
  const long long nblk = (long long)N * ((T + rpb - 1) / rpb);
  hipLaunchKernelGGL(filterbank_kernel, dim3((unsigned)nblk), dim3(256), (size_t)rpb * F * 4, (hipStream_t)stream, a);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_topdb_clamp(float* x, const float* slot_max, int nslot, long long per_seq, int nseq, float top_db,
                            void* stream) {
  if (per_seq <= 0 || nseq <= 0 || nslot <= 0) return SBK_ERR_ARG;
  const long long chunk = 256 * 16;
  hipLaunchKernelGGL(topdb_clamp_kernel, dim3((unsigned)((per_seq + chunk - 1) / chunk), nseq), dim3(256), 0,
                     (hipStream_t)stream, x, slot_max, nslot, per_seq, top_db);
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

// y = [max(x, max_b - top_db) | d1 | d2] (N,T,3F): the concat deltas of an
// fbank whose top_db floor was deferred (slot_max: (N, nslot) maxima from
// sbk_spectrum).  F % 4 == 0, 16-B aligned x / y.
SBK_API int sbk_deltas_floor(const float* x, float* y, int N, int T, int F, int window_length, const float* slot_max,
                             int nslot, float top_db, void* stream) {
  if (N <= 0 || T <= 0 || F <= 0 || F % 4 || window_length < 3 || !slot_max || nslot <= 0) return SBK_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) return SBK_ERR_ARG;
  const int n = (window_length - 1) / 2;
  const float denom = (float)(n * (n + 1) * (2 * n + 1)) / 3.0f;
  // 32-row tiles: 15.1 vs 16.0 us at config 2 for 64 (26.3 for 128; storing
  // each tile's output rows as one contiguous float4 run measured 20.8-22.8:
  // profiles/r06ai_deltas_tile_ab.log)
  int ttile = 32;
  auto lds = [&](int tt) { return (size_t)(tt + 4 * n) * F * 4 * 2; };
  while (ttile > 4 && lds(ttile) > 64 * 1024) ttile >>= 1;
  if (lds(ttile) > 160 * 1024) return SBK_ERR_ARG;
  const int nblk = N * ((T + ttile - 1) / ttile);
  hipLaunchKernelGGL(deltas4_concat_kernel, dim3(nblk), dim3(256), lds(ttile), (hipStream_t)stream, x, y, N, T, F, n,
                     denom, ttile, slot_max, nslot, top_db);
  SBK_CHECK_LAUNCH();
  return 0;
}

// concat=0: y = deltas(x) (N,T,F); concat=1: y = [x | d1 | d2] (N,T,3F)
SBK_API int sbk_deltas(const float* x, float* y, int N, int T, int F, int window_length, int concat, void* stream) {
  if (N <= 0 || T <= 0 || F <= 0 || window_length < 3) return SBK_ERR_ARG;
  const int n = (window_length - 1) / 2;
  const float denom = (float)(n * (n + 1) * (2 * n + 1)) / 3.0f;
  int ttile = 32;  // as sbk_deltas_floor
  const int halo = concat ? 2 * n : n;
  auto lds = [&](int tt) { return (size_t)(tt + 2 * halo) * F * 4 * (concat ? 2 : 1); };
  while (ttile > 4 && lds(ttile) > 64 * 1024) ttile >>= 1;
  if (lds(ttile) > 160 * 1024) return SBK_ERR_ARG;
  const int nblk = N * ((T + ttile - 1) / ttile);
  if (concat && F % 4 == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0)
    hipLaunchKernelGGL(deltas4_concat_kernel, dim3(nblk), dim3(256), lds(ttile), (hipStream_t)stream, x, y, N, T, F,
                       n, denom, ttile, nullptr, 0, 0.f);
  else if (concat)
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

// ---------------------------------------------------------------------------
// Filterbank backward (freeze=False learnable filters, features.py:476-482;
// the reference gets it from autograd of matmul → clamp → log10 → amax → max)
// ---------------------------------------------------------------------------
namespace {

// Per sequence n (one 1024-thread block): xdb = to_db(x), m = max xdb,
// thr = m − top_db; count of elements at m; G = Σ g over elements the clamp
// selected (xdb < thr: g, xdb == thr: g/2 — torch.maximum splits ties).
__global__ void __launch_bounds__(1024) fb_db_stats_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                           long long per_seq, float amin, float amin_db, float mult,
                                                           float off, float top_db, float* __restrict__ stats) {
  __shared__ float red[16];
  const int n = blockIdx.x;
  const float* xs = x + (long long)n * per_seq;
  const float* gs = g + (long long)n * per_seq;
  float m = -INFINITY;
  for (long long i = threadIdx.x; i < per_seq; i += blockDim.x) m = fmaxf(m, to_db(xs[i], amin, amin_db, mult, off));
  m = block_max(m, red);
  const float thr = m - top_db;
  float cnt = 0.f, gthr = 0.f;
  for (long long i = threadIdx.x; i < per_seq; i += blockDim.x) {
    const float d = to_db(xs[i], amin, amin_db, mult, off);
    cnt += d == m ? 1.f : 0.f;
    gthr += d < thr ? gs[i] : (d == thr ? 0.5f * gs[i] : 0.f);
  }
  cnt = block_sum(cnt, red);
  gthr = block_sum(gthr, red);
  if (threadIdx.x == 0) {
    stats[3 * n] = m;
    stats[3 * n + 1] = cnt;
    stats[3 * n + 2] = gthr;
  }
}

// dx = d/dx of the dB + top_db clamp: the element's own path
// (xdb > thr: g, == thr: g/2), plus G/count at the argmax elements (amax
// backward), through log10 (g·mult / (x·ln 10)) and the amin clamp (x ≥ amin).
__global__ void __launch_bounds__(256) fb_db_bwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                        const float* __restrict__ stats, long long per_seq, int log_mel,
                                                        float amin, float amin_db, float mult, float off, float top_db,
                                                        float* __restrict__ dx) {
  const int n = blockIdx.y;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= per_seq) return;
  const long long k = (long long)n * per_seq + i;
  const float xv = x[k], gv = g[k];
  if (!log_mel) {
    dx[k] = gv;
    return;
  }
  const float m = stats[3 * n], thr = m - top_db;
  const float d = to_db(xv, amin, amin_db, mult, off);
  float gd = d > thr ? gv : (d == thr ? 0.5f * gv : 0.f);
  if (d == m) gd += stats[3 * n + 2] / stats[3 * n + 1];
  dx[k] = xv >= amin ? (gd * mult) / (xv * 2.302585093f) : 0.f;
}

// Weight gradient partials: part[c, f, j] = Σ_{r in row chunk c} spec[r, f]·dx[r, j].
// Block (4 frequency rows, chunk c); wave w owns f = 4·blockIdx.x + w, lane
// owns j = lane, lane + 64 (M ≤ 128).  Reduced over chunks by sbk_colsum.
__global__ void __launch_bounds__(256) fb_wgrad_kernel(const float* __restrict__ spec, const float* __restrict__ dx,
                                                       long long rows, int F, int M, long long rows_per_chunk,
                                                       float* __restrict__ part) {
  const int f = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const long long r0 = (long long)blockIdx.y * rows_per_chunk;
  const long long r1 = min(rows, r0 + rows_per_chunk);
  if (f >= F) return;
  float a0 = 0.f, a1 = 0.f;
  for (long long r = r0; r < r1; ++r) {
    const float sv = spec[r * F + f];
    if (lane < M) a0 = fmaf(sv, dx[r * M + lane], a0);
    if (lane + 64 < M) a1 = fmaf(sv, dx[r * M + lane + 64], a1);
  }
  float* o = part + (long long)blockIdx.y * F * M + (long long)f * M;
  if (lane < M) o[lane] = a0;
  if (lane + 64 < M) o[lane + 64] = a1;
}

}  // namespace

// dB/top_db backward of Filterbank: x = linear filterbank energies (N, per_seq)
// (recomputed with sbk_filterbank(log_mel=0)), g = dL/d(output); dx = dL/dx.
// stats: 3·N floats of workspace.
SBK_API int sbk_filterbank_db_bwd(const float* x, const float* g, int N, long long per_seq, int log_mel,
                                  float multiplier, float db_offset, float amin, float top_db, float* stats, float* dx,
                                  void* stream) {
  if (N <= 0 || per_seq <= 0 || (log_mel && !stats)) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const float amin_db = multiplier * (float)log10((double)amin) - db_offset;
  if (log_mel) {
    hipLaunchKernelGGL(fb_db_stats_kernel, dim3(N), dim3(1024), 0, s, x, g, per_seq, amin, amin_db, multiplier,
                       db_offset, top_db, stats);
    SBK_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(fb_db_bwd_kernel, dim3((unsigned)((per_seq + 255) / 256), N), dim3(256), 0, s, x, g, stats,
                     per_seq, log_mel, amin, amin_db, multiplier, db_offset, top_db, dx);
  SBK_CHECK_LAUNCH();
  return 0;
}

// Partial weight gradient of the dense filter matrix: part (nchunk, F, M)
// with nchunk = ceil(rows / rows_per_chunk); sum with sbk_colsum.
SBK_API int sbk_filterbank_wgrad(const float* spec, const float* dx, long long rows, int F, int M,
                                 long long rows_per_chunk, float* part, void* stream) {
  if (rows <= 0 || F <= 0 || M <= 0 || M > 128 || rows_per_chunk <= 0) return SBK_ERR_ARG;
  const long long nchunk = (rows + rows_per_chunk - 1) / rows_per_chunk;
  hipLaunchKernelGGL(fb_wgrad_kernel, dim3((unsigned)((F + 3) / 4), (unsigned)nchunk), dim3(256), 0,
                     (hipStream_t)stream, spec, dx, rows, F, M, rows_per_chunk, part);
  SBK_CHECK_LAUNCH();
  return 0;
}
