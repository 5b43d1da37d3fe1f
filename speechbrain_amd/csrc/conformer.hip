// Conformer encoder support kernels: LayerNorm (single or chained pair),
// fused depthwise conv + LayerNorm + Swish, ConvolutionFrontEnd blocks
// (3x3 stride-2 reflect-padded Conv2d + LayerNorm(freq x channels) +
// LeakyReLU), bf16 casts.
//
// Reference semantics:
//   LayerNorm           nn.LayerNorm via speechbrain/nnet/normalization.py:172-223
//   ConvolutionModule   speechbrain/lobes/models/transformer/Conformer.py:101-115
//                       (depthwise Conv1d k, pad (k-1)/2 or causal chomp,
//                        after_conv = LayerNorm -> Swish -> Linear)
//   ConvBlock           speechbrain/lobes/models/convolution.py:112-175 with
//                       Conv2d "same" reflect padding speechbrain/nnet/CNN.py:616-700
#include "mfma.h"

using namespace sbk;

namespace {

template <typename T>
__device__ __forceinline__ float ld(const T* p, long long i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, long long i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, long long i) { return bf16_to_f32(p[i]); }

__device__ __forceinline__ void st(void* p, long long i, float v, int bf) {
  if (bf)
    reinterpret_cast<bf16_t*>(p)[i] = f32_to_bf16(v);
  else
    reinterpret_cast<float*>(p)[i] = v;
}

// One wave per row.  y1 = LN1(x) (written to out1 if non-null);
// if g2: y2 = LN2(y1) written to out2.  Rows up to D = 64 * 16 elements.
template <int PER>
__global__ void __launch_bounds__(256) layernorm_kernel(const float* __restrict__ x, int M, int D,
                                                        const float* g1, const float* b1, float eps1, void* out1,
                                                        int out1_bf16, const float* g2, const float* b2,
                                                        float eps2, void* out2, int out2_bf16) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* xr = x + row * D;
  float v[PER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < D ? xr[c] : 0.f;
    s += v[i];
  }
  float mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    const float d = c < D ? v[i] - mean : 0.f;
    q += d * d;
  }
  float rstd = 1.0f / sqrtf(wave_sum(q) / D + eps1);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    if (c < D) {
      v[i] = (v[i] - mean) * rstd * g1[c] + b1[c];
      if (out1) st(out1, row * D + c, v[i], out1_bf16);
    }
  }
  if (!g2) return;
  s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) s += (lane + 64 * i) < D ? v[i] : 0.f;
  mean = wave_sum(s) / D;
  q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    const float d = c < D ? v[i] - mean : 0.f;
    q += d * d;
  }
  rstd = 1.0f / sqrtf(wave_sum(q) / D + eps2);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    if (c < D) st(out2, row * D + c, (v[i] - mean) * rstd * g2[c] + b2[c], out2_bf16);
  }
}

// Depthwise Conv1d over time (zero padding padL left / K-1-padL right)
// + bias -> LayerNorm over channels -> Swish.  x: (B, T, C) T-typed.
// Block = TT timesteps of one sequence.  Phase 1: one thread per channel
// keeps its K taps and its (TT + K - 1)-sample input window in registers
// (K, TT compile-time) and writes TT conv outputs to LDS; phase 2: one wave
// per timestep normalises across channels and applies Swish.
template <typename T, int K, int TT>
__global__ void __launch_bounds__(256) dwconv_ln_swish_kernel(const T* __restrict__ x, int B, int Tn, int C,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ bias, int padL,
                                                              const float* __restrict__ g,
                                                              const float* __restrict__ beta, float eps, void* out,
                                                              int out_bf16) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* cv = reinterpret_cast<float*>(smem);  // TT x C
  const int ntile = (Tn + TT - 1) / TT;
  const int b = blockIdx.x / ntile;
  const int t0 = (blockIdx.x - b * ntile) * TT;
  const int nt = min(TT, Tn - t0);
  const T* xb = x + (long long)b * Tn * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float wk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) wk[k] = w[c * K + k];
    float win[TT + K - 1];
#pragma unroll
    for (int r = 0; r < TT + K - 1; ++r) {
      const int t = t0 - padL + r;
      win[r] = (t >= 0 && t < Tn) ? ld(xb, (long long)t * C + c) : 0.f;
    }
    const float bc = bias ? bias[c] : 0.f;
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      float acc = bc;
#pragma unroll
      for (int k = 0; k < K; ++k) acc = fmaf(wk[k], win[tt + k], acc);
      cv[tt * C + c] = acc;
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int tt = wid; tt < nt; tt += 4) {
    const float* r = cv + tt * C;
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += r[c];
    const float mean = wave_sum(s) / C;
    float q = 0.f;
    for (int c = lane; c < C; c += 64) {
      const float d = r[c] - mean;
      q += d * d;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / C + eps);
    const long long ob = ((long long)b * Tn + t0 + tt) * C;
    for (int c = lane; c < C; c += 64) {
      float y = (r[c] - mean) * rstd * g[c] + beta[c];
      y = y * (1.0f / (1.0f + expf(-y)));
      st(out, ob + c, y, out_bf16);
    }
  }
}

// Generic-K fallback: input rows staged in LDS, taps read per channel.
template <typename T>
__global__ void __launch_bounds__(256) dwconv_ln_swish_generic(const T* __restrict__ x, int B, int Tn, int C,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ bias, int K, int padL,
                                                               const float* __restrict__ g,
                                                               const float* __restrict__ beta, float eps, void* out,
                                                               int out_bf16, int TT) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* xin = reinterpret_cast<float*>(smem);  // (TT + K - 1) x C
  float* cv = xin + (TT + K - 1) * C;          // TT x C
  const int ntile = (Tn + TT - 1) / TT;
  const int b = blockIdx.x / ntile;
  const int t0 = (blockIdx.x - b * ntile) * TT;
  const int nt = min(TT, Tn - t0);
  const int rows = nt + K - 1;
  const T* xb = x + (long long)b * Tn * C;
  for (int i = threadIdx.x; i < rows * C; i += blockDim.x) {
    const int r = i / C, c = i - r * C;
    const int t = t0 - padL + r;
    xin[i] = (t >= 0 && t < Tn) ? ld(xb, (long long)t * C + c) : 0.f;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float* wc = w + c * K;
    const float bc = bias ? bias[c] : 0.f;
    for (int tt = 0; tt < nt; ++tt) {
      float acc = bc;
      for (int k = 0; k < K; ++k) acc = fmaf(wc[k], xin[(tt + k) * C + c], acc);
      cv[tt * C + c] = acc;
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int tt = wid; tt < nt; tt += 4) {
    const float* r = cv + tt * C;
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += r[c];
    const float mean = wave_sum(s) / C;
    float q = 0.f;
    for (int c = lane; c < C; c += 64) {
      const float d = r[c] - mean;
      q += d * d;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / C + eps);
    const long long ob = ((long long)b * Tn + t0 + tt) * C;
    for (int c = lane; c < C; c += 64) {
      float y = (r[c] - mean) * rstd * g[c] + beta[c];
      y = y * (1.0f / (1.0f + expf(-y)));
      st(out, ob + c, y, out_bf16);
    }
  }
}

__device__ __forceinline__ int reflect_idx(int i, int n) {
  if (i < 0) i = -i;
  if (i >= n) i = 2 * (n - 1) - i;
  return i;
}

// ConvBlock with Cin == 1: x (B, Tin, Fin) fp32 -> y (B, Tout, Fout, Cout)
// Conv2d(k3, s2, reflect pad 1) over (freq, time) + LayerNorm(Fout*Cout) + LeakyReLU.
// One block per (b, t_out).  w: (Cout, 1, 3(freq), 3(time)).
__global__ void __launch_bounds__(256) conv_block_c1_kernel(const float* __restrict__ x, int B, int Tin, int Fin,
                                                            int Tout, int Fout, int Cout,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ g,
                                                            const float* __restrict__ beta, float eps, float slope,
                                                            void* out, int out_bf16) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* xin = reinterpret_cast<float*>(smem);  // 3 x Fin
  float* yv = xin + 3 * Fin;                     // Fout * Cout
  __shared__ float red[16];
  const int b = blockIdx.x / Tout, to = blockIdx.x - b * Tout;
  for (int i = threadIdx.x; i < 3 * Fin; i += blockDim.x) {
    const int kt = i / Fin, f = i - kt * Fin;
    const int ti = reflect_idx(2 * to - 1 + kt, Tin);
    xin[i] = x[((long long)b * Tin + ti) * Fin + f];
  }
  __syncthreads();
  const int nout = Fout * Cout;
  float s = 0.f;
  for (int o = threadIdx.x; o < nout; o += blockDim.x) {
    const int fo = o / Cout, co = o - fo * Cout;
    const float* wc = w + co * 9;
    float acc = bias ? bias[co] : 0.f;
#pragma unroll
    for (int kf = 0; kf < 3; ++kf) {
      const int fi = reflect_idx(2 * fo - 1 + kf, Fin);
#pragma unroll
      for (int kt = 0; kt < 3; ++kt) acc = fmaf(wc[kf * 3 + kt], xin[kt * Fin + fi], acc);
    }
    yv[o] = acc;
    s += acc;
  }
  const float mean = block_sum(s, red) / nout;
  float q = 0.f;
  for (int o = threadIdx.x; o < nout; o += blockDim.x) {
    const float d = yv[o] - mean;
    q += d * d;
  }
  const float rstd = 1.0f / sqrtf(block_sum(q, red) / nout + eps);
  const long long ob = ((long long)b * Tout + to) * nout;
  for (int o = threadIdx.x; o < nout; o += blockDim.x) {
    float y = (yv[o] - mean) * rstd * g[o] + beta[o];
    y = y >= 0.f ? y : y * slope;
    st(out, ob + o, y, out_bf16);
  }
}

// ConvBlock with Cin % 8 == 0 as an implicit GEMM on MFMA.
// x: (B, Tin, Fin, Cin) T-typed; wp: weights pre-permuted to
// (Cout, 3(time), 3(freq), Cin) in T; y: (B, Tout, Fout*Cout).
// Per block (b, t_out): M = Fout (padded to 16s), N = Cout, K = 9*Cin.
template <typename T>
__global__ void __launch_bounds__(256) conv_block_mfma_kernel(const T* __restrict__ x, int B, int Tin, int Fin,
                                                              int Cin, int Tout, int Fout, int Cout,
                                                              const T* __restrict__ wp,
                                                              const float* __restrict__ bias,
                                                              const float* __restrict__ g,
                                                              const float* __restrict__ beta, float eps, float slope,
                                                              void* out, int out_bf16) {
  using Tr = MT<T>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* xin = reinterpret_cast<T*>(smem);                       // 3 x Fin x Cin
  float* yv = reinterpret_cast<float*>(smem + (((size_t)3 * Fin * Cin * sizeof(T) + 15) & ~(size_t)15));
  __shared__ float red[16];
  const int b = blockIdx.x / Tout, to = blockIdx.x - b * Tout;
  const int rowlen = Fin * Cin;
  constexpr int VEC = Tr::VEC;
  for (int i = threadIdx.x; i < 3 * rowlen / VEC; i += blockDim.x) {
    const int kt = (i * VEC) / rowlen, off = i * VEC - kt * rowlen;
    const int ti = reflect_idx(2 * to - 1 + kt, Tin);
    *reinterpret_cast<uint4*>(xin + kt * rowlen + off) =
        *reinterpret_cast<const uint4*>(x + ((long long)b * Tin + ti) * rowlen + off);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int mt = (Fout + 15) / 16, ntl = Cout / 16;
  const int K = 9 * Cin;
  const int fk = 8 * (lane >> 4), fr = lane & 15;
  for (int tile = wid; tile < mt * ntl; tile += 4) {
    const int tm = tile / ntl, tn = tile - tm * ntl;
    const int fo = tm * 16 + fr;  // A row (output freq) this lane loads
    const int co = tn * 16 + fr;  // B col (output channel) this lane loads
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < K; k0 += 32) {
      const int k = k0 + fk;             // 8 consecutive k: same (kt, kf), ci .. ci+7
      const int kt = k / (3 * Cin), rem = k - kt * 3 * Cin;
      const int kf = rem / Cin, ci = rem - kf * Cin;
      typename Tr::frag fa, fb;
      if (fo < Fout && k < K) {
        const int fi = reflect_idx(2 * fo - 1 + kf, Fin);
        fa = Tr::load(xin + kt * rowlen + fi * Cin + ci);
      } else {
        fa = Tr::zero();
      }
      fb = k < K ? Tr::load(wp + (long long)co * K + k) : Tr::zero();
      Tr::mma(acc, fa, fb);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = tm * 16 + 4 * (lane >> 4) + r;
      const int c = tn * 16 + fr;
      if (f < Fout) yv[f * Cout + c] = acc[r] + (bias ? bias[c] : 0.f);
    }
  }
  __syncthreads();
  const int nout = Fout * Cout;
  float s = 0.f;
  for (int o = threadIdx.x; o < nout; o += blockDim.x) s += yv[o];
  const float mean = block_sum(s, red) / nout;
  float q = 0.f;
  for (int o = threadIdx.x; o < nout; o += blockDim.x) {
    const float d = yv[o] - mean;
    q += d * d;
  }
  const float rstd = 1.0f / sqrtf(block_sum(q, red) / nout + eps);
  const long long ob = ((long long)b * Tout + to) * nout;
  for (int o = threadIdx.x; o < nout; o += blockDim.x) {
    float y = (yv[o] - mean) * rstd * g[o] + beta[o];
    y = y >= 0.f ? y : y * slope;
    st(out, ob + o, y, out_bf16);
  }
}

__global__ void cast_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] = f32_to_bf16(x[i]);
}

__global__ void swish_kernel(const float* __restrict__ x, float* __restrict__ y, long long n, float beta) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float v = x[i];
    y[i] = v * (1.0f / (1.0f + expf(-beta * v)));
  }
}

inline int grid_for(long long n, int block) {
  long long g = (n + block - 1) / block;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

SBK_API int sbk_layernorm(const float* x, int M, int D, const float* g1, const float* b1, float eps1, void* out1,
                          int out1_bf16, const float* g2, const float* b2, float eps2, void* out2, int out2_bf16,
                          void* stream) {
  if (M <= 0 || D <= 0 || D > 1024) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((M + 3) / 4);
#define SBK_LN(P)                                                                                       \
  hipLaunchKernelGGL(layernorm_kernel<P>, grid, dim3(256), 0, s, x, M, D, g1, b1, eps1, out1, out1_bf16, g2, \
                     b2, eps2, out2, out2_bf16)
  if (D <= 64) SBK_LN(1);
  else if (D <= 128) SBK_LN(2);
  else if (D <= 256) SBK_LN(4);
  else if (D <= 512) SBK_LN(8);
  else SBK_LN(16);
#undef SBK_LN
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_dwconv_ln_swish(int in_bf16, const void* x, int B, int Tn, int C, const float* w, const float* bias,
                                int K, int causal, const float* g, const float* beta, float eps, void* out,
                                int out_bf16, void* stream) {
  if (B <= 0 || Tn <= 0 || C <= 0 || K <= 0) return SBK_ERR_ARG;
  const int padL = causal ? K - 1 : (K - 1) / 2;
  hipStream_t s = (hipStream_t)stream;
  if (K == 31 && (size_t)16 * C * 4 <= 64 * 1024) {
    constexpr int TT = 16;
    const int grid = B * ((Tn + TT - 1) / TT);
    const size_t lds = (size_t)TT * C * 4;
    if (in_bf16)
      hipLaunchKernelGGL((dwconv_ln_swish_kernel<bf16_t, 31, TT>), dim3(grid), dim3(256), lds, s,
                         reinterpret_cast<const bf16_t*>(x), B, Tn, C, w, bias, padL, g, beta, eps, out, out_bf16);
    else
      hipLaunchKernelGGL((dwconv_ln_swish_kernel<float, 31, TT>), dim3(grid), dim3(256), lds, s,
                         reinterpret_cast<const float*>(x), B, Tn, C, w, bias, padL, g, beta, eps, out, out_bf16);
    SBK_CHECK_LAUNCH();
    return 0;
  }
  int TT = 16;
  auto lds = [&](int tt) { return (size_t)((tt + K - 1) + tt) * C * 4; };
  while (TT > 1 && lds(TT) > 64 * 1024) TT >>= 1;
  if (lds(TT) > 160 * 1024) return SBK_ERR_ARG;
  const int grid = B * ((Tn + TT - 1) / TT);
  if (in_bf16)
    hipLaunchKernelGGL(dwconv_ln_swish_generic<bf16_t>, dim3(grid), dim3(256), lds(TT), s,
                       reinterpret_cast<const bf16_t*>(x), B, Tn, C, w, bias, K, padL, g, beta, eps, out, out_bf16, TT);
  else
    hipLaunchKernelGGL(dwconv_ln_swish_generic<float>, dim3(grid), dim3(256), lds(TT), s,
                       reinterpret_cast<const float*>(x), B, Tn, C, w, bias, K, padL, g, beta, eps, out, out_bf16, TT);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_conv_block_c1(const float* x, int B, int Tin, int Fin, int Cout, const float* w, const float* bias,
                              const float* g, const float* beta, float eps, float slope, void* out, int out_bf16,
                              int* Tout_, int* Fout_, void* stream) {
  if (B <= 0 || Tin < 2 || Fin < 2 || Cout <= 0) return SBK_ERR_ARG;
  const int Tout = (Tin + 2 - 3) / 2 + 1, Fout = (Fin + 2 - 3) / 2 + 1;
  if (Tout_) *Tout_ = Tout;
  if (Fout_) *Fout_ = Fout;
  if (!x) return 0;  // shape query
  const size_t lds = (size_t)(3 * Fin + Fout * Cout) * 4;
  if (lds > 160 * 1024) return SBK_ERR_ARG;
  hipLaunchKernelGGL(conv_block_c1_kernel, dim3(B * Tout), dim3(256), lds, (hipStream_t)stream, x, B, Tin, Fin, Tout,
                     Fout, Cout, w, bias, g, beta, eps, slope, out, out_bf16);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_conv_block_mfma(int in_bf16, const void* x, int B, int Tin, int Fin, int Cin, int Cout,
                                const void* wperm, const float* bias, const float* g, const float* beta, float eps,
                                float slope, void* out, int out_bf16, int* Tout_, int* Fout_, void* stream) {
  if (B <= 0 || Tin < 2 || Fin < 2 || (Cin % 8) || (Cout % 16)) return SBK_ERR_ARG;
  const int Tout = (Tin + 2 - 3) / 2 + 1, Fout = (Fin + 2 - 3) / 2 + 1;
  if (Tout_) *Tout_ = Tout;
  if (Fout_) *Fout_ = Fout;
  if (!x) return 0;
  const size_t esz = in_bf16 ? 2 : 4;
  const size_t lds = (((size_t)3 * Fin * Cin * esz + 15) & ~(size_t)15) + (size_t)Fout * Cout * 4;
  if (lds > 160 * 1024) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (in_bf16)
    hipLaunchKernelGGL(conv_block_mfma_kernel<bf16_t>, dim3(B * Tout), dim3(256), lds, s,
                       reinterpret_cast<const bf16_t*>(x), B, Tin, Fin, Cin, Tout, Fout, Cout,
                       reinterpret_cast<const bf16_t*>(wperm), bias, g, beta, eps, slope, out, out_bf16);
  else
    hipLaunchKernelGGL(conv_block_mfma_kernel<float>, dim3(B * Tout), dim3(256), lds, s,
                       reinterpret_cast<const float*>(x), B, Tin, Fin, Cin, Tout, Fout, Cout,
                       reinterpret_cast<const float*>(wperm), bias, g, beta, eps, slope, out, out_bf16);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_cast_bf16(const float* x, void* y, long long n, void* stream) {
  if (n <= 0) return SBK_ERR_ARG;
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, x,
                     reinterpret_cast<bf16_t*>(y), n);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_swish(const float* x, float* y, long long n, float beta, void* stream) {
  if (n <= 0) return SBK_ERR_ARG;
  hipLaunchKernelGGL(swish_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, x, y, n, beta);
  SBK_CHECK_LAUNCH();
  return 0;
}
