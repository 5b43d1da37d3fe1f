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

#include <algorithm>
#include <utility>

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
// D == 256 rows: lane l owns columns 4l .. 4l+3 (16-B loads, 8-/16-B
// stores), a wave normalises RPW rows with every load issued up front and the
// RPW reductions interleaved.  Same arithmetic as layernorm_kernel.
template <int RPW>
__global__ void __launch_bounds__(256) layernorm256_kernel(const float* __restrict__ x, int M,
                                                           const float* __restrict__ g1, const float* __restrict__ b1,
                                                           float eps1, void* out1, int out1_bf16,
                                                           const float* __restrict__ g2,
                                                           const float* __restrict__ b2, float eps2, void* out2,
                                                           int out2_bf16) {
  constexpr int D = 256;
  const int lane = threadIdx.x & 63;
  const long long row0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  float v[RPW][4], sm[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const long long row = min(row0 + r, (long long)M - 1);
    const float4 t = *reinterpret_cast<const float4*>(x + row * D + 4 * lane);
    v[r][0] = t.x; v[r][1] = t.y; v[r][2] = t.z; v[r][3] = t.w;
  }
  auto norm = [&](const float* g, const float* b, float eps) __attribute__((always_inline)) {
    const float4 g4 = *reinterpret_cast<const float4*>(g + 4 * lane);
    const float4 b4 = *reinterpret_cast<const float4*>(b + 4 * lane);
    const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
    for (int r = 0; r < RPW; ++r) sm[r] = v[r][0] + v[r][1] + v[r][2] + v[r][3];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
      for (int r = 0; r < RPW; ++r) sm[r] += __shfl_xor(sm[r], o);
    float sq[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      sm[r] *= 1.0f / D;
      sq[r] = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) sq[r] += (v[r][e] - sm[r]) * (v[r][e] - sm[r]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
      for (int r = 0; r < RPW; ++r) sq[r] += __shfl_xor(sq[r], o);
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const float rstd = 1.0f / sqrtf(sq[r] * (1.0f / D) + eps);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[r][e] = (v[r][e] - sm[r]) * rstd * gg[e] + bb[e];
    }
  };
  auto store = [&](void* out, int bf) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const long long row = row0 + r;
      if (row >= M) continue;
      if (bf) {
        uint2 pk;
        pk.x = pack_bf16x2(v[r][0], v[r][1]);
        pk.y = pack_bf16x2(v[r][2], v[r][3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(out) + row * D + 4 * lane) = pk;
      } else {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + row * D + 4 * lane) =
            make_float4(v[r][0], v[r][1], v[r][2], v[r][3]);
      }
    }
  };
  norm(g1, b1, eps1);
  if (out1) store(out1, out1_bf16);
  if (!g2) return;
  norm(g2, b2, eps2);
  store(out2, out2_bf16);
}

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
  float mean = wave_sum_v(s) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    const float d = c < D ? v[i] - mean : 0.f;
    q += d * d;
  }
  float rstd = 1.0f / sqrtf(wave_sum_v(q) / D + eps1);
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
  mean = wave_sum_v(s) / D;
  q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    const float d = c < D ? v[i] - mean : 0.f;
    q += d * d;
  }
  rstd = 1.0f / sqrtf(wave_sum_v(q) / D + eps2);
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
  // Phase 0: the TT + K - 1 input rows (zero-padded at the sequence ends) are
  // staged into LDS with 16-B loads; phase 1: thread c slides its K taps over
  // its channel's column (register window) into an fp32 LDS tile; phase 2:
  // one wave per timestep normalises across channels, 4 channels per lane,
  // Swish, 8-/16-B stores.  Needs C % (64 * 4) == 0 and 16-B aligned rows.
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NR = TT + K - 1;
  T* xs = reinterpret_cast<T*>(smem);                                          // NR x C
  float* cv = reinterpret_cast<float*>(smem + (((size_t)NR * C * sizeof(T) + 15) & ~(size_t)15));  // TT x C
  const int ntile = (Tn + TT - 1) / TT;
  const int b = blockIdx.x / ntile;
  const int t0 = (blockIdx.x - b * ntile) * TT;
  const int nt = min(TT, Tn - t0);
  const T* xb = x + (long long)b * Tn * C;
  constexpr int VEC = 16 / sizeof(T);
  const int vpr = C / VEC;  // 16-B vectors per row
  for (int i = threadIdx.x; i < NR * vpr; i += blockDim.x) {
    const int r = i / vpr, cv0 = (i - r * vpr) * VEC;
    const int t = t0 - padL + r;
    uint4 val = make_uint4(0, 0, 0, 0);
    if (t >= 0 && t < Tn) val = *reinterpret_cast<const uint4*>(xb + (long long)t * C + cv0);
    *reinterpret_cast<uint4*>(xs + r * C + cv0) = val;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float wk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) wk[k] = w[c * K + k];
    float win[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) win[r] = ld(xs, r * C + c);
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
  const int nw = blockDim.x >> 6;
  for (int tt = wid; tt < nt; tt += nw) {
    const float* r = cv + tt * C;
    float s = 0.f;
    for (int c = 4 * lane; c < C; c += 256) {
      const float4 v = *reinterpret_cast<const float4*>(r + c);
      s += (v.x + v.y) + (v.z + v.w);
    }
    const float mean = wave_sum_v(s) / C;
    float q = 0.f;
    for (int c = 4 * lane; c < C; c += 256) {
      const float4 v = *reinterpret_cast<const float4*>(r + c);
      q += (v.x - mean) * (v.x - mean) + (v.y - mean) * (v.y - mean) + (v.z - mean) * (v.z - mean) +
           (v.w - mean) * (v.w - mean);
    }
    const float rstd = 1.0f / sqrtf(wave_sum_v(q) / C + eps);
    const long long ob = ((long long)b * Tn + t0 + tt) * C;
    for (int c = 4 * lane; c < C; c += 256) {
      const float4 v = *reinterpret_cast<const float4*>(r + c);
      float y[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float z = (y[e] - mean) * rstd * g[c + e] + beta[c + e];
        y[e] = z * (1.0f / (1.0f + __expf(-z)));
      }
      if (out_bf16) {
        uint2 pk;
        pk.x = pack_bf16x2(y[0], y[1]);
        pk.y = pack_bf16x2(y[2], y[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(out) + ob + c) = pk;
      } else {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + ob + c) = make_float4(y[0], y[1], y[2], y[3]);
      }
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
    const float mean = wave_sum_v(s) / C;
    float q = 0.f;
    for (int c = lane; c < C; c += 64) {
      const float d = r[c] - mean;
      q += d * d;
    }
    const float rstd = 1.0f / sqrtf(wave_sum_v(q) / C + eps);
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


// Both ConvBlocks of the ConvolutionFrontEnd in one kernel (convolution.py
// :12-84,169-175): conv3x3/s2 reflect (Cin=1) -> LN(F1*C1) -> LeakyReLU ->
// conv3x3/s2 reflect (C1 -> C2, MFMA implicit GEMM) -> LN(F2*C2) -> LeakyReLU.
// A tile is TT2 = 8 output time rows of one utterance: the 2*TT2+1 block-1
// rows they read (reflect-padded) are computed straight into LDS (the
// (B, T1, F1, C1) intermediate never reaches HBM), then block 2 runs as an
// implicit GEMM on MFMA and waves 0..7 normalise one output row each.
// Persistent (round 5): one 768-thread workgroup per CU walks a contiguous
// run of tiles with the block-2 weights resident in LDS; a tile continuing
// the previous one reuses its last block-1 row as row 0 (16 rows computed,
// not 17), and the next tile's input rows are staged into block-1 rows 1-3
// by the four waves that have no epilogue row.
//   x (B, Tin, Fin) fp32; w1 (C1, 3, 3) fp32 in conv_block_c1's tap order;
//   wp2 (C2, 3 time, 3 freq, C1) T; out (B, T2, F2*C2).
// (Tried: two rows per pass over all 10 waves with cross-wave LN reductions
// and VALU FMAs: 188 us; one row per wave on VALU FMAs: 130 us; one
// workgroup per tile with per-tile weight staging: 74.6 us; block 2 with its
// K loop split over wave pairs: +1k cycles per tile; a chunk-pair swizzle of
// the block-1 rows: more LDS bank conflicts, not fewer; block 2 on four
// waves beside the previous tile's epilogue on the other eight, yv in bf16
// and double-buffered: 57.5 vs 56.3 us, profiles/r05ah_fe_overlap_ab_rejected.log;
// frequency tile 2 packed two rows per MFMA (its 8 live frequencies of 16,
// 3 row steps instead of 5, segmented 8-lane statistics): 57.5 vs 55.3 us,
// profiles/r05al_fe_pack_ab_rejected.log — the per-lane row indexing costs
// every wave more than the masked columns did; an XOR bank swizzle of the
// block-2 output rows (its stores are 4-way conflicted): 57.2 vs 55.6 us,
// profiles/r05at_fe_yv_swizzle_ab_rejected.log — the extra index math and
// two spilled VGPRs cost more than the conflicts.)
// s_memtime marks of the waves of workgroup 100, its last tile (probe builds only)
#define FE_TL(i) SBK_PROBE(if (blockIdx.x == 100 && lane == 0) g_fe_tl[w][i] = __builtin_amdgcn_s_memtime();)

// 12 waves x 8 output rows (16-17 block-1 rows over 4 row groups x 3 frequency tiles).
// (8 waves x 7 rows with the block-1 LN affine held in VGPRs: 133 us.)
constexpr int FE_NT = 768, FE_TT2 = 8;
SBK_PROBE_BUFFER(g_fe_tl, FE_NT / 64, 16)

// f(std::integral_constant<int, I>) for I = 0 .. N-1: register arrays indexed
// inside get compile-time indices.  (The staged weights / affine used to sit
// in HIP uint4 / float4 struct arrays that were left in scratch: 96 B per
// thread through HBM, 86 MB of writes per launch; now native vectors.)
template <int... I, class F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(std::make_integer_sequence<int, N>{}, f);
}

// LeakyReLU on a packed pair: max(t, s t) for slopes <= 1 (2 packed-rate ops)
template <bool LMAX>
__device__ __forceinline__ float __attribute__((ext_vector_type(2)))
lrelu2(float __attribute__((ext_vector_type(2))) t, float s) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 ts = t * s;
  if (LMAX) return f2{fmaxf(t[0], ts[0]), fmaxf(t[1], ts[1])};
  return f2{t[0] >= 0.f ? t[0] : ts[0], t[1] >= 0.f ? t[1] : ts[1]};
}

template <typename T, int C1, bool LMAX>
__global__ void __launch_bounds__(FE_NT) frontend2_kernel(const float* __restrict__ x, int ntile, int Tin, int Fin,
                                                        int T1, int F1, int T2, int F2, const float* __restrict__ w1,
                                                        const float* __restrict__ b1, const float* __restrict__ g1,
                                                        const float* __restrict__ be1, float eps1, float slope1,
                                                        const T* __restrict__ wp2, int C2,
                                                        const float* __restrict__ b2, const float* __restrict__ g2,
                                                        const float* __restrict__ be2, float eps2, float slope2,
                                                        void* out, int out_bf16, const float* __restrict__ slot_max,
                                                        int nslot, float top_db) {
  using Tr = MT<T>;
  constexpr int NT = FE_NT, NW = NT / 64, TT2 = FE_TT2, NJ = 2 * TT2 + 1;
  static_assert(C1 == 64, "block-1 MFMA map: 4 channel tiles");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // LDS row strides padded by 16 B: the MFMA fragment reads of 16 lanes at
  // different output frequencies (b1r rows 2 apart) / channels (wl rows)
  // then spread over the banks instead of hitting one 16-B slot column
  constexpr int C1P = C1 + 8;
  const int K = 9 * C1, KP = K + 8;
  // region 0: the block-2 weights, staged once and resident for all of the
  // workgroup's tiles
  T* wl = reinterpret_cast<T*>(smem);                                   // C2 x KP block-2 weights
  const int r0 = (C2 * KP * (int)sizeof(T) + 15) & ~15;
  float* yv = reinterpret_cast<float*>(smem + r0);                      // TT2 x F2*C2 (block 2)
  T* b1r = reinterpret_cast<T*>(yv + TT2 * F2 * C2);                    // NJ x F1 x C1P
  // the block-1 input rows (NJ x 3 x Fin fp32, <= 16.3 KB) live in b1r rows
  // 1 .. 3: staged during the previous tile's epilogue (block 2 is done
  // with b1r), gathered before the block-1 statistics barrier, overwritten
  // by block 1's own rows only after it (host-checked to fit rows 1 .. 15)
  float* xs = reinterpret_cast<float*>(b1r + F1 * C1P);
  uint2* wal = reinterpret_cast<uint2*>(b1r + NJ * F1 * C1P);           // 4 x 64 block-1 A fragments (bf16 taps)
  float* g2s = reinterpret_cast<float*>(wal + 4 * 64);                  // F2*C2 block-2 LN gamma
  float* be2s = g2s + F2 * C2;                                          // F2*C2 block-2 LN beta

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nblk = (T2 + TT2 - 1) / TT2;
  // contiguous tile runs: a tile that continues the previous one (same
  // utterance) takes its block-1 row 0 from the previous tile's row 16
  const int tbeg = (int)(((long long)blockIdx.x * ntile) / gridDim.x);
  const int tend = (int)(((long long)(blockIdx.x + 1) * ntile) / gridDim.x);
  int tile = tbeg;
  FE_TL(14);

  // Persistent workgroups (round 5): one per CU, each walks a contiguous run
  // of tiles.  The per-tile constants — block-2 weights (37 KB) and LN
  // affine, block-1 taps — load into LDS once per workgroup, and the next
  // tile's input rows and top_db floor are staged by the four waves that
  // have no epilogue row, while waves 0-7 run the epilogue.  Block-1 row j
  // is t1 = reflect(2*t20 - 1 + j) and reads x rows reflect(2*t1 - 1 + kt).
  constexpr int WV = (32 * 9 * 64 / 8 + NT - 1) / NT;  // weight vectors per thread (C2 <= 32)
  constexpr int SNT = NT - 64 * TT2;                  // stager threads (waves TT2 ..)
  constexpr int SXV = (NJ * 3 * 20 + SNT - 1) / SNT;  // x vectors per stager thread (Fin <= 80)
  const int fq4 = Fin / 4;        // Fin % 4 == 0, Fin <= 80 (host-checked)
  const float inv_fq4 = 1.0f / (float)fq4;
  // native vectors: the HIP float4 / uint4 structs (a union inside) held in
  // a register array are not always split into registers
  typedef float nf4 __attribute__((ext_vector_type(4)));
  typedef uint32_t nu4 __attribute__((ext_vector_type(4)));
  __shared__ float redm[FE_NT / 64];  // top_db: the stager waves' partial maxima
  // stager thread t (0 .. SNT-1): tile tl's input rows into xs (all loads in
  // flight before the first store) and, for a tile that opens an utterance,
  // the floor's partial maxima into redm
  auto stage_load = [&](int tl, int t, nf4 (&v)[SXV]) __attribute__((always_inline)) {
    const int b = tl / nblk, t20 = (tl - b * nblk) * TT2;
    const float* xb = x + (long long)b * Tin * Fin;
#pragma unroll
    for (int u = 0; u < SXV; ++u) {
      const int i = min(t + u * SNT, NJ * 3 * fq4 - 1);
      const int q = (int)(((float)i + 0.5f) * inv_fq4);  // i / fq4 (exact: i < 2^11, fq4 <= 20)
      const int f4 = i - q * fq4;
      const int j = q / 3, kt = q - 3 * j;
      const int t1 = reflect_idx(2 * t20 - 1 + j, T1);
      v[u] = *reinterpret_cast<const nf4*>(xb + (long long)reflect_idx(2 * t1 - 1 + kt, Tin) * Fin + 4 * f4);
    }
  };
  // the floor's partial maxima of utterance b (stager thread t) into redm
  auto floor_part = [&](int b, int t) __attribute__((always_inline)) {
    float m = -INFINITY;
    for (int i = t; i < nslot; i += SNT) m = fmaxf(m, slot_max[(long long)b * nslot + i]);
    m = wave_max(m);
    if (lane == 0) redm[w - TT2] = m;
  };
  auto stage_store = [&](int t, const nf4 (&v)[SXV]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < SXV; ++u)
      if (t + u * SNT < NJ * 3 * fq4) *reinterpret_cast<nf4*>(xs + 4 * (t + u * SNT)) = v[u];
  };
  // the next tile's rows and, if it opens an utterance, its floor
  auto stage = [&](int tl, int t) __attribute__((always_inline)) {
    nf4 v[SXV];
    stage_load(tl, t, v);
    const int b = tl / nblk;
    if (slot_max && tl == b * nblk) floor_part(b, t);
    stage_store(t, v);
  };
  // prologue: every global load is issued before the first LDS store (one
  // memory latency at the launch's start, not four in a row)
  const int nwv = C2 * K / Tr::VEC;
  nu4 wvin[WV];
  static_for<WV>([&](auto U) { wvin[U] = reinterpret_cast<const nu4*>(wp2)[min(tid + U * NT, nwv - 1)]; });
  const int ngv = 2 * F2 * C2 / 4;  // block-2 LN affine vectors (<= 320 <= NT)
  const nf4 gin = tid < ngv ? (tid < ngv / 2 ? reinterpret_cast<const nf4*>(g2)[tid]
                                             : reinterpret_cast<const nf4*>(be2)[tid - ngv / 2])
                            : nf4{0.f, 0.f, 0.f, 0.f};
  // block-1 A fragments (W^T rows c = 16 mt + fr, taps 4 g4 .. 4 g4 + 3),
  // packed and stored by wave 0 below
  float tw[4][4];
  if (w == 0) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 4 * (lane >> 4) + e, c = 16 * mt + (lane & 15);
        tw[mt][e] = k < 9 ? w1[c * 9 + min(k, 8)] : (k == 9 && b1 ? b1[c] : 0.f);
      }
  }
  nf4 xv0[SXV];
  if (w >= TT2) {
    stage_load(tile, tid - 64 * TT2, xv0);
    // the run's first tile's floor (it may continue an utterance)
    if (slot_max) floor_part(tile / nblk, tid - 64 * TT2);
  }
  static_for<WV>([&](auto U) {
    const int i = tid + U * NT;
    if (i < nwv) {
      const int co = (i * Tr::VEC) / K, kk = i * Tr::VEC - co * K;
      *reinterpret_cast<nu4*>(wl + co * KP + kk) = wvin[U];
    }
  });
  if (tid < ngv) reinterpret_cast<nf4*>(g2s)[tid] = gin;
  if (w >= TT2) stage_store(tid - 64 * TT2, xv0);
  // block 1 on MFMA: the 3x3 / stride-2 convolution of a row is
  // C^T[c][f1] = W^T[c][tap] · X^T[tap][f1] with the 9 taps zero-padded to
  // one 16-deep bf16 step (v_mfma_f32_16x16x16_bf16; conv inputs and taps in
  // bf16, fp32 accumulation — what the reference computes under autocast):
  // 4 x 3 tiles of 16x16 per row.  A lane then holds 4 consecutive channels
  // of one frequency per tile; each tile leaves as one 8-B LDS store.  The
  // B-fragment gathers use row-invariant LDS offsets computed once, the LN
  // statistics and affine run as packed fp32 pairs, bf16 packing is
  // v_cvt_pk_bf16_f32.  Tap order k = kf * 3 + kt (conv_block_c1's layout of w1)
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
  auto pack2 = [](f32x2 v) __attribute__((always_inline)) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
  };
  const int fr = lane & 15, g4 = lane >> 4;
  // A fragments (W^T rows c = 16 mt + fr, taps 4 g4 .. 4 g4 + 3) packed once
  // by wave 0 into LDS; each tile re-reads them (held in VGPRs across the
  // tile loop they pushed block 2 into spills).  Tap 9 carries the bias
  // against a B entry of 1.0, so the MFMA adds it (in bf16, as autocast's
  // conv2d does) and no bias registers are needed; taps 10-15 are zero.
  if (w == 0) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      wal[mt * 64 + lane] = uint2{pack2(f32x2{tw[mt][0], tw[mt][1]}), pack2(f32x2{tw[mt][2], tw[mt][3]})};
  }
  // Block 1, work split: wave w takes frequency tile nt = w % 3 of the rows
  // j = w / 3 + 4 i (12 waves: 4 row groups x 3 tiles), all four channel
  // tiles, which share each gathered B fragment.  The LN affine of the
  // wave's 16 frequencies x 64 channels sits in VGPRs; the rows'
  // accumulators stay in VGPRs while the row statistics combine over the
  // three tile waves through LDS — two workgroup barriers for the 17 rows.
  static_assert(NW == 12, "block 1: 4 row groups x 3 frequency tiles");
  constexpr int RG = 4, RPW = (NJ + RG - 1) / RG;  // rows per wave (5)
  __shared__ float lnred[2][NJ][4];                 // [pass][row][tile] partial sums
  const int nt = w % 3, grp = w / 3;
  const float inv_n1 = 1.0f / (float)(F1 * C1);
  // block 2 (tile-invariant part): rows m = t2_local * F2 + f2, columns the C2
  // channels, K = (kt, kf, ci); wave w < nmw owns m-tiles TMW w .. TMW w + TMW - 1
  const int ntl = C2 / 16;
  constexpr int TMW = 2;  // m-tiles per wave
  const int nout = F2 * C2;  // multiple of 16 (C2 % 16 == 0)
  const float inv_f2 = 1.0f / (float)F2, inv_nout = 1.0f / (float)nout;
  const int nch = nout / 8;
  constexpr int NCH = (32 * 32 / 8 + 63) / 64;  // epilogue chunks per lane (F2, C2 <= 32)

  __syncthreads();  // wl, wal, LN affine, the first tile's xs and floor staged
  float floor_db = -INFINITY;
  for (; tile < tend; ++tile) {
    const int b = tile / nblk, t20 = (tile - b * nblk) * TT2;
    const int carry = tile > tbeg && t20 > 0 ? 1 : 0;  // row 0 already in b1r
    FE_TL(0);
    // lane-derived addressing recomputed per tile from an opaque copy of the
    // lane id: hoisted out of the loop, the tile-invariant LDS addresses of
    // every gather / store occupied ~170 VGPRs (scratch spills)
    int tdl = tid;
    asm volatile("" : "+v"(tdl));
    const int ln = tdl & 63;
    const int frl = ln & 15, g4l = ln >> 4;
    const int f1 = 16 * nt + frl;
    const int f1c = min(f1, F1 - 1);
    const float colm = f1 < F1 ? 1.f : 0.f;
    // this lane's B-fragment taps k = 4 g4 + e of output frequency f1, as
    // row-relative LDS offsets (k >= 9 and frequencies >= F1 read a valid
    // element: the matching A entries are zero / the column is masked)
    int goff[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = min(4 * g4l + e, 8);
      goff[e] = (k % 3) * Fin + reflect_idx(2 * f1c + k / 3 - 1, Fin);
    }
    const int fk = 8 * g4l;
    const bool one9 = g4l == 2;  // this lane's B entry e = 1 is tap 9: the bias's 1.0

    // the Fbank's top_db floor (features.py:706-711): max over the
    // utterance's spectrum-kernel partial maxima - top_db, reduced by the
    // stager waves when the utterance's first tile of this run was staged;
    // applied at the block-1 gathers (the separate clamp pass is gone)
    const bool newutt = tile == tbeg || t20 == 0;
    if (slot_max && newutt) {
      float m = redm[0];
#pragma unroll
      for (int i = 1; i < FE_NT / 64 - TT2; ++i) m = fmaxf(m, redm[i]);
      floor_db = m - top_db;
    }
    FE_TL(1);
    // max(v, floor) as one v_max_f32 (fmaxf of a loaded value adds a NaN-quieting max)
    auto flo = [floor_db](float v) __attribute__((always_inline)) {
      float r;
      asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(floor_db));
      return r;
    };
    s16x4 wa[4];  // (after the barrier: wave 0 staged them before the first tile)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      wa[mt] = __builtin_bit_cast(s16x4, wal[mt * 64 + ln]);
    }
    // the wave's LN affine (L2-resident; per tile, so it is not live through block 2)
    f32x4 gam[4], bet[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      gam[mt] = *reinterpret_cast<const f32x4*>(g1 + f1c * C1 + 16 * mt + 4 * g4l);
      bet[mt] = *reinterpret_cast<const f32x4*>(be1 + f1c * C1 + 16 * mt + 4 * g4l);
    }
    f32x4 acc[RPW][4];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      // rows j = carry + grp + 4 i: 16 rows of a continuing tile (4 per
      // group), else 17 (group 0 takes the fifth); a wave without a fifth
      // row branches over it (uniform)
      const int j = carry + grp + RG * i;
      if (i == RPW - 1 && j >= NJ) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[i][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        continue;
      }
      const float* r = xs + (j * 3) * Fin;
      const s16x4 xb4 = __builtin_bit_cast(
          s16x4, uint2{pack2(f32x2{flo(r[goff[0]]), one9 ? 1.f : flo(r[goff[1]])}),
                       pack2(f32x2{flo(r[goff[2]]), flo(r[goff[3]])})});
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[i][mt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(wa[mt], xb4, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
    // LayerNorm statistics of each row over its F1 x C1 values in one pass:
    // the tile waves' sums and sums of squares combine through LDS behind one
    // barrier (var = E[y^2] - mean^2 in fp32: a row's |mean| / std stays far
    // below the 2^12 where that loses bf16 precision; the second pass over
    // the registers and its barrier cost ~8 % of the kernel)
    float mean[RPW], rstd[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int j = carry + grp + RG * i;
      if (i == RPW - 1 && j >= NJ) continue;
      f32x2 sn = {0.f, 0.f}, sq = {0.f, 0.f};
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x2 a0 = f32x2{acc[i][mt][0], acc[i][mt][1]}, a1 = f32x2{acc[i][mt][2], acc[i][mt][3]};
        sn += a0;
        sn += a1;
        sq = a0 * a0 + sq;
        sq = a1 * a1 + sq;
      }
      const float t = wave_sum_v((sn.x + sn.y) * colm), u = wave_sum_v((sq.x + sq.y) * colm);
      if (j < NJ && lane == 0) {
        lnred[0][j][nt] = t;
        lnred[1][j][nt] = u;
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int j = min(carry + grp + RG * i, NJ - 1);
      const float t = (lnred[0][j][0] + lnred[0][j][1]) + lnred[0][j][2];
      const float u = (lnred[1][j][0] + lnred[1][j][1]) + lnred[1][j][2];
      mean[i] = t * inv_n1;
      rstd[i] = rsqrtf(fmaxf(u * inv_n1 - mean[i] * mean[i], 0.f) + eps1);
    }
    FE_TL(2);
    // this lane's b1r slot in row 0; rows are F1 * C1P apart (a scalar offset)
    T* const b1w = b1r + f1 * C1P + 4 * g4l;
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int j = carry + grp + RG * i;
      if (j >= NJ || f1 >= F1) continue;
      // (x - mean) rstd as one packed FMA, x rstd + (-mean rstd)
      const f32x2 rv = {rstd[i], rstd[i]}, nmr = {-mean[i] * rstd[i], -mean[i] * rstd[i]};
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        f32x2 y0 = (f32x2{acc[i][mt][0], acc[i][mt][1]} * rv + nmr) * f32x2{gam[mt][0], gam[mt][1]} +
                   f32x2{bet[mt][0], bet[mt][1]};
        f32x2 y1 = (f32x2{acc[i][mt][2], acc[i][mt][3]} * rv + nmr) * f32x2{gam[mt][2], gam[mt][3]} +
                   f32x2{bet[mt][2], bet[mt][3]};
        y0 = lrelu2<LMAX>(y0, slope1);
        y1 = lrelu2<LMAX>(y1, slope1);
        *reinterpret_cast<uint2*>(b1w + j * (F1 * C1P) + 16 * mt) = uint2{pack2(y0), pack2(y1)};
      }
    }
    FE_TL(3);
    __syncthreads();  // b1r complete; xs free for yv

    // block 2 as one implicit GEMM over the tile's output positions (8 x 20
    // = 160 rows = 10 m-tiles at config 3, no padded rows): each K step
    // issues 2 TMW MFMAs behind TMW + 2 fragment reads.  (One m-tile per
    // wave — ten multiplying waves of 18 steps — measured equal to five
    // waves of two, 74.4 vs 74.6 us, profiles/r05t_fe_tl.log.)
    const int nrow = min(TT2, T2 - t20);  // valid output rows of this tile
    const int Mv = nrow * F2;
    const int nmw = (Mv + 16 * TMW - 1) / (16 * TMW);  // waves with MFMA work (<= NW: F1 <= 40, F2 <= 20, TT2 = 8)
    f32x4 acc2[TMW][2];
#pragma unroll
    for (int tm = 0; tm < TMW; ++tm)
#pragma unroll
      for (int tn = 0; tn < 2; ++tn) acc2[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
    float cb[2] = {0.f, 0.f};
    if (w < nmw) {
      int aoff[TMW][3];  // A-row (m = 16 TMW w + 16 tm + frl) offsets into b1r per kf, kt = 0
#pragma unroll
      for (int tm = 0; tm < TMW; ++tm) {
        const int m = 16 * TMW * w + 16 * tm + frl;
        const int mc = m < Mv ? m : 0;
        const int tl = (int)(((float)mc + 0.5f) * inv_f2), fo = mc - tl * F2;  // mc / F2 (mc < 160)
#pragma unroll
        for (int kf = 0; kf < 3; ++kf) aoff[tm][kf] = (2 * tl * F1 + reflect_idx(2 * fo - 1 + kf, F1)) * C1P + fk;
      }
#pragma unroll
      for (int tn = 0; tn < 2; ++tn) cb[tn] = b2 && tn < ntl ? b2[tn * 16 + frl] : 0.f;
      // unconditional fragment reads (rows past Mv / channel tiles past C2 read
      // valid LDS and are discarded at the store), fully unrolled so the reads
      // of later K steps issue ahead of the MFMAs
      const int wo = frl * KP + fk;
      const T* wrow[2] = {wl + wo, wl + wo + (ntl > 1 ? 16 : 0) * KP};
      // (reading step st + 1's fragments ahead of step st's MFMAs measured
      // 1-1.5 us slower: profiles/r05ac_fe_pipe_ab.log)
      typename Tr::frag fa[1][TMW], fbw[1][2];
      auto ld = [&](auto S, int buf) __attribute__((always_inline)) {
        constexpr int st = decltype(S)::value;
        constexpr int kt = st / 6, kf = (st / 2) % 3, c0 = 32 * (st % 2);
        constexpr int k = (kt * 3 + kf) * C1 + c0;
#pragma unroll
        for (int tm = 0; tm < TMW; ++tm) fa[buf][tm] = Tr::load(b1r + kt * F1 * C1P + aoff[tm][kf] + c0);
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) fbw[buf][tn] = Tr::load(wrow[tn] + k);
      };
      static_for<18>([&](auto S) {
        ld(S, 0);
#pragma unroll
        for (int tm = 0; tm < TMW; ++tm)
#pragma unroll
          for (int tn = 0; tn < 2; ++tn) Tr::mma(acc2[tm][tn], fa[0][tm], fbw[0][tn]);
      });
      // D rows m = 16 TMW w + 16 tm + 4 (lane >> 4) + r -> yv[m][co] (rows of
      // one output time step are contiguous: yv[t2_local][f2][co]); row
      // offsets beyond the lane base are scalar, and a full tile stores
      // without row guards
      const int mb = 16 * TMW * w + 4 * g4l;
      float* const yw0 = yv + mb * C2 + frl;
      const bool full = Mv == TT2 * F2 && 16 * TMW * nmw <= Mv;
#pragma unroll
      for (int tm = 0; tm < TMW; ++tm)
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) {
          if (tn >= ntl) continue;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (full || mb + 16 * tm + r < Mv) yw0[(16 * tm + r) * C2 + 16 * tn] = acc2[tm][tn][r] + cb[tn];
        }
    }
    FE_TL(12);
    __syncthreads();  // yv complete; block 2 done with b1r
    if (w >= TT2) {
      // the waves without an epilogue row: carry block-1 row 16 into row 0
      // for a continuing next tile (its row 0 is this tile's row 16), and
      // stage the next tile's input rows (b1r rows 1 .. 3) and floor
      const int nv = F1 * C1P * (int)sizeof(T) / 16;
      for (int v = tdl - 64 * TT2; v < nv; v += SNT)
        reinterpret_cast<nu4*>(b1r)[v] = reinterpret_cast<const nu4*>(b1r + (NJ - 1) * F1 * C1P)[v];
      if (tile + 1 < tend) stage(tile + 1, tdl - 64 * TT2);
    }
    if (w < nrow) {
      const int t2 = t20 + w;
      const float* yw = yv + w * F2 * C2;
      // the wave's own LDS row: LN over F2*C2 (wave-local), LeakyReLU, store.
      // Lane l owns elements 8c .. 8c+7 for chunks c = l, l + 64, ... (16-B LDS
      // reads, 2 x 16-B affine loads, one 16-B bf16 store per chunk)
      float yv8[NCH][8];
      float s2 = 0.f;
#pragma unroll
      for (int u = 0; u < NCH; ++u) {
        const int c = ln + 64 * u;
        const int cc = min(c, nch - 1);
        const float4 a0 = *reinterpret_cast<const float4*>(yw + 8 * cc);
        const float4 a1 = *reinterpret_cast<const float4*>(yw + 8 * cc + 4);
        const float t8[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          yv8[u][e] = c < nch ? t8[e] : 0.f;
          s2 += yv8[u][e];
        }
      }
      const float m2 = wave_sum_v(s2) * inv_nout;
      float q2 = 0.f;
#pragma unroll
      for (int u = 0; u < NCH; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dv = ln + 64 * u < nch ? yv8[u][e] - m2 : 0.f;
          q2 += dv * dv;
        }
      const float r2 = rsqrtf(wave_sum_v(q2) * inv_nout + eps2);
      const long long ob = ((long long)b * T2 + t2) * nout;
#pragma unroll
      for (int u = 0; u < NCH; ++u) {
        const int c = ln + 64 * u;
        if (c >= nch) continue;
        // the LN affine from LDS (staged once; in registers it pushed the
        // prefetched rows into scratch)
        const float4 ga = *reinterpret_cast<const float4*>(g2s + 8 * c);
        const float4 gb = *reinterpret_cast<const float4*>(g2s + 8 * c + 4);
        const float4 ba = *reinterpret_cast<const float4*>(be2s + 8 * c);
        const float4 bb = *reinterpret_cast<const float4*>(be2s + 8 * c + 4);
        const float gg[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
        const float bt[8] = {ba.x, ba.y, ba.z, ba.w, bb.x, bb.y, bb.z, bb.w};
        float y[8];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const f32x2 t = (f32x2{yv8[u][e], yv8[u][e + 1]} * f32x2{r2, r2} + f32x2{-m2 * r2, -m2 * r2}) *
                              f32x2{gg[e], gg[e + 1]} + f32x2{bt[e], bt[e + 1]};
          const f32x2 l = lrelu2<LMAX>(t, slope2);
          y[e] = l[0];
          y[e + 1] = l[1];
        }
        if (out_bf16) {
          *reinterpret_cast<typename MT<bf16_t>::frag*>(reinterpret_cast<bf16_t*>(out) + ob + 8 * c) = MT<bf16_t>::from8(y);
        } else {
          float* o = reinterpret_cast<float*>(out) + ob + 8 * c;
          *reinterpret_cast<float4*>(o) = make_float4(y[0], y[1], y[2], y[3]);
          *reinterpret_cast<float4*>(o + 4) = make_float4(y[4], y[5], y[6], y[7]);
        }
      }
    }
    FE_TL(13);
    __syncthreads();  // yv read; the next tile's xs, row 0 and floor staged
  }
  FE_TL(15);
}

// key padding mask from relative lengths (TransformerASR.py:295-301):
// out[b, t] = t > floor(rel_len[b] * T)   (fp32 product, as torch computes it)
__global__ void length_mask_kernel(const float* __restrict__ rel_len, int B, int T, uint8_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * T) return;
  const int b = i / T, t = i - b * T;
  out[i] = (float)t > floorf(rel_len[b] * (float)T) ? 1 : 0;
}

// 4 values per thread (16-B loads, 8-B stores) when n % 4 == 0 and aligned
__global__ void cast_bf16x4_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long long n4) {
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (long long)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(x)[q];
    uint2 u;
    u.x = pack_bf16x2(v.x, v.y);
    u.y = pack_bf16x2(v.z, v.w);
    reinterpret_cast<uint2*>(y)[q] = u;
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

SBK_PROBE_EXPORT(sbk_probe_fe_tl, g_fe_tl)

SBK_API int sbk_layernorm(const float* x, int M, int D, const float* g1, const float* b1, float eps1, void* out1,
                          int out1_bf16, const float* g2, const float* b2, float eps2, void* out2, int out2_bf16,
                          void* stream) {
  if (M <= 0 || D <= 0 || D > 1024) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const uintptr_t al = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(g1) |
                       reinterpret_cast<uintptr_t>(b1) | reinterpret_cast<uintptr_t>(g2) |
                       reinterpret_cast<uintptr_t>(b2) | reinterpret_cast<uintptr_t>(out1) |
                       reinterpret_cast<uintptr_t>(out2);
  if (D == 256 && !(al & 15)) {
    constexpr int RPW = 4;
    hipLaunchKernelGGL(layernorm256_kernel<RPW>, dim3((M + 4 * RPW - 1) / (4 * RPW)), dim3(256), 0, s, x, M, g1, b1,
                       eps1, out1, out1_bf16, g2, b2, eps2, out2, out2_bf16);
    SBK_CHECK_LAUNCH();
    return 0;
  }
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
  if (K == 31 && C % 256 == 0 && (size_t)(16 + 30) * C * 4 + (size_t)16 * C * 4 <= 64 * 1024) {
    constexpr int TT = 16;
    const int grid = B * ((Tn + TT - 1) / TT);
    const size_t esz = in_bf16 ? 2 : 4;
    const size_t lds = (((size_t)(TT + 30) * C * esz + 15) & ~(size_t)15) + (size_t)TT * C * 4;
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

SBK_API int sbk_conv_frontend2(int dtype_bf16, const float* x, int B, int Tin, int Fin, const float* w1,
                               const float* b1, const float* g1, const float* be1, float eps1, float slope1, int C1,
                               const void* wp2, const float* b2, const float* g2, const float* be2, float eps2,
                               float slope2, int C2, void* out, int out_bf16, const float* slot_max, int nslot,
                               float top_db, int* Tout_, int* Fout_, void* stream) {
  if (B <= 0 || Tin < 2 || Fin < 4 || C1 != 64 || C2 % 16 || C2 <= 0 || (slot_max && nslot <= 0)) return SBK_ERR_ARG;
  const int T1 = (Tin - 1) / 2 + 1, F1 = (Fin - 1) / 2 + 1;
  const int T2 = (T1 - 1) / 2 + 1, F2 = (F1 - 1) / 2 + 1;
  if (Tout_) *Tout_ = T2;
  if (Fout_) *Fout_ = F2;
  if (!x) return 0;
  if (F1 > 40 || T1 < 2 || F1 < 2 || F2 > 32 || C2 > 32 || Fin % 4 || Fin > 80) return SBK_ERR_ARG;
  // 16-B vector loads / stores of x rows, LN affine and out rows
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(g1) | reinterpret_cast<uintptr_t>(be1) |
       reinterpret_cast<uintptr_t>(g2) | reinterpret_cast<uintptr_t>(be2) | reinterpret_cast<uintptr_t>(out) |
       reinterpret_cast<uintptr_t>(wp2)) & 15)
    return SBK_ERR_ARG;
  constexpr int TT2 = FE_TT2, NJ = 2 * TT2 + 1;
  const size_t esz = dtype_bf16 ? 2 : 4;
  const size_t lds = (((size_t)C2 * (9 * C1 + 8) * esz + 15) & ~(size_t)15) +
                     (size_t)TT2 * F2 * C2 * 4 + (size_t)NJ * F1 * (C1 + 8) * esz +
                     4 * 64 * 8 + (size_t)2 * F2 * C2 * 4;  // block-1 A fragments, block-2 LN affine
  if (dtype_bf16 && lds > 160 * 1024 - 640) return SBK_ERR_ARG;  // + 592 B of static LDS
  // the block-1 input rows live in b1r rows 1 .. 15 (kernel)
  if ((size_t)NJ * 3 * Fin * 4 > (size_t)(NJ - 2) * F1 * (C1 + 8) * esz) return SBK_ERR_ARG;
  // persistent: one workgroup per CU (the LDS allows no second), each
  // walking tiles blockIdx.x + k gridDim.x
  const int ntile = B * ((T2 + TT2 - 1) / TT2);
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  const dim3 grid(std::min(ntile, ncu));
  hipStream_t s = (hipStream_t)stream;
  if (!dtype_bf16) return SBK_ERR_ARG;  // fp32 path: the per-block kernels (LDS would not fit)
  auto launch = [&](auto kern) -> int {
    // lds depends on the shapes (F1, F2, C2): lds_optin raises the opt-in when a launch needs more
    if (hipError_t e = sbk::lds_optin(reinterpret_cast<const void*>(kern), lds)) return (int)e;
    hipLaunchKernelGGL(kern, grid, dim3(FE_NT), lds, s, x, ntile, Tin, Fin, T1, F1, T2, F2, w1, b1, g1, be1, eps1, slope1,
                       reinterpret_cast<const bf16_t*>(wp2), C2, b2, g2, be2, eps2, slope2, out, out_bf16, slot_max,
                       nslot, top_db);
    return 0;
  };
  const int rc = slope1 <= 1.f && slope2 <= 1.f ? launch(&frontend2_kernel<bf16_t, 64, true>)
                               : launch(&frontend2_kernel<bf16_t, 64, false>);
  if (rc) return rc;
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_length_mask(const float* rel_len, int B, int T, uint8_t* out, void* stream) {
  if (B <= 0 || T <= 0 || !rel_len || !out) return SBK_ERR_ARG;
  hipLaunchKernelGGL(length_mask_kernel, dim3((B * T + 255) / 256), dim3(256), 0, (hipStream_t)stream, rel_len, B, T,
                     out);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_cast_bf16(const float* x, void* y, long long n, void* stream) {
  if (n <= 0) return SBK_ERR_ARG;
  if (n % 4 == 0 && !((reinterpret_cast<uintptr_t>(x) & 15) | (reinterpret_cast<uintptr_t>(y) & 7))) {
    hipLaunchKernelGGL(cast_bf16x4_kernel, dim3(grid_for(n / 4, 256)), dim3(256), 0, (hipStream_t)stream, x,
                       reinterpret_cast<bf16_t*>(y), n / 4);
    SBK_CHECK_LAUNCH();
    return 0;
  }
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
