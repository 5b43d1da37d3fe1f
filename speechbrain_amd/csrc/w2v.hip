// Config 5 front-end: the wav2vec2 latent extractor (W2VLatentExtractor,
// speechbrain/lobes/models/wav2vec.py:28-106) and the row LayerNorm /
// activation / MXFP8-quantisation kernel shared by the extractor's later
// layers and the TransformerEncoder (lobes/models/transformer/Transformer.py:
// 246-486).
//
//   sbk_w2v_wav_stats  per-utterance mean / rstd of F.layer_norm(x, x.shape[1:])
//                      (wav2vec.py:92-93), fp64 accumulation, one block per
//                      utterance, deterministic
//   sbk_w2v_conv0      layer 0 (Cin = 1, k = 11, stride 5, no bias, "valid")
//                      with the waveform normalisation applied on load, then
//                      LayerNorm over the channels and GELU (ConvBlock order
//                      conv → norm → act, convolution.py:134-147), written as
//                      fp32, bf16 or MXFP8 (+ E8M0 block scales): the
//                      (B, 47998, 512) activation never exists in fp32
//   sbk_ln_act         one wave per row: optional LayerNorm, optional GELU /
//                      ReLU, output fp32 / bf16 / MXFP8 — the post-GEMM
//                      epilogue of extractor layers 1..6 and the pre-norms of
//                      the transformer layers (their MXFP8 A operands)
//
// Layer 0 is VALU work (11 MACs per output, 17 GFLOP at B = 32 x 15 s) and
// its output is the largest tensor of the path (786 M values), so it is
// bound by the output write: in MXFP8 that is 1 byte + 1/32 scale byte per
// value instead of 4.
#include "mx.h"

using namespace sbk;

namespace {

__global__ void __launch_bounds__(1024) wav_stats_kernel(const float* __restrict__ wav, long long S, float eps,
                                                         float* __restrict__ stats) {
  __shared__ double red[32];
  const int b = blockIdx.x;
  const float* x = wav + (long long)b * S;
  double s = 0.0, q = 0.0;
  for (long long i = threadIdx.x; i < S; i += blockDim.x) {
    const double v = x[i];
    s += v;
    q += v * v;
  }
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    q += __shfl_xor(q, o);
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w] = s;
    red[16 + w] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ts = 0.0, tq = 0.0;
    for (int i = 0; i < nw; ++i) {
      ts += red[i];
      tq += red[16 + i];
    }
    const double mean = ts / (double)S;
    double var = tq / (double)S - mean * mean;
    if (var < 0.0) var = 0.0;
    stats[2 * b] = (float)mean;
    stats[2 * b + 1] = (float)(1.0 / sqrt(var + (double)eps));
  }
}

// out_mode: 0 fp32, 1 bf16, 2 MXFP8 (+ scales: one byte per 32 channels)
template <int R>
__global__ void __launch_bounds__(1024) conv0_kernel(const float* __restrict__ wav, const float* __restrict__ stats,
                                                     long long S, int T0, int C, int K, int stride,
                                                     const float* __restrict__ w, const float* __restrict__ g,
                                                     const float* __restrict__ be, float eps, void* __restrict__ out,
                                                     int out_mode, uint8_t* __restrict__ scales) {
  extern __shared__ __attribute__((aligned(16))) float xs[];  // (R-1)*stride + K samples
  __shared__ float red[R][16];
  const int nblk_t = (T0 + R - 1) / R;
  const int b = blockIdx.x / nblk_t;
  const int t0 = (blockIdx.x - b * nblk_t) * R;
  const int nr = min(R, T0 - t0);
  const int win = (nr - 1) * stride + K;
  const float* x = wav + (long long)b * S + (long long)t0 * stride;
  const float mean = stats ? stats[2 * b] : 0.f, rstd = stats ? stats[2 * b + 1] : 1.f;
  for (int i = threadIdx.x; i < win; i += blockDim.x) xs[i] = (x[i] - mean) * rstd;
  const int c = threadIdx.x;
  const bool live = c < C;
  float wk[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) wk[k] = (live && k < K) ? w[c * K + k] : 0.f;
  __syncthreads();
  float v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < K) a = fmaf(wk[k], xs[min(r, nr - 1) * stride + k], a);
    v[r] = live ? a : 0.f;
  }
  // LayerNorm over the C channels of each frame: two passes (mean, then the
  // centred second moment), wave sums then a cross-wave LDS sum
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  const float invC = 1.f / (float)C;
  float mu[R], rs[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float s = wave_sum_v(v[r]);
    if (lane == 0) red[r][wv] = s;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += red[r][i];
    mu[r] = s * invC;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float d = live ? v[r] - mu[r] : 0.f;
    const float s = wave_sum_v(d * d);
    if (lane == 0) red[r][wv] = s;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += red[r][i];
    rs[r] = rsqrtf(s * invC + eps);
  }
  const float gc = live ? g[c] : 0.f, bc = live ? be[c] : 0.f;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r >= nr) break;
    const float y = gelu_erf((v[r] - mu[r]) * rs[r] * gc + bc);
    const long long o = ((long long)b * T0 + t0 + r) * C + c;
    if (out_mode == 2) {
      // 32 consecutive channels = 32 consecutive lanes (C % 32 == 0)
      float am = fabsf(live ? y : 0.f);
#pragma unroll
      for (int s = 1; s < 32; s <<= 1) am = fmaxf(am, __shfl_xor(am, s));
      const int sb = mx_scale_byte(am);
      const float q = clamp_e4m3(y * mx_inv_scale(sb));
      const int p = __builtin_amdgcn_cvt_pk_fp8_f32(q, q, 0, false);
      if (live) {
        reinterpret_cast<uint8_t*>(out)[o] = (uint8_t)(p & 0xFF);
        if ((c & 31) == 0) scales[o >> 5] = (uint8_t)sb;
      }
    } else if (live) {
      if (out_mode == 1)
        reinterpret_cast<uint16_t*>(out)[o] = f32_to_bf16(y);
      else
        reinterpret_cast<float*>(out)[o] = y;
    }
  }
}

// Layer 0, fast form for C = 64*CPL channels (CPL = 1, 2, 4, 8): lane l owns
// the CPL consecutive channels [l*CPL, l*CPL + CPL) with their K taps in
// registers, so every LayerNorm statistic is ONE wave reduction (DPP, no
// LDS, no barrier) and an MXFP8 block of 32 channels is 32/CPL lanes
// (group_max).  A 256-thread block owns FPW frames per wave; the window of
// samples all its frames touch is staged (normalised) in LDS once and read
// as broadcasts.  Each lane stores its CPL outputs of a frame as one 4-/8-B
// (MXFP8) or CPL*4-B (fp32) vector.
template <int CPL, int FPW, int KT>  // KT: compile-time tap count (0 = runtime K <= 16)
__global__ void __launch_bounds__(256) conv0_wave_kernel(const float* __restrict__ wav, const float* __restrict__ stats,
                                                         long long S, int T0, int K, int stride,
                                                         const float* __restrict__ w, const float* __restrict__ g,
                                                         const float* __restrict__ be, float eps,
                                                         void* __restrict__ out, int out_mode,
                                                         uint8_t* __restrict__ scales) {
  extern __shared__ __attribute__((aligned(16))) float xs[];
  constexpr int C = 64 * CPL, FPB = 4 * FPW;
  const int nblk_t = (T0 + FPB - 1) / FPB;
  const int b = blockIdx.x / nblk_t;
  const int t0 = (blockIdx.x - b * nblk_t) * FPB;
  const int nr = min(FPB, T0 - t0);
  const int win = (nr - 1) * stride + K;
  const float* x = wav + (long long)b * S + (long long)t0 * stride;
  const float mean = stats ? stats[2 * b] : 0.f, rstd = stats ? stats[2 * b + 1] : 1.f;
  for (int i = threadIdx.x; i < win; i += blockDim.x) xs[i] = (x[i] - mean) * rstd;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = lane * CPL;
  constexpr int KM = KT ? KT : 16;
  if (KT) K = KT;
  float wk[CPL][KM], gc[CPL], bc[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
#pragma unroll
    for (int k = 0; k < KM; ++k) wk[j][k] = k < K ? w[(c0 + j) * K + k] : 0.f;
    gc[j] = g[c0 + j];
    bc[j] = be[c0 + j];
  }
  __syncthreads();
  const float invC = 1.f / (float)C;
  for (int f = 0; f < FPW; ++f) {
    const int r = wv * FPW + f;
    if (r >= nr) break;
    const float* xr = xs + r * stride;
    float v[CPL];
#pragma unroll
    for (int j = 0; j < CPL; ++j) v[j] = 0.f;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (KT || k < K) {
        const float xv = xr[k];
#pragma unroll
        for (int j = 0; j < CPL; ++j) v[j] = fmaf(wk[j][k], xv, v[j]);
      }
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) s += v[j];
    const float mu = wave_sum_v(s) * invC;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const float d = v[j] - mu;
      q = fmaf(d, d, q);
    }
    const float rs = rsqrtf(wave_sum_v(q) * invC + eps);
    float y[CPL];
#pragma unroll
    for (int j = 0; j < CPL; ++j) y[j] = gelu_erf((v[j] - mu) * rs * gc[j] + bc[j]);
    const long long row = (long long)b * T0 + t0 + r;
    if (out_mode == 2) {
      float am = 0.f;
#pragma unroll
      for (int j = 0; j < CPL; ++j) am = fmaxf(am, fabsf(y[j]));
      am = group_max<32 / CPL>(am);
      const int sb = mx_scale_byte(am);
      const float inv = mx_inv_scale(sb);
      uint8_t* o = reinterpret_cast<uint8_t*>(out) + row * C + c0;
      if constexpr (CPL >= 4) {
#pragma unroll
        for (int j = 0; j < CPL; j += 4)
          *reinterpret_cast<uint32_t*>(o + j) = pack4_e4m3(y[j] * inv, y[j + 1] * inv, y[j + 2] * inv, y[j + 3] * inv);
      } else {
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
          const float qv = clamp_e4m3(y[j] * inv);
          o[j] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(qv, qv, 0, false) & 0xFF);
        }
      }
      if ((c0 & 31) == 0) scales[row * (C / 32) + (c0 >> 5)] = (uint8_t)sb;
    } else if (out_mode == 1) {
      uint16_t* o = reinterpret_cast<uint16_t*>(out) + row * C + c0;
#pragma unroll
      for (int j = 0; j < CPL; ++j) o[j] = f32_to_bf16(y[j]);
    } else {
      float* o = reinterpret_cast<float*>(out) + row * C + c0;
#pragma unroll
      for (int j = 0; j < CPL; ++j) o[j] = y[j];
    }
  }
}

// One wave per row of D = 64*V values; lane l owns the contiguous run
// [l*V, l*V + V).  ln: LayerNorm with g/b (g null → no LayerNorm);
// act 0 none, 3 relu, 4 gelu(erf).  in_bf16 selects the input type.
// out_mode 0 fp32, 1 bf16, 2 MXFP8 (+ scales, (M, D/32) bytes).
template <int V>
__global__ void __launch_bounds__(256) ln_act_kernel(const void* __restrict__ x, int in_bf16, long long ldx, int M,
                                                     const float* __restrict__ g, const float* __restrict__ be,
                                                     float eps, int act, void* __restrict__ out, long long ldo,
                                                     int out_mode, uint8_t* __restrict__ scales, long long lds) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int lane = threadIdx.x & 63;
  constexpr int D = 64 * V;
  float v[V];
  if (in_bf16) {
    const uint16_t* xr = reinterpret_cast<const uint16_t*>(x) + (long long)row * ldx + lane * V;
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = bf16_to_f32(xr[j]);
  } else {
    const float* xr = reinterpret_cast<const float*>(x) + (long long)row * ldx + lane * V;
    if constexpr (V % 4 == 0) {
#pragma unroll
      for (int j = 0; j < V; j += 4) {
        const float4 q = *reinterpret_cast<const float4*>(xr + j);
        v[j] = q.x; v[j + 1] = q.y; v[j + 2] = q.z; v[j + 3] = q.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] = xr[j];
    }
  }
  if (g) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) s += v[j];
    const float mu = wave_sum_v(s) * (1.f / (float)D);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float d = v[j] - mu;
      q = fmaf(d, d, q);
    }
    const float rs = rsqrtf(wave_sum_v(q) * (1.f / (float)D) + eps);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = lane * V + j;
      v[j] = (v[j] - mu) * rs * g[c] + be[c];
    }
  }
  if (act == 4) {
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = gelu_erf(v[j]);
  } else if (act == 3) {
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = fmaxf(v[j], 0.f);
  }
  if (out_mode == 2) {
    // blocks of 32: within a lane when V >= 32, else across 32/V lanes
    constexpr int NB = V >= 32 ? V / 32 : 1;
    constexpr int BL = V >= 32 ? 32 : V;  // values of one block held by this lane
    uint8_t* orow = reinterpret_cast<uint8_t*>(out) + (long long)row * ldo + lane * V;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      float am = 0.f;
#pragma unroll
      for (int j = 0; j < BL; ++j) am = fmaxf(am, fabsf(v[nb * BL + j]));
      if constexpr (V < 32) am = group_max<32 / V>(am);
      const int sb = mx_scale_byte(am);
      const float inv = mx_inv_scale(sb);
      if constexpr (BL >= 4) {
#pragma unroll
        for (int j = 0; j < BL; j += 4)
          *reinterpret_cast<uint32_t*>(orow + nb * BL + j) =
              pack4_e4m3(v[nb * BL + j] * inv, v[nb * BL + j + 1] * inv, v[nb * BL + j + 2] * inv,
                         v[nb * BL + j + 3] * inv);
      } else {
#pragma unroll
        for (int j = 0; j < BL; ++j) {
          const float q = clamp_e4m3(v[nb * BL + j] * inv);
          orow[nb * BL + j] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(q, q, 0, false) & 0xFF);
        }
      }
      const int col = lane * V + nb * BL;
      if ((col & 31) == 0) scales[(long long)row * lds + (col >> 5)] = (uint8_t)sb;
    }
  } else if (out_mode == 1) {
    uint16_t* orow = reinterpret_cast<uint16_t*>(out) + (long long)row * ldo + lane * V;
#pragma unroll
    for (int j = 0; j < V; ++j) orow[j] = f32_to_bf16(v[j]);
  } else {
    float* orow = reinterpret_cast<float*>(out) + (long long)row * ldo + lane * V;
#pragma unroll
    for (int j = 0; j < V; ++j) orow[j] = v[j];
  }
}

// Any D (fp32 / bf16 output): one wave per row, three passes over the row
// (sum, centred squares, write) — the small / odd widths of test configs.
__global__ void __launch_bounds__(256) ln_act_generic_kernel(const void* __restrict__ x, int in_bf16, long long ldx,
                                                             int M, int D, const float* __restrict__ g,
                                                             const float* __restrict__ be, float eps, int act,
                                                             void* __restrict__ out, long long ldo, int out_bf16) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int lane = threadIdx.x & 63;
  auto ld = [&](int c) {
    return in_bf16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(x)[(long long)row * ldx + c])
                   : reinterpret_cast<const float*>(x)[(long long)row * ldx + c];
  };
  float mu = 0.f, rs = 1.f;
  if (g) {
    float s = 0.f;
    for (int c = lane; c < D; c += 64) s += ld(c);
    mu = wave_sum_v(s) / (float)D;
    float q = 0.f;
    for (int c = lane; c < D; c += 64) {
      const float d = ld(c) - mu;
      q = fmaf(d, d, q);
    }
    rs = rsqrtf(wave_sum_v(q) / (float)D + eps);
  }
  for (int c = lane; c < D; c += 64) {
    float v = ld(c);
    if (g) v = (v - mu) * rs * g[c] + be[c];
    if (act == 4) v = gelu_erf(v);
    else if (act == 3) v = fmaxf(v, 0.f);
    if (out_bf16)
      reinterpret_cast<uint16_t*>(out)[(long long)row * ldo + c] = f32_to_bf16(v);
    else
      reinterpret_cast<float*>(out)[(long long)row * ldo + c] = v;
  }
}

template <int V>
int launch_ln_act(const void* x, int in_bf16, long long ldx, int M, const float* g, const float* be, float eps,
                  int act, void* out, long long ldo, int out_mode, uint8_t* scales, long long lds, hipStream_t s) {
  hipLaunchKernelGGL(ln_act_kernel<V>, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, s, x, in_bf16, ldx, M, g, be,
                     eps, act, out, ldo, out_mode, scales, lds);
  SBK_CHECK_LAUNCH();
  return 0;
}

}  // namespace

SBK_API int sbk_w2v_wav_stats(const float* wav, int B, long long S, float eps, float* stats, void* stream) {
  if (B <= 0 || S <= 0) return SBK_ERR_ARG;
  hipLaunchKernelGGL(wav_stats_kernel, dim3(B), dim3(1024), 0, (hipStream_t)stream, wav, S, eps, stats);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_w2v_conv0(const float* wav, const float* stats, int B, long long S, int T0, int C, int K, int stride,
                          const float* w, const float* g, const float* b, float eps, void* out, int out_mode,
                          uint8_t* scales, void* stream) {
  if (B <= 0 || S <= 0 || T0 <= 0 || C <= 0 || C > 1024 || K <= 0 || K > 16 || stride <= 0) return SBK_ERR_ARG;
  if ((long long)(T0 - 1) * stride + K > S) return SBK_ERR_ARG;
  if (out_mode == 2 && ((C % 32) || !scales)) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  constexpr int FPW = 32;  // frames per wave: weights loaded once per 128 frames
  if (C == 64 || C == 128 || C == 256 || C == 512) {
    const size_t lds = (size_t)((4 * FPW - 1) * stride + K) * sizeof(float);
    const long long nblk = (long long)B * ((T0 + 4 * FPW - 1) / (4 * FPW));
#define SBK_CONV0(CPL)                                                                                         \
  if (K == 11)                                                                                                   \
    hipLaunchKernelGGL((conv0_wave_kernel<CPL, FPW, 11>), dim3((unsigned)nblk), dim3(256), lds, s, wav, stats, S, \
                       T0, K, stride, w, g, b, eps, out, out_mode, scales);                                       \
  else                                                                                                           \
    hipLaunchKernelGGL((conv0_wave_kernel<CPL, FPW, 0>), dim3((unsigned)nblk), dim3(256), lds, s, wav, stats, S,  \
                       T0, K, stride, w, g, b, eps, out, out_mode, scales)
    if (C == 64) SBK_CONV0(1);
    else if (C == 128) SBK_CONV0(2);
    else if (C == 256) SBK_CONV0(4);
    else SBK_CONV0(8);
#undef SBK_CONV0
    SBK_CHECK_LAUNCH();
    return 0;
  }
  constexpr int R = 16;
  const int threads = ((C + 63) / 64) * 64;
  const size_t lds = (size_t)((R - 1) * stride + K) * sizeof(float);
  const long long nblk = (long long)B * ((T0 + R - 1) / R);
  hipLaunchKernelGGL(conv0_kernel<R>, dim3((unsigned)nblk), dim3(threads), lds, s, wav, stats, S,
                     T0, C, K, stride, w, g, b, eps, out, out_mode, scales);
  SBK_CHECK_LAUNCH();
  return 0;
}

// Row LayerNorm (g non-null) / activation / output conversion; MXFP8 output
// for D in {64, 128, ..., 4096}, fp32 / bf16 for any D; ld* in elements
// (scales: bytes).
SBK_API int sbk_ln_act(const void* x, int in_bf16, long long ldx, int M, int D, const float* g, const float* b,
                       float eps, int act, void* out, long long ldo, int out_mode, uint8_t* scales, long long lds,
                       void* stream) {
  if (M <= 0 || (out_mode == 2 && !scales)) return SBK_ERR_ARG;
  if (act != 0 && act != 3 && act != 4) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  switch (D) {
    case 64: return launch_ln_act<1>(x, in_bf16, ldx, M, g, b, eps, act, out, ldo, out_mode, scales, lds, s);
    case 128: return launch_ln_act<2>(x, in_bf16, ldx, M, g, b, eps, act, out, ldo, out_mode, scales, lds, s);
    case 256: return launch_ln_act<4>(x, in_bf16, ldx, M, g, b, eps, act, out, ldo, out_mode, scales, lds, s);
    case 512: return launch_ln_act<8>(x, in_bf16, ldx, M, g, b, eps, act, out, ldo, out_mode, scales, lds, s);
    case 1024: return launch_ln_act<16>(x, in_bf16, ldx, M, g, b, eps, act, out, ldo, out_mode, scales, lds, s);
    case 2048: return launch_ln_act<32>(x, in_bf16, ldx, M, g, b, eps, act, out, ldo, out_mode, scales, lds, s);
    case 4096: return launch_ln_act<64>(x, in_bf16, ldx, M, g, b, eps, act, out, ldo, out_mode, scales, lds, s);
    default:
      if (out_mode == 2 || D <= 0) return SBK_ERR_ARG;
      hipLaunchKernelGGL(ln_act_generic_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, s, x, in_bf16, ldx, M, D,
                         g, b, eps, act, out, ldo, out_mode == 1);
      SBK_CHECK_LAUNCH();
      return 0;
  }
}

// x[m, :] += pe[m % T, :] for x (M, D) fp32 in place (EncoderWrapper adds the
// positional table to every utterance, wav2vec.py:222).
namespace {
__global__ void add_rows_periodic_kernel(float* __restrict__ x, long long n, int D, const float* __restrict__ pe,
                                         int T) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / D;
    x[i] += pe[(row % T) * D + (i - row * D)];
  }
}
}  // namespace

SBK_API int sbk_add_rows_periodic(float* x, int M, int D, const float* pe, int T, void* stream) {
  if (M <= 0 || D <= 0 || T <= 0) return SBK_ERR_ARG;
  const long long n = (long long)M * D;
  long long g = (n + 255) / 256;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(add_rows_periodic_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, x, n, D, pe, T);
  SBK_CHECK_LAUNCH();
  return 0;
}
