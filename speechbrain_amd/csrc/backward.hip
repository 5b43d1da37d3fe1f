// Training-path kernels (backward of the Conformer-Transducer hot path).
//
// The forward inference path fuses aggressively (ffn.hip, attention.hip,
// conformer.hip).  Training needs the intermediate activations, so the
// autograd path (speechbrain_amd/_autograd.py) runs the same arithmetic as a
// chain of smaller launches and differentiates each:
//
//   LayerNorm backward            nn.LayerNorm (normalization.py:172-223), row
//                                 LNs of the Conformer and the (freq x chan)
//                                 LN of ConvBlock (convolution.py:169-175)
//   activations fwd/bwd           Swish (activations.py:111-142), GLU
//                                 (Conformer.py:73-79), LeakyReLU
//   depthwise conv fwd/bwd        Conformer.py:80-86,106
//   rel-pos softmax backward      attention.py:594-631 (softmax, rel_shift
//                                 :468-483 transposed into the band layout)
//   im2col / col2im (reflect)     Conv2d "same" reflect padding
//                                 (CNN.py:616-700) for the ConvBlock GEMMs
//   transducer joint fwd/bwd      transducer_joint.py:57-95 ("sum" + act)
//
// Dense contractions of the backward (dX = dY W, dW = dY^T X, the attention
// batched products) run on the MFMA GEMMs of gemm.hip / gemm_tn.hip;
// everything here is bandwidth-bound elementwise / reduction work: coalesced
// rows, one wave per row where a row reduction is needed, deterministic
// per-block partial sums (no float atomics) reduced by sbk_colsum.
#include "mfma.h"

#include <algorithm>
#include <initializer_list>

using namespace sbk;

namespace {

__device__ __forceinline__ float ldv(const void* p, long long i, int bf) {
  return bf ? bf16_to_f32(reinterpret_cast<const bf16_t*>(p)[i]) : reinterpret_cast<const float*>(p)[i];
}
__device__ __forceinline__ void stv(void* p, long long i, float v, int bf) {
  if (bf)
    reinterpret_cast<bf16_t*>(p)[i] = f32_to_bf16(v);
  else
    reinterpret_cast<float*>(p)[i] = v;
}

inline int grid_for(long long n, int block, int cap = 16384) {
  long long g = (n + block - 1) / block;
  return (int)(g > cap ? cap : (g < 1 ? 1 : g));
}

// ---------------------------------------------------------------- LayerNorm
// One wave per row (grid-stride over rows); lane owns columns lane + 64 i.
//   xhat = (x - mean) * rstd, gy = dy * g
//   dx   = rstd * (gy - mean(gy) - xhat * mean(gy * xhat))   (+ dres)
//   dg  += dy * xhat, db += dy     (per-block partials, rows fixed per block)
template <int PER>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const float* __restrict__ x, const void* __restrict__ dy,
                                                     int dy_bf16, int M, int D, const float* __restrict__ g,
                                                     float eps, const float* __restrict__ dres,
                                                     float* __restrict__ dx, float* __restrict__ part) {
  __shared__ float red[2 * 64 * PER];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float ag[PER], ab[PER], gg[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    ag[i] = 0.f;
    ab[i] = 0.f;
    gg[i] = c < D ? g[c] : 0.f;
  }
  const float invD = 1.0f / D;
  for (long long row = (long long)blockIdx.x * 4 + w; row < M; row += (long long)gridDim.x * 4) {
    const float* xr = x + row * D;
    float v[PER], d[PER];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      v[i] = c < D ? xr[c] : 0.f;
      d[i] = c < D ? ldv(dy, row * D + c, dy_bf16) : 0.f;
      s += v[i];
    }
    const float mean = wave_sum(s) * invD;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      const float t = c < D ? v[i] - mean : 0.f;
      q += t * t;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) * invD + eps);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      v[i] = (v[i] - mean) * rstd;  // xhat (0 beyond D since d == 0 there)
      const float gy = d[i] * gg[i];
      s1 += gy;
      s2 += gy * v[i];
      ag[i] += d[i] * v[i];
      ab[i] += d[i];
    }
    s1 = wave_sum(s1) * invD;
    s2 = wave_sum(s2) * invD;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      if (c < D) {
        float r = rstd * (d[i] * gg[i] - s1 - v[i] * s2);
        if (dres) r += dres[row * D + c];
        dx[row * D + c] = r;
      }
    }
  }
  if (!part) return;
  // waves add their column partials into one LDS slab in turn
  for (int ww = 0; ww < 4; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        red[lane + 64 * i] = ww ? red[lane + 64 * i] + ag[i] : ag[i];
        red[64 * PER + lane + 64 * i] = ww ? red[64 * PER + lane + 64 * i] + ab[i] : ab[i];
      }
    }
    __syncthreads();
  }
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    part[(long long)blockIdx.x * 2 * D + c] = red[c];
    part[(long long)blockIdx.x * 2 * D + D + c] = red[64 * PER + c];
  }
}

// Row LayerNorm forward for the wide (freq x channel) rows of ConvBlock
// (D up to 2560): one wave per row; y fp32 or bf16.
template <int PER>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const float* __restrict__ x, int M, int D,
                                                     const float* __restrict__ g, const float* __restrict__ b,
                                                     float eps, void* __restrict__ y, int y_bf16) {
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
  const float mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    const float t = c < D ? v[i] - mean : 0.f;
    q += t * t;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / D + eps);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    if (c < D) stv(y, row * D + c, (v[i] - mean) * rstd * g[c] + b[c], y_bf16);
  }
}

// Rows wider than 2560 (the default ConvolutionFrontEnd's first block:
// LayerNorm over 80 freq x 128 channels = 10240): one workgroup per row,
// three strided passes over the row (mean, variance, output) re-reading it
// from L2.
__global__ void __launch_bounds__(256) ln_fwd_row_kernel(const float* __restrict__ x, int M, int D,
                                                         const float* __restrict__ g, const float* __restrict__ b,
                                                         float eps, void* __restrict__ y, int y_bf16) {
  __shared__ float red[16];
  for (long long row = blockIdx.x; row < M; row += gridDim.x) {
    const float* xr = x + row * D;
    float s = 0.f;
    for (int c = threadIdx.x; c < D; c += blockDim.x) s += xr[c];
    const float mean = block_sum(s, red) / D;
    float q = 0.f;
    for (int c = threadIdx.x; c < D; c += blockDim.x) {
      const float t = xr[c] - mean;
      q += t * t;
    }
    const float rstd = 1.0f / sqrtf(block_sum(q, red) / D + eps);
    for (int c = threadIdx.x; c < D; c += blockDim.x) stv(y, row * D + c, (xr[c] - mean) * rstd * g[c] + b[c], y_bf16);
  }
}

// Backward of the wide rows: one workgroup per row (grid-stride), the
// per-workgroup [dgamma | dbeta] partials accumulated in LDS (2 D floats,
// dynamic) and written once, as ln_bwd_kernel's.
__global__ void __launch_bounds__(256) ln_bwd_row_kernel(const float* __restrict__ x, const void* __restrict__ dy,
                                                         int dy_bf16, int M, int D, const float* __restrict__ g,
                                                         float eps, const float* __restrict__ dres,
                                                         float* __restrict__ dx, float* __restrict__ part) {
  __shared__ float red[16];
  extern __shared__ float acc[];  // [dgamma (D) | dbeta (D)]
  for (int c = threadIdx.x; c < 2 * D; c += blockDim.x) acc[c] = 0.f;
  for (long long row = blockIdx.x; row < M; row += gridDim.x) {
    const float* xr = x + row * D;
    float s = 0.f;
    for (int c = threadIdx.x; c < D; c += blockDim.x) s += xr[c];
    const float mean = block_sum(s, red) / D;
    float q = 0.f;
    for (int c = threadIdx.x; c < D; c += blockDim.x) {
      const float t = xr[c] - mean;
      q += t * t;
    }
    const float rstd = 1.0f / sqrtf(block_sum(q, red) / D + eps);
    float s1 = 0.f, s2 = 0.f;
    for (int c = threadIdx.x; c < D; c += blockDim.x) {
      const float xh = (xr[c] - mean) * rstd, d = ldv(dy, row * D + c, dy_bf16), gy = d * g[c];
      s1 += gy;
      s2 += gy * xh;
      acc[c] += d * xh;  // each column owned by one thread: no LDS race
      acc[D + c] += d;
    }
    s1 = block_sum(s1, red) / D;
    s2 = block_sum(s2, red) / D;
    for (int c = threadIdx.x; c < D; c += blockDim.x) {
      const float xh = (xr[c] - mean) * rstd;
      float r = rstd * (ldv(dy, row * D + c, dy_bf16) * g[c] - s1 - xh * s2);
      if (dres) r += dres[row * D + c];
      dx[row * D + c] = r;
    }
  }
  if (!part) return;
  __syncthreads();  // acc[D + c] was written by another thread than the one storing it
  for (int c = threadIdx.x; c < 2 * D; c += blockDim.x) part[(long long)blockIdx.x * 2 * D + c] = acc[c];
}

// part[j, c] = sum of x[r, c] over rows r of chunk j (thread per column;
// 8 loads in flight per thread).
// Batched over grid.z: x (batch, rows, cols) -> part[j][z * cols + c], so
// one colsum over the chunks yields out[z * cols + c].
__global__ void rowsum_partial_kernel(const void* __restrict__ x, int x_bf16, long long rows, int cols, int rows_per,
                                      float* __restrict__ part) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  const int z = blockIdx.z;
  x = x_bf16 ? static_cast<const void*>(reinterpret_cast<const bf16_t*>(x) + (long long)z * rows * cols)
             : static_cast<const void*>(reinterpret_cast<const float*>(x) + (long long)z * rows * cols);
  part += (long long)z * cols;
  const int ldp = cols * gridDim.z;
  const long long r0 = (long long)blockIdx.x * rows_per;
  const long long r1 = min(r0 + rows_per, rows);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  long long r = r0;
  for (; r + 8 <= r1; r += 8) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = ldv(x, (r + i) * cols + c, x_bf16);
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i & 3] += v[i];
  }
  for (; r < r1; ++r) s[0] += ldv(x, r * cols + c, x_bf16);
  part[(long long)blockIdx.x * ldp + c] = (s[0] + s[1]) + (s[2] + s[3]);
}

// out[c] (+)= sum_r part[r, c] — deterministic column reduction.  A block
// covers 64 columns with 16 waves; wave w sums rows w, w + 16, ... and the 16
// wave partials are added in a fixed order.
__global__ void __launch_bounds__(1024) colsum_kernel(const float* __restrict__ part, int rows, int cols,
                                                      float* __restrict__ out, int accumulate) {
  __shared__ float red[16][65];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  // 8 independent loads in flight per trip (the partial rows are L2-resident)
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    int r = w;
    for (; r + 7 * 16 < rows; r += 8 * 16) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = part[(long long)(r + 16 * k) * cols + c];
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += v[k];
    }
    for (; r < rows; r += 16) s[0] += part[(long long)r * cols + c];
  }
  red[w][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (w == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][lane];
    out[c] = accumulate ? out[c] + t : t;
  }
}

// ------------------------------------------------------------- activations
// mode 1 Swish y = x sigmoid(x); 2 GLU y = a sigmoid(b), x = [a | b] (2 cols);
// 3 LeakyReLU(slope); 4 GELU y = x Φ(x) with the exact erf (torch.nn.GELU,
// the TransformerEncoder FFN's activation).  rows x cols outputs.
__device__ __forceinline__ float gelu_f(float v) { return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)); }
// d/dx x Φ(x) = Φ(x) + x φ(x)
__device__ __forceinline__ float gelu_d(float v) {
  return 0.5f * (1.0f + erff(v * 0.70710678118654752f)) + v * 0.39894228040143268f * expf(-0.5f * v * v);
}
__global__ void act_fwd_kernel(int mode, const void* __restrict__ x, int x_bf16, long long rows, int cols,
                               void* __restrict__ y, int y_bf16, float slope) {
  const long long n = rows * cols;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float r;
    if (mode == 2) {
      const long long row = i / cols, c = i - row * cols;
      const float a = ldv(x, row * 2 * cols + c, x_bf16), b = ldv(x, row * 2 * cols + cols + c, x_bf16);
      r = a * (1.0f / (1.0f + expf(-b)));
    } else {
      const float v = ldv(x, i, x_bf16);
      r = mode == 1 ? v * (1.0f / (1.0f + expf(-v))) : mode == 4 ? gelu_f(v) : (v >= 0.f ? v : v * slope);
    }
    stv(y, i, r, y_bf16);
  }
}

// Backward of act_fwd_kernel; dx has the shape of x (GLU: rows x 2 cols).
__global__ void act_bwd_kernel(int mode, const void* __restrict__ x, int x_bf16, const void* __restrict__ dy,
                               int dy_bf16, long long rows, int cols, void* __restrict__ dx, int dx_bf16,
                               float slope) {
  const long long n = rows * cols;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float g = ldv(dy, i, dy_bf16);
    if (mode == 2) {
      const long long row = i / cols, c = i - row * cols;
      const long long ia = row * 2 * cols + c, ib = ia + cols;
      const float a = ldv(x, ia, x_bf16), b = ldv(x, ib, x_bf16);
      const float s = 1.0f / (1.0f + expf(-b));
      stv(dx, ia, g * s, dx_bf16);
      stv(dx, ib, g * a * s * (1.0f - s), dx_bf16);
    } else if (mode == 1) {
      const float v = ldv(x, i, x_bf16);
      const float s = 1.0f / (1.0f + expf(-v));
      stv(dx, i, g * (s + v * s * (1.0f - s)), dx_bf16);
    } else if (mode == 4) {
      stv(dx, i, g * gelu_d(ldv(x, i, x_bf16)), dx_bf16);
    } else {
      const float v = ldv(x, i, x_bf16);
      stv(dx, i, v > 0.f ? g : g * slope, dx_bf16);
    }
  }
}

// 4-wide variants (16-B fp32 / 8-B bf16 accesses) for n % 4 == 0 (GLU:
// cols % 4 == 0) and aligned pointers — the per-element kernels above issue
// one 2- or 4-byte access per lane and ran at a third of HBM bandwidth.
__device__ __forceinline__ float4 ld4(const void* p, long long i, int bf) {
  if (bf) {
    const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(p) + i);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                       __uint_as_float(u.y & 0xffff0000u));
  }
  return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + i);
}
__device__ __forceinline__ void st4(void* p, long long i, float4 v, int bf) {
  if (bf) {
    uint2 u;
    u.x = pack_bf16x2(v.x, v.y);
    u.y = pack_bf16x2(v.z, v.w);
    *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p) + i) = u;
  } else {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(p) + i) = v;
  }
}
__device__ __forceinline__ float sigm(float v) { return 1.0f / (1.0f + expf(-v)); }

template <int MODE>
__global__ void act_fwd4_kernel(const void* __restrict__ x, int x_bf16, long long rows, int cols,
                                void* __restrict__ y, int y_bf16, float slope) {
  const long long n4 = rows * cols / 4;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (long long)gridDim.x * blockDim.x) {
    const long long i = 4 * q;
    float4 r;
    if (MODE == 2) {
      const long long row = i / cols, c = i - row * cols;
      const float4 a = ld4(x, row * 2 * cols + c, x_bf16), b = ld4(x, row * 2 * cols + cols + c, x_bf16);
      r = make_float4(a.x * sigm(b.x), a.y * sigm(b.y), a.z * sigm(b.z), a.w * sigm(b.w));
    } else {
      const float4 v = ld4(x, i, x_bf16);
      if (MODE == 1) r = make_float4(v.x * sigm(v.x), v.y * sigm(v.y), v.z * sigm(v.z), v.w * sigm(v.w));
      else r = make_float4(v.x >= 0.f ? v.x : v.x * slope, v.y >= 0.f ? v.y : v.y * slope,
                           v.z >= 0.f ? v.z : v.z * slope, v.w >= 0.f ? v.w : v.w * slope);
    }
    st4(y, i, r, y_bf16);
  }
}

template <int MODE>
__global__ void act_bwd4_kernel(const void* __restrict__ x, int x_bf16, const void* __restrict__ dy, int dy_bf16,
                                long long rows, int cols, void* __restrict__ dx, int dx_bf16, float slope) {
  const long long n4 = rows * cols / 4;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (long long)gridDim.x * blockDim.x) {
    const long long i = 4 * q;
    const float4 g = ld4(dy, i, dy_bf16);
    if (MODE == 2) {
      const long long row = i / cols, c = i - row * cols;
      const long long ia = row * 2 * cols + c, ib = ia + cols;
      const float4 a = ld4(x, ia, x_bf16), b = ld4(x, ib, x_bf16);
      const float4 sg = make_float4(sigm(b.x), sigm(b.y), sigm(b.z), sigm(b.w));
      st4(dx, ia, make_float4(g.x * sg.x, g.y * sg.y, g.z * sg.z, g.w * sg.w), dx_bf16);
      st4(dx, ib,
          make_float4(g.x * a.x * sg.x * (1.0f - sg.x), g.y * a.y * sg.y * (1.0f - sg.y),
                      g.z * a.z * sg.z * (1.0f - sg.z), g.w * a.w * sg.w * (1.0f - sg.w)),
          dx_bf16);
    } else {
      const float4 v = ld4(x, i, x_bf16);
      float4 r;
      if (MODE == 1) {
        const float4 sg = make_float4(sigm(v.x), sigm(v.y), sigm(v.z), sigm(v.w));
        r = make_float4(g.x * (sg.x + v.x * sg.x * (1.0f - sg.x)), g.y * (sg.y + v.y * sg.y * (1.0f - sg.y)),
                        g.z * (sg.z + v.z * sg.z * (1.0f - sg.z)), g.w * (sg.w + v.w * sg.w * (1.0f - sg.w)));
      } else {
        r = make_float4(v.x > 0.f ? g.x : g.x * slope, v.y > 0.f ? g.y : g.y * slope,
                        v.z > 0.f ? g.z : g.z * slope, v.w > 0.f ? g.w : g.w * slope);
      }
      st4(dx, i, r, dx_bf16);
    }
  }
}

inline bool vec4_ok(long long rows, int cols, int mode, std::initializer_list<const void*> ps) {
  if (cols % 4 || (rows * cols) % 4) return false;
  for (const void* p : ps)
    if (reinterpret_cast<uintptr_t>(p) & 15) return false;
  return mode >= 1 && mode <= 3;
}

// ------------------------------------------------------- depthwise conv1d
// Register-window kernels: a thread owns one channel c of one utterance b
// and a run of DW_RUN consecutive frames; the 31-tap window of x slides
// through VGPRs (one load per output instead of K).  Taps beyond K are zero,
// so one KMAX = 31 instantiation serves every K <= 31.
//   y[b, t, c] = bias[c] + sum_k w[c, k] x[b, t + k - padL, c]   (zero padding)
constexpr int DW_KMAX = 31;
constexpr int DW_RUN = 32;

__global__ void __launch_bounds__(256) dwconv_fwd_kernel(const void* __restrict__ x, int x_bf16, int B, int T, int C,
                                                         const float* __restrict__ w, const float* __restrict__ bias,
                                                         int K, int padL, int reverse, void* __restrict__ y,
                                                         int y_bf16) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int nrun = (T + DW_RUN - 1) / DW_RUN;
  const int b = blockIdx.y / nrun, t0 = (blockIdx.y % nrun) * DW_RUN;
  if (c >= C) return;
  float wk[DW_KMAX], win[DW_KMAX];
#pragma unroll
  for (int k = 0; k < DW_KMAX; ++k) wk[k] = k < K ? w[c * K + (reverse ? K - 1 - k : k)] : 0.f;
  const long long base = (long long)b * T * C + c;
  // the run's whole input window (DW_RUN + K - 1 frames) is loaded up front:
  // one load per frame inside the loop put a memory latency on every output
  // (46 us for 32 x 376 x 256); same summation order as before
  (void)win;
  const int t1 = min(t0 + DW_RUN, T);
  const int nin = t1 - t0 + K - 1;
  float xin[DW_RUN + DW_KMAX - 1];
#pragma unroll
  for (int i = 0; i < DW_RUN + DW_KMAX - 1; ++i) {
    const int ts = t0 + i - padL;
    xin[i] = (i < nin && ts >= 0 && ts < T) ? ldv(x, base + (long long)ts * C, x_bf16) : 0.f;
  }
  const float b0 = bias ? bias[c] : 0.f;
#pragma unroll
  for (int j = 0; j < DW_RUN; ++j) {
    if (t0 + j >= t1) break;  // uniform
    float s = b0;
#pragma unroll
    for (int k = 0; k < DW_KMAX; ++k) s += wk[k] * xin[j + k];
    stv(y, base + (long long)(t0 + j) * C, s, y_bf16);
  }
}

// Per-run partial weight / bias gradients: part (B * nrun, C, K + 1) of
// [dw taps | dbias], dw[c, k] = sum_t dy[b, t, c] x[b, t + k - padL, c].
__global__ void __launch_bounds__(256) dwconv_wgrad_kernel(const void* __restrict__ x, int x_bf16,
                                                           const float* __restrict__ dy, int B, int T, int C, int K,
                                                           int padL, float* __restrict__ part) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int nrun = (T + DW_RUN - 1) / DW_RUN;
  const int b = blockIdx.y / nrun, t0 = (blockIdx.y % nrun) * DW_RUN;
  if (c >= C) return;
  float acc[DW_KMAX + 1], win[DW_KMAX];
#pragma unroll
  for (int k = 0; k <= DW_KMAX; ++k) acc[k] = 0.f;
  const long long base = (long long)b * T * C + c;
  // (loading the run's whole window and dy up front, as the forward does,
  // measured 110 vs 61 us here: kept per frame)
#pragma unroll
  for (int k = 0; k < DW_KMAX - 1; ++k) {
    const int ts = t0 + k - padL;
    win[k] = (k < K - 1 && ts >= 0 && ts < T) ? ldv(x, base + (long long)ts * C, x_bf16) : 0.f;
  }
  const int t1 = min(t0 + DW_RUN, T);
  for (int t = t0; t < t1; ++t) {
    const int ts = t + K - 1 - padL;
    win[DW_KMAX - 1] = 0.f;
#pragma unroll
    for (int k = 0; k < DW_KMAX; ++k)
      if (k == K - 1) win[k] = (ts >= 0 && ts < T) ? ldv(x, base + (long long)ts * C, x_bf16) : 0.f;
    const float g = dy[base + (long long)t * C];
    acc[DW_KMAX] += g;
#pragma unroll
    for (int k = 0; k < DW_KMAX; ++k) acc[k] += g * win[k];
#pragma unroll
    for (int k = 0; k < DW_KMAX - 1; ++k) win[k] = win[k + 1];
  }
  float* p = part + ((long long)blockIdx.y * C + c) * (K + 1);
#pragma unroll
  for (int k = 0; k < DW_KMAX; ++k)
    if (k < K) p[k] = acc[k];
  p[K] = acc[DW_KMAX];
}

// ------------------------------------------- ConvBlock im2col / col2im
// Conv2d with "same" reflect padding (CNN.py:616-700, get_padding_elem
// :1459-1481: (k - 1) / 2 each side for odd k) and any stride: x (B, Ti,
// Fi, Ci) -> col (B*To*Fo, kt*kf*Ci) with column order (time tap, freq
// tap, ci) — the (Cout, kT, kF, Ci) weight permutation.  pt / pf < Ti / Fi
// (one reflection).
struct ConvGeom {
  int kt, kf, st, sf, pt, pf;
};

__device__ __forceinline__ int reflect_idx(int s, int n) {  // unpadded index of padded-minus-pad s
  return s < 0 ? -s : (s >= n ? 2 * n - 2 - s : s);
}

__global__ void im2col_kernel(const void* __restrict__ x, int x_bf16, int B, int Ti, int Fi, int Ci, int To, int Fo,
                              ConvGeom gm, int ldcol, void* __restrict__ col, int col_bf16) {
  const long long n = (long long)B * To * Fo * ldcol;
  const int kcols = gm.kt * gm.kf * Ci;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int kk = (int)(i % ldcol);
    long long q = i / ldcol;
    if (kk >= kcols) {  // K padding up to the GEMM's vector width
      stv(col, i, 0.f, col_bf16);
      continue;
    }
    const int ci = kk % Ci;
    const int kf = (kk / Ci) % gm.kf;
    const int kt = kk / (gm.kf * Ci);
    const int fo = (int)(q % Fo); q /= Fo;
    const int to = (int)(q % To);
    const int b = (int)(q / To);
    const int ti = reflect_idx(to * gm.st + kt - gm.pt, Ti), fi = reflect_idx(fo * gm.sf + kf - gm.pf, Fi);
    stv(col, i, ldv(x, (((long long)b * Ti + ti) * Fi + fi) * Ci + ci, x_bf16), col_bf16);
  }
}

// padded positions p (0 <= p < n + 2 pad) whose reflection is index i: the
// direct one and up to two mirrored ones; returns their count
__device__ __forceinline__ int reflect_sources(int i, int n, int pad, int* p) {
  int k = 0;
  p[k++] = i + pad;
  if (i >= 1 && i <= pad) p[k++] = pad - i;                           // s = -i
  if (i <= n - 2 && 2 * n - 2 - i <= n - 1 + pad) p[k++] = 2 * n - 2 - i + pad;  // s = 2n - 2 - i
  return k;
}

// dx[b, ti, fi, ci] = sum of dcol over the (output position, tap) pairs
// whose padded input position reflects onto (ti, fi): the adjoint of
// im2col, as a gather (deterministic).
__global__ void col2im_kernel(const void* __restrict__ dcol, int dcol_bf16, int B, int Ti, int Fi, int Ci, int To,
                              int Fo, ConvGeom gm, int ldcol, void* __restrict__ dx, int dx_bf16) {
  const long long n = (long long)B * Ti * Fi * Ci;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % Ci);
    long long q = i / Ci;
    const int fi = (int)(q % Fi); q /= Fi;
    const int ti = (int)(q % Ti);
    const int b = (int)(q / Ti);
    int pts[3], pfs[3];
    const int npt = reflect_sources(ti, Ti, gm.pt, pts), npf = reflect_sources(fi, Fi, gm.pf, pfs);
    float s = 0.f;
    for (int a = 0; a < npt; ++a)
      for (int kt = 0; kt < gm.kt; ++kt) {
        const int d = pts[a] - kt;
        if (d < 0 || d % gm.st) continue;
        const int to = d / gm.st;
        if (to >= To) continue;
        for (int e = 0; e < npf; ++e)
          for (int kf = 0; kf < gm.kf; ++kf) {
            const int df = pfs[e] - kf;
            if (df < 0 || df % gm.sf) continue;
            const int fo = df / gm.sf;
            if (fo >= Fo) continue;
            s += ldv(dcol, (((long long)b * To + to) * Fo + fo) * ldcol + (kt * gm.kf + kf) * Ci + ci, dcol_bf16);
          }
      }
    stv(dx, i, s, dx_bf16);
  }
}

// ------------------------------------------------- transducer joint ("sum")
// z[b, t, u, :] = act(tn[b, t, :] + pn[b, u, :]); act 0 none, 3 LeakyReLU,
// 5 tanh, 6 ReLU.  Rows of J contiguous; out fp32 or bf16.
__device__ __forceinline__ float joint_act(int act, float v, float slope) {
  if (act == 3) return v >= 0.f ? v : v * slope;
  if (act == 5) return tanhf(v);
  if (act == 6) return v > 0.f ? v : 0.f;
  return v;
}
__device__ __forceinline__ float joint_dact(int act, float v, float slope) {
  if (act == 3) return v > 0.f ? 1.f : slope;
  if (act == 5) { const float t = tanhf(v); return 1.f - t * t; }
  if (act == 6) return v > 0.f ? 1.f : 0.f;
  return 1.f;
}

// z[b, t, u, :] for all u of one (b, t): block per (b, t), thread per 4
// columns (float4 tn/pn loads, 8/16-byte stores); tn read once per (b, t).
__global__ void __launch_bounds__(256) joint_fwd_kernel(const float* __restrict__ tn, const float* __restrict__ pn,
                                                        int T, int U1, int J, int act, float slope,
                                                        void* __restrict__ z, int z_bf16) {
  const long long bt = blockIdx.x;
  const int b = (int)(bt / T);
  for (int j = threadIdx.x * 4; j < J; j += blockDim.x * 4) {
    const float4 a = *reinterpret_cast<const float4*>(tn + bt * J + j);
    for (int u = 0; u < U1; ++u) {
      const float4 c = *reinterpret_cast<const float4*>(pn + ((long long)b * U1 + u) * J + j);
      const float v0 = joint_act(act, a.x + c.x, slope), v1 = joint_act(act, a.y + c.y, slope);
      const float v2 = joint_act(act, a.z + c.z, slope), v3 = joint_act(act, a.w + c.w, slope);
      const long long o = (bt * U1 + u) * J + j;
      if (z_bf16) {
        uint2 q;
        q.x = (unsigned)f32_to_bf16(v0) | ((unsigned)f32_to_bf16(v1) << 16);
        q.y = (unsigned)f32_to_bf16(v2) | ((unsigned)f32_to_bf16(v3) << 16);
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(z) + o) = q;
      } else {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(z) + o) = make_float4(v0, v1, v2, v3);
      }
    }
  }
}

// Scalar variants for J not a multiple of the vector width.
__global__ void joint_fwd_scalar_kernel(const float* __restrict__ tn, const float* __restrict__ pn, int T, int U1,
                                        int J, int act, float slope, void* __restrict__ z, int z_bf16) {
  const long long bt = blockIdx.x;
  const int b = (int)(bt / T);
  for (int j = threadIdx.x; j < J; j += blockDim.x) {
    const float a = tn[bt * J + j];
    for (int u = 0; u < U1; ++u)
      stv(z, (bt * U1 + u) * J + j, joint_act(act, a + pn[((long long)b * U1 + u) * J + j], slope), z_bf16);
  }
}

__global__ void joint_bwd_scalar_kernel(const float* __restrict__ tn, const float* __restrict__ pn,
                                        const void* __restrict__ dz, int dz_bf16, int T, int U1, int J, int act,
                                        float slope, float* __restrict__ dtn, float* __restrict__ part, int B) {
  const long long bt = blockIdx.x;  // part: (T, B, U1, J) — one run per frame
  const int b = (int)(bt / T), t = (int)(bt % T);
  for (int j = threadIdx.x; j < J; j += blockDim.x) {
    const float a = tn[bt * J + j];
    float s = 0.f;
    for (int u = 0; u < U1; ++u) {
      const float g = ldv(dz, (bt * U1 + u) * J + j, dz_bf16) * joint_dact(act, a + pn[((long long)b * U1 + u) * J + j], slope);
      s += g;
      part[(((long long)t * B + b) * U1 + u) * J + j] = g;
    }
    dtn[bt * J + j] = s;
  }
}

// Joint backward, dz read once: block per (b, run of JB_T frames, 512
// columns); thread per 2 columns keeps tn and dtn of its JB_T frames in
// VGPRs and loops u: dtn[b, t, :] = sum_u dz act'(.) (complete), and the
// run's partial dpn[b, u, :] = sum_{t in run} dz act'(.) -> part (nrun, B, U1, J).
constexpr int JB_T = 16;
__global__ void __launch_bounds__(256) joint_bwd_kernel(const float* __restrict__ tn, const float* __restrict__ pn,
                                                        const void* __restrict__ dz, int dz_bf16, int B, int T, int U1,
                                                        int J, int act, float slope, float* __restrict__ dtn,
                                                        float* __restrict__ part) {
  const int nrun = (T + JB_T - 1) / JB_T;
  const int b = blockIdx.y / nrun, run = blockIdx.y % nrun, t0 = run * JB_T;
  const int j = (blockIdx.x * blockDim.x + threadIdx.x) * 2;
  if (j >= J) return;
  const int nt = min(JB_T, T - t0);
  float a0[JB_T], a1[JB_T], d0[JB_T], d1[JB_T];
#pragma unroll
  for (int i = 0; i < JB_T; ++i) {
    const bool ok = i < nt;
    const long long r = ((long long)b * T + t0 + (ok ? i : 0)) * J + j;
    const float2 v = *reinterpret_cast<const float2*>(tn + r);
    a0[i] = v.x;
    a1[i] = v.y;
    d0[i] = 0.f;
    d1[i] = 0.f;
  }
  for (int u = 0; u < U1; ++u) {
    const float2 c = *reinterpret_cast<const float2*>(pn + ((long long)b * U1 + u) * J + j);
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int i = 0; i < JB_T; ++i) {
      if (i < nt) {
        const long long o = (((long long)b * T + t0 + i) * U1 + u) * J + j;
        float g0, g1;
        if (dz_bf16) {
          const unsigned q = *reinterpret_cast<const unsigned*>(reinterpret_cast<const bf16_t*>(dz) + o);
          g0 = bf16_to_f32((bf16_t)(q & 0xffffu));
          g1 = bf16_to_f32((bf16_t)(q >> 16));
        } else {
          const float2 q = *reinterpret_cast<const float2*>(reinterpret_cast<const float*>(dz) + o);
          g0 = q.x;
          g1 = q.y;
        }
        g0 *= joint_dact(act, a0[i] + c.x, slope);
        g1 *= joint_dact(act, a1[i] + c.y, slope);
        d0[i] += g0;
        d1[i] += g1;
        s0 += g0;
        s1 += g1;
      }
    }
    *reinterpret_cast<float2*>(part + (((long long)run * B + b) * U1 + u) * J + j) = make_float2(s0, s1);
  }
#pragma unroll
  for (int i = 0; i < JB_T; ++i)
    if (i < nt) *reinterpret_cast<float2*>(dtn + ((long long)b * T + t0 + i) * J + j) = make_float2(d0[i], d1[i]);
}

// ------------------------------------------------ dropout / residual add
// Counter-based keep mask: bit-identical for the forward and the backward
// launch of one (seed, element) pair, independent of grid shape.
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ bool keep_elem(unsigned long long seed, long long i, unsigned thresh) {
  return (unsigned)(mix64(seed + (unsigned long long)i * 0x9E3779B97F4A7C15ull) >> 40) < thresh;
}

// out = res + alpha * rowmask0(drop(x)); drop(x) = keep ? x / (1 - p) : 0.
// The backward of this op is the same launch on dy with res = null.
__global__ void dropout_add_kernel(const void* __restrict__ x, int x_bf16, const float* __restrict__ res,
                                   long long rows, int cols, const unsigned char* __restrict__ rowmask, float alpha,
                                   unsigned thresh, float inv_keep, unsigned long long seed, int use_drop,
                                   void* __restrict__ out, int out_bf16) {
  const long long n = rows * cols;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float v = ldv(x, i, x_bf16) * alpha;
    if (use_drop) v = keep_elem(seed, i, thresh) ? v * inv_keep : 0.f;
    if (rowmask && rowmask[i / cols]) v = 0.f;
    if (res) v += res[i];
    stv(out, i, v, out_bf16);
  }
}

// 4 consecutive elements per thread (same keep hash per element index as
// dropout_add_kernel, so the masks are identical); cols % 4 == 0, aligned.
__global__ void dropout_add4_kernel(const void* __restrict__ x, int x_bf16, const float* __restrict__ res,
                                    long long rows, int cols, const unsigned char* __restrict__ rowmask, float alpha,
                                    unsigned thresh, float inv_keep, unsigned long long seed, int use_drop,
                                    void* __restrict__ out, int out_bf16) {
  const long long n4 = rows * cols / 4;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (long long)gridDim.x * blockDim.x) {
    const long long i = 4 * q;
    float4 v = ld4(x, i, x_bf16);
    float e[4] = {v.x * alpha, v.y * alpha, v.z * alpha, v.w * alpha};
    if (use_drop) {
#pragma unroll
      for (int k = 0; k < 4; ++k) e[k] = keep_elem(seed, i + k, thresh) ? e[k] * inv_keep : 0.f;
    }
    if (rowmask && rowmask[i / cols]) e[0] = e[1] = e[2] = e[3] = 0.f;
    if (res) {
      const float4 r = *reinterpret_cast<const float4*>(res + i);
      e[0] += r.x;
      e[1] += r.y;
      e[2] += r.z;
      e[3] += r.w;
    }
    st4(out, i, make_float4(e[0], e[1], e[2], e[3]), out_bf16);
  }
}

// ------------------------------------------ rel-pos attention backward
// The per-(utterance, head) products of the backward run on the MFMA GEMMs
// (sbk_gemm_batched, sbk_gemm_tn{,_f32}), whose operands need 16-B rows.  So
// every per-(b, h) operand is laid out over Tp = T rounded up to 8 rows and
// dhp = dh rounded up to 8 columns, zero-filled: the padded rows / columns
// add nothing to any product, and any T or head size takes the same kernels.
// Storage is bf16 or fp32 (`bf`), the compute dtype of the step.

// Operands from the in_proj output (and dO) of one (b, h) and 64 frames, in
// two coalesced phases through an LDS tile:
//   phase 1 (lanes along d): qu = q + pos_bias_u, v, dO  (B*H, Tp, dhp) and
//           qv = q + pos_bias_v head-major (H, B*T, dhp);
//   phase 2 (lanes along t): kT, vT (B*H, dhp, Tp).
// Bias sums in fp32 rounded once to the storage type (torch autocast adds
// the fp32 parameter to the bf16 projection in fp32 and rounds the sum at
// the next matmul).  Any output may be null.
__global__ void __launch_bounds__(256) attn_prep_kernel(const void* __restrict__ qkv, const void* __restrict__ dO,
                                                        const float* __restrict__ pbu, const float* __restrict__ pbv,
                                                        int B, int H, int T, int dh, int Tp, int dhp, int bf,
                                                        void* __restrict__ qu, void* __restrict__ qv,
                                                        void* __restrict__ kT, void* __restrict__ vo,
                                                        void* __restrict__ vT, void* __restrict__ doh) {
  __shared__ float tk[64][65], tv[64][65];
  const int t0 = blockIdx.x * 64, bh = blockIdx.y, d0 = blockIdx.z * 64;
  const int b = bh / H, h = bh - b * H, tid = threadIdx.x;
  {
    const int d = d0 + (tid & 63);
    const bool dv = d < dh;
#pragma unroll 4
    for (int k = 0; k < 16; ++k) {
      const int tl = (tid >> 6) + 4 * k, t = t0 + tl;
      if (t >= Tp || d >= dhp) continue;
      const bool ok = dv && t < T;
      const long long src = (((long long)b * T + t) * H + h) * 3 * dh + d;
      const float q = ok ? ldv(qkv, src, bf) : 0.f;
      const float kk = ok ? ldv(qkv, src + dh, bf) : 0.f;
      const float vv = ok ? ldv(qkv, src + 2 * dh, bf) : 0.f;
      const long long o = ((long long)bh * Tp + t) * dhp + d;
      if (qu) stv(qu, o, ok ? q + pbu[h * dh + d] : 0.f, bf);
      if (vo) stv(vo, o, vv, bf);
      if (doh) stv(doh, o, ok ? ldv(dO, (((long long)b * T + t) * H + h) * dh + d, bf) : 0.f, bf);
      if (qv && t < T) stv(qv, ((long long)h * B * T + (long long)b * T + t) * dhp + d, dv ? q + pbv[h * dh + d] : 0.f, bf);
      tk[tl][tid & 63] = kk;
      tv[tl][tid & 63] = vv;
    }
  }
  if (!kT && !vT) return;  // uniform
  __syncthreads();
  const int t = t0 + (tid & 63);
  if (t >= Tp) return;
#pragma unroll 4
  for (int k = 0; k < 16; ++k) {
    const int dl = (tid >> 6) + 4 * k, d = d0 + dl;
    if (d >= dhp) break;
    const long long o = ((long long)bh * dhp + d) * Tp + t;
    if (kT) stv(kT, o, tk[tid & 63][dl], bf);
    if (vT) stv(vT, o, tv[tid & 63][dl], bf);
  }
}

// pkT (H, dhp, Wp) = the linear_pos output pk (W, ldp) per head, transposed
// (W = 2T-1 relative offsets, Wp rounded up to 8), zero-padded.
__global__ void __launch_bounds__(256) attn_pkT_kernel(const void* __restrict__ pk, int ldp, int H, int dh, int W,
                                                       int Wp, int dhp, int bf, void* __restrict__ pkT) {
  __shared__ float tile[64][65];
  const int w0 = blockIdx.x * 64, h = blockIdx.y, d0 = blockIdx.z * 64, tid = threadIdx.x;
  {
    const int d = d0 + (tid & 63);
#pragma unroll 4
    for (int k = 0; k < 16; ++k) {
      const int wl = (tid >> 6) + 4 * k, w = w0 + wl;
      tile[wl][tid & 63] = (w < W && d < dh) ? ldv(pk, (long long)w * ldp + h * dh + d, bf) : 0.f;
    }
  }
  __syncthreads();
  const int w = w0 + (tid & 63);
  if (w >= Wp) return;
#pragma unroll 4
  for (int k = 0; k < 16; ++k) {
    const int dl = (tid >> 6) + 4 * k, d = d0 + dl;
    if (d >= dhp) break;
    stv(pkT, ((long long)h * dhp + d) * Wp + w, tile[tid & 63][dl], bf);
  }
}

// Softmax / dropout / rel_shift backward, one wave per padded score row
// (b, h, i < Tp).  P (B, H, T, T) fp32 probabilities (before dropout), dP =
// dO V^T over the padded rows (B*H, Tp, Tp), D = the dropout scale of each
// probability (keep(seed, index of P) / (1 - p), regenerated — the forward's
// sbk_dropout_add mask), attention.py:594-631:
//   Pd = D P                                  (the operand of dV = Pd^T dO)
//   dS = scale * P (D dP - sum_j P D dP)      (B*H, Tp, Tp)
//   dBD[i, T-1-i+j] = dS[i, j]                (rel_shift :468-483 transposed)
// dBD head-major (H, B*T, Wp), zero outside the band; padded rows / columns
// of Pd and dS are zero.
__global__ void __launch_bounds__(256) relpos_softmax_bwd_pad_kernel(
    const float* __restrict__ P, const void* __restrict__ dP, float scale, int B, int H, int T, int Tp, int Wp,
    unsigned thresh, float inv_keep, unsigned long long seed, int use_drop, void* __restrict__ dS,
    void* __restrict__ Pd, void* __restrict__ dBD, int bf) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long long)B * H * Tp) return;  // whole wave; no barrier below
  const int lane = threadIdx.x & 63;
  const long long bh = row / Tp;
  const int i = (int)(row - bh * Tp);
  const long long so = row * Tp;
  if (i >= T) {
    for (int j = lane; j < Tp; j += 64) {
      stv(dS, so + j, 0.f, bf);
      stv(Pd, so + j, 0.f, bf);
    }
    return;
  }
  const long long pi = (bh * T + i) * T;  // P row; the dropout index base
  const float* pr = P + pi;
  auto dscale = [&](int j) __attribute__((always_inline)) {
    return use_drop ? (keep_elem(seed, pi + j, thresh) ? inv_keep : 0.f) : 1.f;
  };
  float s = 0.f;
  for (int j = lane; j < T; j += 64) s += pr[j] * dscale(j) * ldv(dP, so + j, bf);
  s = wave_sum_v(s);
  for (int j = lane; j < Tp; j += 64) {
    float pd = 0.f, ds = 0.f;
    if (j < T) {
      const float p = pr[j], dd = dscale(j);
      pd = p * dd;
      ds = scale * p * (dd * ldv(dP, so + j, bf) - s);
    }
    stv(Pd, so + j, pd, bf);
    stv(dS, so + j, ds, bf);
  }
  const int h = (int)(bh % H), b = (int)(bh / H);
  const long long bo = (((long long)h * B + b) * T + i) * Wp;
  const int W = 2 * T - 1;
  for (int r = lane; r < Wp; r += 64) {
    const int j = r - (T - 1 - i);
    float v = 0.f;
    if (r < W && j >= 0 && j < T) v = scale * pr[j] * (dscale(j) * ldv(dP, so + j, bf) - s);
    stv(dBD, bo + r, v, bf);
  }
}

// Forward attention dropout (attention.py:626): attn = D P (fp32 (B, H, T, T),
// the module's returned weights; may be null) and the same values over the
// padded rows (B*H, Tp, Tp) in the compute dtype — the A operand of
// drop(P) V on sbk_gemm_batched.  Same mask as sbk_dropout_add on P.
__global__ void attn_probs_pad_kernel(const float* __restrict__ P, long long BH, int T, int Tp, unsigned thresh,
                                      float inv_keep, unsigned long long seed, int use_drop, float* __restrict__ attn,
                                      void* __restrict__ Pd, int bf) {
  const long long n = BH * Tp * Tp;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(e % Tp);
    const long long r = e / Tp;
    const int i = (int)(r % Tp);
    const long long bh = r / Tp;
    float v = 0.f;
    if (i < T && j < T) {
      const long long idx = (bh * T + i) * T + j;
      v = P[idx];
      if (use_drop) v = keep_elem(seed, idx, thresh) ? v * inv_keep : 0.f;
      if (attn) attn[idx] = v;
    }
    stv(Pd, e, v, bf);
  }
}

// dqkv (B*T, H*3*dh) in the in_proj layout (b, t, h, {q,k,v}, d) from the
// per-(b, h) products over padded rows — dq = dS K + dBD P_k (the second
// term head-major (H, B*T, dhp)), dk, dv (B*H, Tp, dhp) — in one pass.
// V values per thread (4 when dh % 4 == 0, 16-B loads).
template <int V>
__global__ void attn_dqkv_kernel(const float* __restrict__ dq_ac, const float* __restrict__ dq_bd,
                                 const float* __restrict__ dk, const float* __restrict__ dv, int B, int H, int T,
                                 int dh, int Tp, int dhp, void* __restrict__ out, int out_bf16) {
  const int dvn = dh / V;
  const long long n = (long long)B * T * H * dvn;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (long long)gridDim.x * blockDim.x) {
    const int d = (int)(q % dvn) * V;
    long long r = q / dvn;
    const int h = (int)(r % H);
    r /= H;
    const int t = (int)(r % T);
    const int b = (int)(r / T);
    const long long src = (((long long)b * H + h) * Tp + t) * dhp + d;
    const long long sbd = ((long long)h * B * T + (long long)b * T + t) * dhp + d;
    const long long o = (((long long)b * T + t) * H + h) * 3 * dh + d;
    if constexpr (V == 4) {
      const float4 a = *reinterpret_cast<const float4*>(dq_ac + src);
      const float4 c = *reinterpret_cast<const float4*>(dq_bd + sbd);
      st4(out, o, make_float4(a.x + c.x, a.y + c.y, a.z + c.z, a.w + c.w), out_bf16);
      st4(out, o + dh, *reinterpret_cast<const float4*>(dk + src), out_bf16);
      st4(out, o + 2 * dh, *reinterpret_cast<const float4*>(dv + src), out_bf16);
    } else {
      stv(out, o, dq_ac[src] + dq_bd[sbd], out_bf16);
      stv(out, o + dh, dk[src], out_bf16);
      stv(out, o + 2 * dh, dv[src], out_bf16);
    }
  }
}

}  // namespace

// Operands of the rel-pos attention products over padded rows (see
// attn_prep_kernel): qkv (B*T, H*3*dh), dO (B*T, H*dh) (may be null), pk
// (2T-1, ldp) (may be null); outputs qu, v, doh (B*H, Tp, dhp), kT, vT
// (B*H, dhp, Tp), qv (H, B*T, dhp), pkT (H, dhp, Wp), each nullable; bf16
// (dtype_bf16) or fp32 storage throughout.  Tp >= T, dhp >= dh, Wp >= 2T-1.
SBK_API int sbk_attn_prep(int dtype_bf16, const void* qkv, const void* dO, const void* pk, int ldp, const float* pbu,
                          const float* pbv, int B, int H, int T, int dh, int Tp, int dhp, int Wp, void* qu, void* qv,
                          void* kT, void* v, void* vT, void* doh, void* pkT, void* stream) {
  if (B <= 0 || H <= 0 || T <= 0 || dh <= 0 || Tp < T || dhp < dh || Wp < 2 * T - 1) return SBK_ERR_ARG;
  if (B * H > 65535 || (dhp + 63) / 64 > 65535) return SBK_ERR_ARG;
  if ((qu && !pbu) || (qv && !pbv) || (doh && !dO) || (pkT && (!pk || ldp < H * dh))) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (qu || qv || kT || v || vT || doh) {
    attn_prep_kernel<<<dim3((Tp + 63) / 64, B * H, (dhp + 63) / 64), 256, 0, s>>>(
        qkv, dO, pbu, pbv, B, H, T, dh, Tp, dhp, dtype_bf16, qu, qv, kT, v, vT, doh);
    SBK_CHECK_LAUNCH();
  }
  if (pkT) {
    attn_pkT_kernel<<<dim3((Wp + 63) / 64, H, (dhp + 63) / 64), 256, 0, s>>>(pk, ldp, H, dh, 2 * T - 1, Wp, dhp,
                                                                            dtype_bf16, pkT);
    SBK_CHECK_LAUNCH();
  }
  return 0;
}

// dqkv from the padded per-(b, h) gradients (attn_dqkv_kernel); fp32 inputs,
// out fp32 or bf16.
SBK_API int sbk_attn_dqkv(const float* dq_ac, const float* dq_bd, const float* dk, const float* dv, int B, int H,
                          int T, int dh, int Tp, int dhp, void* out, int out_bf16, void* stream) {
  if (B <= 0 || H <= 0 || T <= 0 || dh <= 0 || Tp < T || dhp < dh) return SBK_ERR_ARG;
  const bool v4 = dh % 4 == 0 && dhp % 4 == 0 &&
                  ((reinterpret_cast<uintptr_t>(dq_ac) | reinterpret_cast<uintptr_t>(dq_bd) |
                    reinterpret_cast<uintptr_t>(dk) | reinterpret_cast<uintptr_t>(dv) |
                    reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  const long long n = (long long)B * T * H * dh;
  if (v4)
    attn_dqkv_kernel<4><<<grid_for(n / 4, 256), 256, 0, (hipStream_t)stream>>>(dq_ac, dq_bd, dk, dv, B, H, T, dh, Tp,
                                                                               dhp, out, out_bf16);
  else
    attn_dqkv_kernel<1><<<grid_for(n, 256), 256, 0, (hipStream_t)stream>>>(dq_ac, dq_bd, dk, dv, B, H, T, dh, Tp,
                                                                           dhp, out, out_bf16);
  SBK_CHECK_LAUNCH();
  return 0;
}

static unsigned drop_thresh(float p) {
  const double keep = 1.0 - (double)p;
  return (unsigned)std::min(keep * 16777216.0, 16777216.0);
}

// Forward attention dropout on the probabilities: attn (fp32, may be null)
// and Pd over padded rows (B*H, Tp, Tp) in the compute dtype.  p = 0: Pd = P.
SBK_API int sbk_attn_probs_pad(const float* P, int BH, int T, int Tp, float p, unsigned long long seed, float* attn,
                               void* Pd, int pd_bf16, void* stream) {
  if (BH <= 0 || T <= 0 || Tp < T || !(p >= 0.f) || p >= 1.f) return SBK_ERR_ARG;
  const long long n = (long long)BH * Tp * Tp;
  attn_probs_pad_kernel<<<grid_for(n, 256), 256, 0, (hipStream_t)stream>>>(
      P, BH, T, Tp, drop_thresh(p), (float)(1.0 / (1.0 - (double)p)), seed, p > 0.f, attn, Pd, pd_bf16);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_dropout_add(const void* x, int x_bf16, const float* res, long long rows, int cols,
                            const unsigned char* rowmask, float alpha, float p, unsigned long long seed, void* out,
                            int out_bf16, void* stream) {
  if (rows < 0 || cols <= 0 || !(p >= 0.f) || p >= 1.f) return SBK_ERR_ARG;
  if (rows == 0) return 0;
  const double keep = 1.0 - (double)p;
  const unsigned thresh = (unsigned)std::min(keep * 16777216.0, 16777216.0);
  if (vec4_ok(rows, cols, 1, {x, res, out})) {
    dropout_add4_kernel<<<grid_for(rows * cols / 4, 256), 256, 0, (hipStream_t)stream>>>(
        x, x_bf16, res, rows, cols, rowmask, alpha, thresh, (float)(1.0 / keep), seed, p > 0.f, out, out_bf16);
    SBK_CHECK_LAUNCH();
    return 0;
  }
  dropout_add_kernel<<<grid_for(rows * cols, 256), 256, 0, (hipStream_t)stream>>>(
      x, x_bf16, res, rows, cols, rowmask, alpha, thresh, (float)(1.0 / keep), seed, p > 0.f, out, out_bf16);
  SBK_CHECK_LAUNCH();
  return 0;
}

// up to 1024 workgroups (4 rows per workgroup per trip): at 256 the ~12 rows
// each wave walked in series left the kernel latency-bound (33 us at 12k x 256)
SBK_API int sbk_layernorm_bwd_blocks(int M) { return grid_for((M + 3) / 4, 1, 1024); }

SBK_API int sbk_layernorm_bwd(const float* x, const void* dy, int dy_bf16, int M, int D, const float* g, float eps,
                              const float* dres, float* dx, float* part, void* stream) {
  if (M <= 0 || D <= 0 || D > 16384) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int grid = sbk_layernorm_bwd_blocks(M);
  if (D > 2560) {  // workgroup per row; dgamma / dbeta partials in LDS
    const size_t lds = (size_t)2 * D * sizeof(float);
    if (hipError_t e = sbk::lds_optin(reinterpret_cast<const void*>(&ln_bwd_row_kernel), lds)) return (int)e;
    ln_bwd_row_kernel<<<grid, 256, lds, s>>>(x, dy, dy_bf16, M, D, g, eps, dres, dx, part);
    SBK_CHECK_LAUNCH();
    return 0;
  }
  if (D <= 256)
    ln_bwd_kernel<4><<<grid, 256, 0, s>>>(x, dy, dy_bf16, M, D, g, eps, dres, dx, part);
  else if (D <= 1024)
    ln_bwd_kernel<16><<<grid, 256, 0, s>>>(x, dy, dy_bf16, M, D, g, eps, dres, dx, part);
  else
    ln_bwd_kernel<40><<<grid, 256, 0, s>>>(x, dy, dy_bf16, M, D, g, eps, dres, dx, part);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_layernorm_wide(const float* x, int M, int D, const float* g, const float* b, float eps, void* y,
                               int y_bf16, void* stream) {
  // the same row limit as sbk_layernorm_bwd (its workgroup-per-row kernel
  // keeps 2 x D fp32 partials in LDS): a row the backward cannot take is
  // refused here, before any forward work
  if (M <= 0 || D <= 0 || D > 16384) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (D > 2560) {
    ln_fwd_row_kernel<<<grid_for(M, 1, 4096), 256, 0, s>>>(x, M, D, g, b, eps, y, y_bf16);
    SBK_CHECK_LAUNCH();
    return 0;
  }
  const int grid = (M + 3) / 4;
  if (D <= 256)
    ln_fwd_kernel<4><<<grid, 256, 0, s>>>(x, M, D, g, b, eps, y, y_bf16);
  else if (D <= 1024)
    ln_fwd_kernel<16><<<grid, 256, 0, s>>>(x, M, D, g, b, eps, y, y_bf16);
  else
    ln_fwd_kernel<40><<<grid, 256, 0, s>>>(x, M, D, g, b, eps, y, y_bf16);
  SBK_CHECK_LAUNCH();
  return 0;
}

// up to 1024 row chunks of >= 8 rows: 128 chunks of ~94 rows (one workgroup
// per 256 columns each) left most CUs idle (26 us for 12k x 256)
SBK_API int sbk_rowsum_chunks(long long rows) { return (int)std::min<long long>(1024, std::max<long long>(1, rows / 8)); }

// out (cols) fp32 = sum over rows of x (rows, cols) (+ out when accumulate);
// part: sbk_rowsum_chunks(rows) * cols floats of scratch.
SBK_API int sbk_rowsum_batched(const void* x, int x_bf16, int batch, long long rows, int cols, float* part,
                               float* out, int accumulate, void* stream) {
  if (rows <= 0 || cols <= 0 || batch <= 0 || batch > 65535) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int nchunk = sbk_rowsum_chunks(rows);
  const int rows_per = (int)((rows + nchunk - 1) / nchunk);
  dim3 grid(nchunk, (cols + 255) / 256, batch);
  rowsum_partial_kernel<<<grid, 256, 0, s>>>(x, x_bf16, rows, cols, rows_per, part);
  SBK_CHECK_LAUNCH();
  colsum_kernel<<<(batch * cols + 63) / 64, 1024, 0, s>>>(part, nchunk, batch * cols, out, accumulate);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_rowsum(const void* x, int x_bf16, long long rows, int cols, float* part, float* out, int accumulate,
                       void* stream) {
  return sbk_rowsum_batched(x, x_bf16, 1, rows, cols, part, out, accumulate, stream);
}

SBK_API int sbk_colsum(const float* part, int rows, int cols, float* out, int accumulate, void* stream) {
  if (rows <= 0 || cols <= 0) return SBK_ERR_ARG;
  colsum_kernel<<<(cols + 63) / 64, 1024, 0, (hipStream_t)stream>>>(part, rows, cols, out, accumulate);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_act_fwd(int mode, const void* x, int x_bf16, long long rows, int cols, void* y, int y_bf16,
                        float slope, void* stream) {
  if (mode < 1 || mode > 4 || rows < 0 || cols <= 0) return SBK_ERR_ARG;
  if (rows == 0) return 0;
  if (mode != 4 && vec4_ok(rows, cols, mode, {x, y})) {
    const int g4 = grid_for(rows * cols / 4, 256);
    hipStream_t st = (hipStream_t)stream;
    if (mode == 1) act_fwd4_kernel<1><<<g4, 256, 0, st>>>(x, x_bf16, rows, cols, y, y_bf16, slope);
    else if (mode == 2) act_fwd4_kernel<2><<<g4, 256, 0, st>>>(x, x_bf16, rows, cols, y, y_bf16, slope);
    else act_fwd4_kernel<3><<<g4, 256, 0, st>>>(x, x_bf16, rows, cols, y, y_bf16, slope);
    SBK_CHECK_LAUNCH();
    return 0;
  }
  act_fwd_kernel<<<grid_for(rows * cols, 256), 256, 0, (hipStream_t)stream>>>(mode, x, x_bf16, rows, cols, y, y_bf16,
                                                                              slope);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_act_bwd(int mode, const void* x, int x_bf16, const void* dy, int dy_bf16, long long rows, int cols,
                        void* dx, int dx_bf16, float slope, void* stream) {
  if (mode < 1 || mode > 4 || rows < 0 || cols <= 0) return SBK_ERR_ARG;
  if (rows == 0) return 0;
  if (mode != 4 && vec4_ok(rows, cols, mode, {x, dy, dx})) {
    const int g4 = grid_for(rows * cols / 4, 256);
    hipStream_t st = (hipStream_t)stream;
    if (mode == 1) act_bwd4_kernel<1><<<g4, 256, 0, st>>>(x, x_bf16, dy, dy_bf16, rows, cols, dx, dx_bf16, slope);
    else if (mode == 2) act_bwd4_kernel<2><<<g4, 256, 0, st>>>(x, x_bf16, dy, dy_bf16, rows, cols, dx, dx_bf16, slope);
    else act_bwd4_kernel<3><<<g4, 256, 0, st>>>(x, x_bf16, dy, dy_bf16, rows, cols, dx, dx_bf16, slope);
    SBK_CHECK_LAUNCH();
    return 0;
  }
  act_bwd_kernel<<<grid_for(rows * cols, 256), 256, 0, (hipStream_t)stream>>>(mode, x, x_bf16, dy, dy_bf16, rows,
                                                                              cols, dx, dx_bf16, slope);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_dwconv_fwd(const void* x, int x_bf16, int B, int T, int C, const float* w, const float* bias, int K,
                           int causal, void* y, int y_bf16, void* stream) {
  if (B <= 0 || T <= 0 || C <= 0 || K <= 0 || K > DW_KMAX) return SBK_ERR_ARG;
  const int padL = causal ? K - 1 : (K - 1) / 2;
  const int nrun = (T + DW_RUN - 1) / DW_RUN;
  dim3 grid((C + 255) / 256, B * nrun);
  dwconv_fwd_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(x, x_bf16, B, T, C, w, bias, K, padL, 0, y, y_bf16);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_dwconv_wgrad_chunks(int B, int T) { return B * ((T + DW_RUN - 1) / DW_RUN); }

// dx (optional) and per-run (nchunk, C, K+1) weight|bias partials.  dx is the
// forward kernel on dy with the taps reversed and padL' = K - 1 - padL.
SBK_API int sbk_dwconv_bwd(const void* x, int x_bf16, const float* dy, int B, int T, int C, const float* w, int K,
                           int causal, void* dx, int dx_bf16, float* part, void* stream) {
  if (B <= 0 || T <= 0 || C <= 0 || K <= 0 || K > DW_KMAX) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int padL = causal ? K - 1 : (K - 1) / 2;
  const int nrun = (T + DW_RUN - 1) / DW_RUN;
  dim3 grid((C + 255) / 256, B * nrun);
  if (dx) {
    dwconv_fwd_kernel<<<grid, 256, 0, s>>>(dy, 0, B, T, C, w, nullptr, K, K - 1 - padL, 1, dx, dx_bf16);
    SBK_CHECK_LAUNCH();
  }
  if (part) {
    dwconv_wgrad_kernel<<<grid, 256, 0, s>>>(x, x_bf16, dy, B, T, C, K, padL, part);
    SBK_CHECK_LAUNCH();
  }
  return 0;
}

// RelPosMHAXL softmax / dropout / rel_shift backward over padded rows
// (relpos_softmax_bwd_pad_kernel): P (B, H, T, T) fp32, dP (B*H, Tp, Tp);
// out dS, Pd (B*H, Tp, Tp), dBD (H, B*T, Wp); dP and the outputs bf16
// (dtype_bf16) or fp32.  p, seed: the forward's attention dropout.
SBK_API int sbk_relpos_softmax_bwd_pad(int dtype_bf16, const float* P, const void* dP, int B, int H, int T, int Tp,
                                       int Wp, float scale, float p, unsigned long long seed, void* dS, void* Pd,
                                       void* dBD, void* stream) {
  if (B <= 0 || H <= 0 || T <= 0 || Tp < T || Wp < 2 * T - 1 || !(p >= 0.f) || p >= 1.f) return SBK_ERR_ARG;
  const long long nrows = (long long)B * H * Tp;
  relpos_softmax_bwd_pad_kernel<<<(unsigned)((nrows + 3) / 4), 256, 0, (hipStream_t)stream>>>(
      P, dP, scale, B, H, T, Tp, Wp, drop_thresh(p), (float)(1.0 / (1.0 - (double)p)), seed, p > 0.f, dS, Pd, dBD,
      dtype_bf16);
  SBK_CHECK_LAUNCH();
  return 0;
}

static bool conv_geom_ok(int Ti, int Fi, int kt, int kf, int st, int sf, int pt, int pf, int* To, int* Fo) {
  if (kt <= 0 || kf <= 0 || st <= 0 || sf <= 0 || pt < 0 || pf < 0 || pt >= Ti || pf >= Fi) return false;
  *To = (Ti + 2 * pt - kt) / st + 1;
  *Fo = (Fi + 2 * pf - kf) / sf + 1;
  return Ti + 2 * pt >= kt && Fi + 2 * pf >= kf;
}

SBK_API int sbk_im2col(const void* x, int x_bf16, int B, int Ti, int Fi, int Ci, int kt, int kf, int st, int sf, int pt,
                       int pf, int ldcol, void* col, int col_bf16, void* stream) {
  int To, Fo;
  if (B <= 0 || Ci <= 0 || !conv_geom_ok(Ti, Fi, kt, kf, st, sf, pt, pf, &To, &Fo) || ldcol < kt * kf * Ci)
    return SBK_ERR_ARG;
  im2col_kernel<<<grid_for((long long)B * To * Fo * ldcol, 256), 256, 0, (hipStream_t)stream>>>(
      x, x_bf16, B, Ti, Fi, Ci, To, Fo, ConvGeom{kt, kf, st, sf, pt, pf}, ldcol, col, col_bf16);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_col2im(const void* dcol, int dcol_bf16, int B, int Ti, int Fi, int Ci, int kt, int kf, int st, int sf,
                       int pt, int pf, int ldcol, void* dx, int dx_bf16, void* stream) {
  int To, Fo;
  if (B <= 0 || Ci <= 0 || !conv_geom_ok(Ti, Fi, kt, kf, st, sf, pt, pf, &To, &Fo) || ldcol < kt * kf * Ci)
    return SBK_ERR_ARG;
  col2im_kernel<<<grid_for((long long)B * Ti * Fi * Ci, 256), 256, 0, (hipStream_t)stream>>>(
      dcol, dcol_bf16, B, Ti, Fi, Ci, To, Fo, ConvGeom{kt, kf, st, sf, pt, pf}, ldcol, dx, dx_bf16);
  SBK_CHECK_LAUNCH();
  return 0;
}

// ---- general Conv2d geometry: dilation, leading / trailing padding per
// axis and the F.pad modes (0 reflect, 1 zeros, 2 replicate, 3 circular):
// the standalone Conv2d drop-in (CNN.py:556-700: "same" with any
// padding_mode, "valid", "causal", dilation; groups and skip_transpose by
// the host).  col (B*To*Fo, ldcol), column order (time tap, freq tap, ci).
struct ConvGeomX {
  int kt, kf, st, sf, dt, df, pt, pf, mode;
};

// input index of padded-minus-lead position s, or -1 for a zero
__device__ __forceinline__ int pad_map(int s, int n, int mode) {
  if (s >= 0 && s < n) return s;
  if (mode == 1) return -1;
  if (mode == 2) return s < 0 ? 0 : n - 1;
  if (mode == 3) return ((s % n) + n) % n;
  return reflect_idx(s, n);  // one reflection (host: pad < n)
}

__global__ void im2colx_kernel(const void* __restrict__ x, int x_bf16, int B, int Ti, int Fi, int Ci, int To, int Fo,
                               ConvGeomX gm, int ldcol, void* __restrict__ col, int col_bf16) {
  const long long n = (long long)B * To * Fo * ldcol;
  const int kcols = gm.kt * gm.kf * Ci;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int kk = (int)(i % ldcol);
    long long q = i / ldcol;
    if (kk >= kcols) {
      stv(col, i, 0.f, col_bf16);
      continue;
    }
    const int ci = kk % Ci;
    const int kf = (kk / Ci) % gm.kf;
    const int kt = kk / (gm.kf * Ci);
    const int fo = (int)(q % Fo); q /= Fo;
    const int to = (int)(q % To);
    const int b = (int)(q / To);
    const int ti = pad_map(to * gm.st + kt * gm.dt - gm.pt, Ti, gm.mode);
    const int fi = pad_map(fo * gm.sf + kf * gm.df - gm.pf, Fi, gm.mode);
    const float v = (ti < 0 || fi < 0) ? 0.f : ldv(x, (((long long)b * Ti + ti) * Fi + fi) * Ci + ci, x_bf16);
    stv(col, i, v, col_bf16);
  }
}

// the adjoint, first onto the padded grid (Tp x Fp, fp32): every padded
// position gathers the (output position, tap) pairs that read it
__global__ void col2padx_kernel(const void* __restrict__ dcol, int dcol_bf16, int B, int Tp, int Fp, int Ci, int To,
                                int Fo, ConvGeomX gm, int ldcol, float* __restrict__ dxp) {
  const long long n = (long long)B * Tp * Fp * Ci;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % Ci);
    long long q = i / Ci;
    const int fp = (int)(q % Fp); q /= Fp;
    const int tp = (int)(q % Tp);
    const int b = (int)(q / Tp);
    float s = 0.f;
    for (int kt = 0; kt < gm.kt; ++kt) {
      const int d = tp - kt * gm.dt;
      if (d < 0 || d % gm.st) continue;
      const int to = d / gm.st;
      if (to >= To) continue;
      for (int kf = 0; kf < gm.kf; ++kf) {
        const int df = fp - kf * gm.df;
        if (df < 0 || df % gm.sf) continue;
        const int fo = df / gm.sf;
        if (fo >= Fo) continue;
        s += ldv(dcol, (((long long)b * To + to) * Fo + fo) * ldcol + (kt * gm.kf + kf) * Ci + ci, dcol_bf16);
      }
    }
    dxp[i] = s;
  }
}

// then folded onto the input: dx[ti, fi] = sum of the padded positions that
// map onto it (the direct one and, in the pad zones, its reflections /
// replications / wraps), in a fixed order (deterministic)
__global__ void foldx_kernel(const float* __restrict__ dxp, int B, int Tp, int Fp, int Ti, int Fi, int Ci, int pt,
                             int pf, int mode, void* __restrict__ dx, int dx_bf16) {
  const long long n = (long long)B * Ti * Fi * Ci;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % Ci);
    long long q = i / Ci;
    const int fi = (int)(q % Fi); q /= Fi;
    const int ti = (int)(q % Ti);
    const int b = (int)(q / Ti);
    // candidates per axis: the leading pad zone, the direct position, the
    // trailing pad zone (the interior maps 1:1)
    const int zt = max(0, Tp - pt - Ti), zf = max(0, Fp - pf - Fi);
    float s = 0.f;
    for (int u = 0; u < pt + 1 + zt; ++u) {
      const int tp = u < pt ? u : (u == pt ? ti + pt : pt + Ti + (u - pt - 1));
      if (tp >= Tp || pad_map(tp - pt, Ti, mode) != ti) continue;
      for (int v = 0; v < pf + 1 + zf; ++v) {
        const int fp = v < pf ? v : (v == pf ? fi + pf : pf + Fi + (v - pf - 1));
        if (fp >= Fp || pad_map(fp - pf, Fi, mode) != fi) continue;
        s += dxp[(((long long)b * Tp + tp) * Fp + fp) * Ci + ci];
      }
    }
    stv(dx, i, s, dx_bf16);
  }
}

namespace {
bool convx_ok(int B, int Ti, int Fi, int Ci, int kt, int kf, int st, int sf, int dt, int df, int pt, int pf, int To,
              int Fo, int mode, int ldcol) {
  return B > 0 && Ti > 0 && Fi > 0 && Ci > 0 && kt > 0 && kf > 0 && st > 0 && sf > 0 && dt > 0 && df > 0 && pt >= 0 &&
         pf >= 0 && To > 0 && Fo > 0 && mode >= 0 && mode <= 3 && ldcol >= kt * kf * Ci &&
         (mode != 0 || (pt < Ti && pf < Fi)) &&
         // every tap of the last output lies within one pad of the input
         (To - 1) * st + (kt - 1) * dt - pt < Ti + (mode == 0 ? Ti - 1 : 1 << 30) &&
         (Fo - 1) * sf + (kf - 1) * df - pf < Fi + (mode == 0 ? Fi - 1 : 1 << 30);
}
}  // namespace

SBK_API int sbk_im2col_x(const void* x, int x_bf16, int B, int Ti, int Fi, int Ci, int kt, int kf, int st, int sf,
                         int dt, int df, int pt, int pf, int To, int Fo, int mode, int ldcol, void* col, int col_bf16,
                         void* stream) {
  if (!convx_ok(B, Ti, Fi, Ci, kt, kf, st, sf, dt, df, pt, pf, To, Fo, mode, ldcol)) return SBK_ERR_ARG;
  im2colx_kernel<<<grid_for((long long)B * To * Fo * ldcol, 256), 256, 0, (hipStream_t)stream>>>(
      x, x_bf16, B, Ti, Fi, Ci, To, Fo, ConvGeomX{kt, kf, st, sf, dt, df, pt, pf, mode}, ldcol, col, col_bf16);
  SBK_CHECK_LAUNCH();
  return 0;
}

// dxpad: fp32 scratch of B*Tp*Fp*Ci, Tp = (To-1) st + (kt-1) dt + 1 (and Fp
// alike): the padded extent the outputs read
SBK_API int sbk_col2im_x(const void* dcol, int dcol_bf16, int B, int Ti, int Fi, int Ci, int kt, int kf, int st,
                         int sf, int dt, int df, int pt, int pf, int To, int Fo, int mode, int ldcol, float* dxpad,
                         void* dx, int dx_bf16, void* stream) {
  if (!convx_ok(B, Ti, Fi, Ci, kt, kf, st, sf, dt, df, pt, pf, To, Fo, mode, ldcol) || !dxpad) return SBK_ERR_ARG;
  const int Tp = (To - 1) * st + (kt - 1) * dt + 1, Fp = (Fo - 1) * sf + (kf - 1) * df + 1;
  const ConvGeomX gm{kt, kf, st, sf, dt, df, pt, pf, mode};
  col2padx_kernel<<<grid_for((long long)B * Tp * Fp * Ci, 256), 256, 0, (hipStream_t)stream>>>(
      dcol, dcol_bf16, B, Tp, Fp, Ci, To, Fo, gm, ldcol, dxpad);
  SBK_CHECK_LAUNCH();
  foldx_kernel<<<grid_for((long long)B * Ti * Fi * Ci, 256), 256, 0, (hipStream_t)stream>>>(
      dxpad, B, Tp, Fp, Ti, Fi, Ci, pt, pf, mode, dx, dx_bf16);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_joint_fwd(const float* tn, const float* pn, int B, int T, int U1, int J, int act, float slope, void* z,
                          int z_bf16, void* stream) {
  if (B <= 0 || T <= 0 || U1 <= 0 || J <= 0) return SBK_ERR_ARG;
  if (J % 4)
    joint_fwd_scalar_kernel<<<(unsigned)((long long)B * T), 256, 0, (hipStream_t)stream>>>(tn, pn, T, U1, J, act,
                                                                                          slope, z, z_bf16);
  else
    joint_fwd_kernel<<<(unsigned)((long long)B * T), 256, 0, (hipStream_t)stream>>>(tn, pn, T, U1, J, act, slope, z,
                                                                                   z_bf16);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API long long sbk_joint_bwd_workspace_floats(int B, int T, int U1, int J) {
  return (long long)(J % 2 ? T : (T + JB_T - 1) / JB_T) * B * U1 * J;
}

// ws: sbk_joint_bwd_workspace_floats() floats (per-run dpn partials).
SBK_API int sbk_joint_bwd(const float* tn, const float* pn, const void* dz, int dz_bf16, int B, int T, int U1, int J,
                          int act, float slope, float* dtn, float* dpn, float* ws, void* stream) {
  if (B <= 0 || T <= 0 || U1 <= 0 || J <= 0 || !ws) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  int nrun;
  if (J % 2) {
    nrun = T;
    joint_bwd_scalar_kernel<<<(unsigned)((long long)B * T), 256, 0, s>>>(tn, pn, dz, dz_bf16, T, U1, J, act, slope,
                                                                         dtn, ws, B);
  } else {
    nrun = (T + JB_T - 1) / JB_T;
    dim3 grid((J / 2 + 255) / 256, B * nrun);
    joint_bwd_kernel<<<grid, 256, 0, s>>>(tn, pn, dz, dz_bf16, B, T, U1, J, act, slope, dtn, ws);
  }
  SBK_CHECK_LAUNCH();
  const long long cols = (long long)B * U1 * J;
  if (cols > 0x7fffffffLL) return SBK_ERR_ARG;
  colsum_kernel<<<(unsigned)((cols + 63) / 64), 1024, 0, s>>>(ws, nrun, (int)cols, dpn, 0);
  SBK_CHECK_LAUNCH();
  return 0;
}
