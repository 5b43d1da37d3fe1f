// RNN-T (transducer) loss: fused log-softmax gather, anti-diagonal α/β
// wavefront, sparse gradient, dense gradient wrt logits.
//
// Reference: speechbrain/nnet/loss/transducer_loss.py (Numba CUDA):
//   cu_kernel_forward  :31-106   α,  log_p = (α[T-1,U] + lp[T-1,U,∅]) / T
//   cu_kernel_backward :109-180  β
//   cu_kernel_compute_grad :183-236  ∂(-log P)/∂lp at blank / label entries
//   Transducer.forward/backward :252-293 ; losses.py:27-85 (log_softmax wrapper)
//
// The Numba kernels pipeline one thread per label position u with spin-locks
// on global atomics; inside a lock-stepped wave64 such intra-wave spinning
// deadlocks, so the lattice is recast as an anti-diagonal wavefront: cells
// with t + u = n depend only on diagonal n - 1, kept in an LDS double buffer;
// one workgroup per (utterance, direction), one barrier per diagonal.
// The log-add is computed exactly as the reference writes it,
// max(a,b) + log1p(exp(-|a-b|)), with the correction term evaluated in f64
// and rounded to f32 (the oracle's convention), all other arithmetic f32.
//
// Layouts: logits / log_probs (B, T, U1, V) fp32 (U1 = max labels + 1),
// labels (B, U1-1) int32, lens T_b, U_b int32 (absolute).
#include "sbk_common.h"

using namespace sbk;

namespace {

__device__ __forceinline__ float lae(float a, float b) {
  const float m = fmaxf(a, b);
  return m + (float)log1p(exp(-(double)fabsf(a - b)));
}

// One wave per (b, t, u) row: lse (if logits), lp at blank and at label y_u.
__global__ void __launch_bounds__(256) gather_kernel(const float* __restrict__ x, const int* __restrict__ labels,
                                                     int B, int T, int U1, int V, int blank, int is_logits,
                                                     float* __restrict__ lpb, float* __restrict__ lpl,
                                                     float* __restrict__ lse_out) {
  const long long rows = (long long)B * T * U1;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const int u = (int)(row % U1);
  const int b = (int)(row / ((long long)T * U1));
  const float* xr = x + row * V;
  float lse = 0.f;
  if (is_logits) {
    float m = -INFINITY;
    for (int v = lane; v < V; v += 64) m = fmaxf(m, xr[v]);
    m = wave_max(m);
    float s = 0.f;
    for (int v = lane; v < V; v += 64) s += expf(xr[v] - m);
    s = wave_sum(s);
    lse = m + logf(s);
  }
  if (lane == 0) {
    lpb[row] = xr[blank] - lse;
    const int Um = U1 - 1;
    const int y = u < Um ? labels[b * Um + u] : 0;
    // a label outside [0, V) poisons its cell (NaN loss) instead of reading
    // past the row
    lpl[row] = u < Um ? ((unsigned)y < (unsigned)V ? xr[y] - lse : __builtin_nanf("")) : 0.f;
    if (lse_out) lse_out[row] = lse;
  }
}

// grid (B, 2): y = 0 -> α, y = 1 -> β.  Threads over u (loops if U1 > blockDim).
__global__ void __launch_bounds__(256) lattice_kernel(const float* __restrict__ lpb, const float* __restrict__ lpl,
                                                      const int* __restrict__ Tl, const int* __restrict__ Ul, int T,
                                                      int U1, float* __restrict__ alpha, float* __restrict__ beta,
                                                      float* __restrict__ logp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* diag = reinterpret_cast<float*>(smem);  // 2 x U1
  const int b = blockIdx.x;
  const bool fwd = blockIdx.y == 0;
  const int Tb = Tl[b], Ub = Ul[b];
  if (Tb < 1 || Tb > T || Ub < 0 || Ub > U1 - 1) {
    // lengths outside the (T, U1) lattice: NaN loss for this utterance, no
    // access outside its slab or the 2*U1 diagonal buffer
    if (threadIdx.x == 0) logp[(fwd ? 0 : gridDim.x) + b] = __builtin_nanf("");
    return;
  }
  const long long base = (long long)b * T * U1;
  const float* pb = lpb + base;
  const float* pl = lpl + base;
  float* out = (fwd ? alpha : beta) + base;
  const int ndiag = Tb + Ub;  // diagonals n = 0 .. Tb + Ub - 1
  for (int n = 0; n < ndiag; ++n) {
    float* cur = diag + (n & 1) * U1;
    const float* prv = diag + ((n & 1) ^ 1) * U1;
    for (int u = threadIdx.x; u <= Ub; u += blockDim.x) {
      if (fwd) {
        const int t = n - u;
        if (t < 0 || t >= Tb) continue;
        float a;
        if (t == 0 && u == 0)
          a = 0.f;
        else if (u == 0)
          a = prv[0] + pb[(long long)(t - 1) * U1];  // α[t-1,0] + lp[t-1,0,∅]
        else if (t == 0)
          a = prv[u - 1] + pl[u - 1];                 // α[0,u-1] + lp[0,u-1,y]
        else {
          const float emit = prv[u - 1] + pl[(long long)t * U1 + u - 1];
          const float no_emit = prv[u] + pb[(long long)(t - 1) * U1 + u];
          a = lae(no_emit, emit);
        }
        cur[u] = a;
        out[(long long)t * U1 + u] = a;
      } else {
        // reverse diagonal: n = (Tb-1-t) + (Ub-u)
        const int t = Tb - 1 - (n - (Ub - u));
        if (t < 0 || t >= Tb || n - (Ub - u) < 0) continue;
        float v;
        if (u == Ub && t == Tb - 1)
          v = pb[(long long)t * U1 + u];
        else if (u == Ub)
          v = prv[u] + pb[(long long)t * U1 + u];            // β[t+1,U] + lp[t,U,∅]
        else if (t == Tb - 1)
          v = prv[u + 1] + pl[(long long)t * U1 + u];        // β[T-1,u+1] + lp[T-1,u,y_u]
        else {
          const float emit = prv[u + 1] + pl[(long long)t * U1 + u];
          const float no_emit = prv[u] + pb[(long long)t * U1 + u];
          v = lae(no_emit, emit);
        }
        cur[u] = v;
        out[(long long)t * U1 + u] = v;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (fwd)
      logp[b] = (out[(long long)(Tb - 1) * U1 + Ub] + pb[(long long)(Tb - 1) * U1 + Ub]) / (float)Tb;
    else
      logp[gridDim.x + b] = out[0];  // β[0,0] (un-normalised log P)
  }
}


// Sparse gradients wrt log-probs at the blank and label entries of every
// lattice cell (transducer_loss.py:206-236), f32 ops in the reference order:
//   g_blank[t,u] = -exp(α[t,u] + β[t+1,u] + lp∅ - β00)   t < T-1, u <= U
//   g_blank[T-1,U] = -exp(α[T-1,U] + lp∅ - β00)
//   g_label[t,u] = -exp(α[t,u] + β[t,u+1] + lp_y - β00)  u < U
// Cells outside the valid lattice get 0.
__global__ void sparse_grad_kernel(const float* __restrict__ lpb, const float* __restrict__ lpl,
                                   const float* __restrict__ alpha, const float* __restrict__ beta,
                                   const int* __restrict__ Tl, const int* __restrict__ Ul, const float* __restrict__ logp,
                                   int B, int T, int U1, float* __restrict__ gb, float* __restrict__ gl) {
  const long long n = (long long)B * T * U1;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int u = (int)(i % U1);
    const int t = (int)((i / U1) % T);
    const int b = (int)(i / ((long long)T * U1));
    const int Tb = Tl[b], Ub = Ul[b];
    const float b00 = logp[B + b];
    const long long base = (long long)b * T * U1;
    float vb = 0.f, vl = 0.f;
    if (Tb < 1 || Tb > T || Ub < 0 || Ub > U1 - 1) {
      vb = vl = __builtin_nanf("");  // invalid lengths: NaN gradient, as the loss
    } else if (t < Tb && u <= Ub) {
      const float a = alpha[i];
      if (t < Tb - 1) {
        const float s = (a + beta[base + (long long)(t + 1) * U1 + u]) + lpb[i];
        vb = -(float)exp((double)(s - b00));
      } else if (u == Ub) {
        const float s = a + lpb[i];
        vb = -(float)exp((double)(s - b00));
      }
      if (u < Ub) {
        const float s = (a + beta[base + (long long)t * U1 + u + 1]) + lpl[i];
        vl = -(float)exp((double)(s - b00));
      }
    }
    gb[i] = vb;
    gl[i] = vl;
  }
}

// Dense gradient rows.  mode 0 (wrt log-probs, the Transducer.apply
// contract): g[v] = [v==∅]·gb + [v==y]·gl.  mode 1 (wrt logits through the
// log-softmax): g[v] = [v==∅]·gb + [v==y]·gl - softmax_v·(gb + gl).
// Each row is scaled by scale[b] (grad_output, reduction).  One wave per row.
__global__ void __launch_bounds__(256) dense_grad_kernel(const float* __restrict__ x, const float* __restrict__ lse,
                                                         const float* __restrict__ gb, const float* __restrict__ gl,
                                                         const int* __restrict__ labels, const float* __restrict__ scale,
                                                         int scale_per_b, int B, int T, int U1, int V, int blank,
                                                         int mode, float* __restrict__ out) {
  const long long rows = (long long)B * T * U1;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const int u = (int)(row % U1);
  const int b = (int)(row / ((long long)T * U1));
  const float sc = scale[scale_per_b ? b : 0];
  const float g_b = gb[row] * sc, g_l = gl[row] * sc;
  const int Um = U1 - 1;
  const int y = u < Um ? labels[b * Um + u] : -1;
  float* orow = out + row * V;
  if (mode == 0) {
    for (int v = lane; v < V; v += 64) orow[v] = (v == blank ? g_b : 0.f) + (v == y ? g_l : 0.f);
    return;
  }
  const float* xr = x + row * V;
  const float l = lse[row], gs = g_b + g_l;
  for (int v = lane; v < V; v += 64) {
    const float p = expf(xr[v] - l);
    orow[v] = (v == blank ? g_b : 0.f) + (v == y ? g_l : 0.f) - p * gs;
  }
}

// loss: mode 0 (SpeechBrain/Numba): -log_p_alpha = -(α+lp)/T ; mode 1 (standard):
// -β00.  reduction 0 mean, 1 sum, 2 none.  One block.
__global__ void finalize_kernel(const float* __restrict__ logp, int B, int loss_mode, int reduction,
                                float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const float l = loss_mode == 0 ? -logp[b] : -logp[B + b];
    if (reduction == 2) out[b] = l;
    s += l;
  }
  if (reduction == 2) return;
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] = reduction == 0 ? s / (float)B : s;
}

}  // namespace

SBK_API int sbk_rnnt_lattice(const int* Tl, const int* Ul, int B, int T, int U1, int loss_mode, int reduction,
                             float* ws, float* out, void* stream);

// Forward: per-cell log-probs, α, β, log P, sparse grads and the reduced loss.
//   x: logits (is_logits=1, log-softmax fused) or log-probs (is_logits=0).
//   ws: workspace of 6*B*T*U1 + 2*B floats: [lpb | lpl | lse | α | β | gb | gl ... ]
//   (layout below), loss_mode 0 = SpeechBrain Numba semantics (loss/T),
//   1 = standard -log P.  out: 1 float (mean/sum) or B floats (none).
SBK_API int sbk_rnnt_forward(const float* x, const int* labels, const int* Tl, const int* Ul, int B, int T, int U1,
                             int V, int blank, int is_logits, int loss_mode, int reduction, float* ws, float* out,
                             void* stream) {
  if (B <= 0 || T <= 0 || U1 <= 0 || V <= 0 || blank < 0 || blank >= V) return SBK_ERR_ARG;
  const long long n = (long long)B * T * U1;
  // ws: [lpb | lpl | lse | α | β | gb | gl | log P (2B)]
  hipLaunchKernelGGL(gather_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, labels, B, T,
                     U1, V, blank, is_logits, ws, ws + n, ws + 2 * n);
  SBK_CHECK_LAUNCH();
  return sbk_rnnt_lattice(Tl, Ul, B, T, U1, loss_mode, reduction, ws, out, stream);
}

// The lattice half of sbk_rnnt_forward for log-probs gathered elsewhere (the
// fused transducer head, thead.hip): ws[lpb | lpl | lse] filled, α, β,
// log P, sparse grads and the reduced loss computed.
SBK_API int sbk_rnnt_lattice(const int* Tl, const int* Ul, int B, int T, int U1, int loss_mode, int reduction,
                             float* ws, float* out, void* stream) {
  if (B <= 0 || T <= 0 || U1 <= 0 || !ws || !out || !Tl || !Ul) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const long long n = (long long)B * T * U1;
  float* lpb = ws;
  float* lpl = ws + n;
  float* alpha = ws + 3 * n;
  float* beta = ws + 4 * n;
  float* gb = ws + 5 * n;
  float* gl = ws + 6 * n;
  float* logp = ws + 7 * n;  // 2B
  hipLaunchKernelGGL(lattice_kernel, dim3(B, 2), dim3(U1 >= 256 ? 256 : ((U1 + 63) / 64) * 64), (size_t)2 * U1 * 4, s,
                     lpb, lpl, Tl, Ul, T, U1, alpha, beta, logp);
  SBK_CHECK_LAUNCH();
  long long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(sparse_grad_kernel, dim3((unsigned)g), dim3(256), 0, s, lpb, lpl, alpha, beta, Tl, Ul, logp, B,
                     T, U1, gb, gl);
  SBK_CHECK_LAUNCH();
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(256), 0, s, logp, B, loss_mode, reduction, out);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API long long sbk_rnnt_workspace_floats(int B, int T, int U1) { return 7LL * B * T * U1 + 2LL * B; }

// Dense gradient (B, T, U1, V): mode 0 wrt log-probs, mode 1 wrt logits.
SBK_API int sbk_rnnt_backward(const float* x, const int* labels, int B, int T, int U1, int V, int blank, int mode,
                              const float* ws, const float* scale, int scale_per_b, float* grad, void* stream) {
  if (B <= 0 || T <= 0 || U1 <= 0 || V <= 0) return SBK_ERR_ARG;
  const long long n = (long long)B * T * U1;
  hipLaunchKernelGGL(dense_grad_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x,
                     ws + 2 * n, ws + 5 * n, ws + 6 * n, labels, scale, scale_per_b, B, T, U1, V, blank, mode, grad);
  SBK_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// Transducer decoding (decoders/transducer.py:137-377): log-softmax of the
// joint logits and their top-k in one pass, one wave per row.  Replaces
// LogSoftmax → torch.max (greedy, k = 1) / torch.topk (beam) on (rows, V).
// Ties resolve to the lower vocabulary index.  vals = x[idx] - lse.
namespace {
__global__ void __launch_bounds__(256) logsoftmax_topk_kernel(const float* __restrict__ x, long long ldx, int R,
                                                              int V, int k, float* __restrict__ vals,
                                                              long long* __restrict__ idx) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int lane = threadIdx.x & 63;
  const float* xr = x + (long long)row * ldx;
  float m = -INFINITY;
  for (int v = lane; v < V; v += 64) m = fmaxf(m, xr[v]);
  m = wave_max(m);
  float s = 0.f;
  for (int v = lane; v < V; v += 64) s += expf(xr[v] - m);
  const float lse = m + logf(wave_sum(s));
  int prev_i = -1;
  float prev_v = INFINITY;
  for (int j = 0; j < k; ++j) {
    // next best strictly after (prev_v, prev_i) in (value desc, index asc) order
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int v = lane; v < V; v += 64) {
      const float xv = xr[v];
      const bool after = xv < prev_v || (xv == prev_v && v > prev_i);
      if (after && (xv > bv || (xv == bv && v < bi))) {
        bv = xv;
        bi = v;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o);
      const int oi = __shfl_xor(bi, o);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      vals[(long long)row * k + j] = bv - lse;
      idx[(long long)row * k + j] = bi;
    }
    prev_v = bv;
    prev_i = bi;
  }
}
}  // namespace

SBK_API int sbk_logsoftmax_topk(const float* x, long long ldx, int R, int V, int k, float* vals, long long* idx,
                                void* stream) {
  if (R <= 0 || V <= 0 || k <= 0 || k > V) return SBK_ERR_ARG;
  hipLaunchKernelGGL(logsoftmax_topk_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, ldx,
                     R, V, k, vals, idx);
  SBK_CHECK_LAUNCH();
  return 0;
}
