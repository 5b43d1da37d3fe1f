// RelPosMHAXL with query != key/value and q_len != k_len: the attention core
// of speechbrain/nnet/attention.py:554-639 for separate q / k / v
// projections (the projections themselves run on sbk_gemm), with the
// reference's rel_shift (:468-483) on a (q_len, P) positional band, its
// mask_pos_future tril, attn_mask, key padding, softmax, attention dropout
// and P·V — and the backward of all of it.
//
// Not on the encoder's hot path (every Conformer call site is
// self-attention, which runs in the fused flash kernel of attention.hip), so
// these kernels are plain fp32 VALU: one workgroup per (query row | key row
// | band column, head, batch), the row of scores in LDS.  What they must get
// right is the rel_shift of a non-square band: output (i, j) of the
// reference's pad / view / drop-row trick is flat element
// p = i*P + j + q_len of the left-padded (q_len, P+1) band, i.e. row
// r = p / (P+1), column c = p % (P+1) (c == 0: the zero pad, else
// bd[r][c-1]).  For q_len > k_len, r can be i + 1 or further: the reference
// reads the next row there, and so do these kernels.
//
// Layouts: q (B*Lq, ldq), k (B*Lk, ldk), v (B*Lk, ldv), pk (P, ldp), head h
// at columns [h*dh, (h+1)*dh), fp32 or bf16; pbu / pbv (H*dh) fp32 (the
// (dh, H) parameters read as (H, dh), attention.py:586-592); probabilities
// (B, H, Lq, Lk) fp32.
//
// pk == nullptr selects plain scaled dot-product attention (the
// MultiheadAttention drop-in's general path, attention.py:642-778): no
// positional term, no u / v biases (pbu / pbv may be null), and the backward
// skips the band passes — dq comes straight out of the row pass.
#include "sbk_common.h"

#include <math.h>

namespace {

using sbk::bf16_to_f32;
using sbk::f32_to_bf16;

constexpr int kThreads = 256;

__device__ __forceinline__ float ld(const float* p, long long i) { return p[i]; }
__device__ __forceinline__ float ld(const uint16_t* p, long long i) { return bf16_to_f32(p[i]); }
__device__ __forceinline__ void st(float* p, long long i, float v) { p[i] = v; }
__device__ __forceinline__ void st(uint16_t* p, long long i, float v) { p[i] = f32_to_bf16(v); }

// counter-based dropout keep mask (the hash of backward.hip's dropout:
// forward and backward launches regenerate the same bits)
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ bool keep_elem(unsigned long long seed, long long i, unsigned thresh) {
  return (unsigned)(mix64(seed + (unsigned long long)i * 0x9E3779B97F4A7C15ull) >> 40) < thresh;
}

__device__ float block_reduce(float v, float* red, bool is_max) {
  v = is_max ? sbk::wave_max(v) : sbk::wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int k = 1; k < kThreads / 64; ++k) r = is_max ? fmaxf(r, red[k]) : r + red[k];
  return r;
}

// y[d] = sum_n w[n] * X[n][d] over n < N for d < dh; X row n at X + n * ldx
// (+ head offset already applied); w in LDS.  Four 64-lane groups split n;
// partials combine through `part` (4 * 64 floats).  Calls fn(d, y) once per d.
template <typename TI, typename F>
__device__ void weighted_rows(const float* w, const TI* X, long long ldx, int N, int dh, float* part, F fn) {
  const int dl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  for (int d0 = 0; d0 < dh; d0 += 64) {
    const int d = d0 + dl;
    float acc = 0.f;
    if (d < dh)
      for (int n = grp; n < N; n += 4) acc += w[n] * ld(X, n * ldx + d);
    __syncthreads();
    part[grp * 64 + dl] = acc;
    __syncthreads();
    if (grp == 0 && d < dh) fn(d, part[dl] + part[64 + dl] + part[128 + dl] + part[192 + dl]);
  }
}

// the source element of output (i, j) of rel_shift: returns the band row r
// and column c (c < 0: the zero pad or a mask_pos_future zero)
__device__ __forceinline__ void shift_src(int i, int j, int Lq, int P, int mpf, int& r, int& c) {
  const long long p = (long long)i * P + j + Lq;
  r = (int)(p / (P + 1));
  c = (int)(p % (P + 1)) - 1;
  if (mpf && j - i > P - Lq) c = -1;
}

template <typename TI>
__global__ __launch_bounds__(kThreads) void xattn_fwd_kernel(
    const TI* __restrict__ q, int ldq, const TI* __restrict__ k, int ldk, const TI* __restrict__ v, int ldv,
    const TI* __restrict__ pk, int ldp, int P, const float* __restrict__ pbu, const float* __restrict__ pbv,
    const unsigned char* __restrict__ kpm, const float* __restrict__ am, long long am_sb, long long am_sh, int Lq,
    int Lk, int H, int dh, float scale, int mpf, unsigned thresh, float inv_keep, unsigned long long seed,
    int use_drop, TI* __restrict__ out, int ldo, float* __restrict__ probs, float* __restrict__ attn) {
  extern __shared__ float sm[];
  float* s = sm;             // Lk scores -> probabilities (dropped)
  float* qu = s + Lk;        // q_i + u
  float* red = qu + dh;      // 64
  float* part = red + 64;    // 256
  const int i = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const TI* qrow = q + (long long)(b * Lq + i) * ldq + h * dh;
  for (int d = threadIdx.x; d < dh; d += kThreads) qu[d] = ld(qrow, d) + (pbu ? pbu[h * dh + d] : 0.f);
  __syncthreads();
  const float* am_row = am ? am + b * am_sb + h * am_sh + (long long)i * Lk : nullptr;
  float mx = -INFINITY;
  for (int j = threadIdx.x; j < Lk; j += kThreads) {
    const TI* krow = k + (long long)(b * Lk + j) * ldk + h * dh;
    float ac = 0.f;
    for (int d = 0; d < dh; ++d) ac += qu[d] * ld(krow, d);
    float bd = 0.f;
    int r = 0, c = -1;
    if (pk) shift_src(i, j, Lq, P, mpf, r, c);
    if (c >= 0) {
      const TI* qr = q + (long long)(b * Lq + r) * ldq + h * dh;
      const TI* pr = pk + (long long)c * ldp + h * dh;
      for (int d = 0; d < dh; ++d) bd += (ld(qr, d) + pbv[h * dh + d]) * ld(pr, d);
    }
    float sc = (ac + bd) * scale;
    if (am_row) sc += am_row[j];
    if (kpm && kpm[(long long)b * Lk + j]) sc = -INFINITY;
    s[j] = sc;
    mx = fmaxf(mx, sc);
  }
  mx = block_reduce(mx, red, true);
  float sum = 0.f;
  for (int j = threadIdx.x; j < Lk; j += kThreads) {
    const float e = expf(s[j] - mx);  // all -inf: NaN, as the reference's softmax
    s[j] = e;
    sum += e;
  }
  sum = block_reduce(sum, red, false);
  const float inv = 1.f / sum;
  const long long prow = (((long long)b * H + h) * Lq + i) * Lk;
  for (int j = threadIdx.x; j < Lk; j += kThreads) {
    const float pv = s[j] * inv;
    probs[prow + j] = pv;
    float pd = pv;
    if (use_drop) {
      pd = keep_elem(seed, prow + j, thresh) ? pv * inv_keep : 0.f;
      attn[prow + j] = pd;
    }
    s[j] = pd;
  }
  __syncthreads();
  TI* orow = out + (long long)(b * Lq + i) * ldo + h * dh;
  weighted_rows(s, v + (long long)b * Lk * ldv + h * dh, ldv, Lk, dh, part,
                [&](int d, float y) { st(orow, d, y); });
}

// Backward, row pass: per query row i, dP = dO·Vᵀ (through the dropout
// mask), G = P ⊙ (dP - Σ P dP) · scale (the gradient of the pre-scale
// score (ac + bd)), and dq_ac = G·K.
template <typename TI>
__global__ __launch_bounds__(kThreads) void xattn_bwd_rows_kernel(
    const TI* __restrict__ k, int ldk, const TI* __restrict__ v, int ldv, const TI* __restrict__ dO, int lddo,
    const float* __restrict__ probs, int Lq, int Lk, int H, int dh, float scale, unsigned thresh, float inv_keep,
    unsigned long long seed, int use_drop, float* __restrict__ G, float* __restrict__ dqu) {
  extern __shared__ float sm[];
  float* g = sm;           // Lk
  float* dor = g + Lk;     // dh
  float* red = dor + dh;   // 64
  float* part = red + 64;  // 256
  const int i = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const TI* drow = dO + (long long)(b * Lq + i) * lddo + h * dh;
  for (int d = threadIdx.x; d < dh; d += kThreads) dor[d] = ld(drow, d);
  __syncthreads();
  const long long prow = (((long long)b * H + h) * Lq + i) * Lk;
  float dot = 0.f;
  for (int j = threadIdx.x; j < Lk; j += kThreads) {
    const TI* vrow = v + (long long)(b * Lk + j) * ldv + h * dh;
    float dp = 0.f;
    for (int d = 0; d < dh; ++d) dp += dor[d] * ld(vrow, d);
    if (use_drop) dp = keep_elem(seed, prow + j, thresh) ? dp * inv_keep : 0.f;
    g[j] = dp;
    dot += probs[prow + j] * dp;
  }
  dot = block_reduce(dot, red, false);
  for (int j = threadIdx.x; j < Lk; j += kThreads) {
    const float gv = probs[prow + j] * (g[j] - dot) * scale;
    g[j] = gv;
    G[prow + j] = gv;
  }
  __syncthreads();
  float* dq = dqu + (long long)(b * Lq + i) * H * dh + h * dh;
  weighted_rows(g, k + (long long)b * Lk * ldk + h * dh, ldk, Lk, dh, part, [&](int d, float y) { dq[d] = y; });
}

// the band gradient dBD[r][c] of row r of batch b / head h: the G element
// whose rel_shift source is (r, c), or 0 (pad, masked, or sliced away)
__device__ __forceinline__ float dband(const float* Gbh, int r, int c, int Lq, int Lk, int P, int mpf) {
  const long long f = (long long)r * (P + 1) + c + 1 - Lq;
  if (f < 0) return 0.f;
  const int i = (int)(f / P), j = (int)(f % P);
  if (i >= Lq || j >= Lk) return 0.f;
  if (mpf && j - i > P - Lq) return 0.f;
  return Gbh[(long long)i * Lk + j];
}

// Backward, band-row pass: dq_bd[r] = Σ_c dBD[r][c] pk[c]; dq = dq_ac + dq_bd.
template <typename TI>
__global__ __launch_bounds__(kThreads) void xattn_bwd_qv_kernel(
    const TI* __restrict__ pk, int ldp, int P, const float* __restrict__ G, const float* __restrict__ dqu, int Lq,
    int Lk, int H, int dh, int mpf, float* __restrict__ dqv, float* __restrict__ dq) {
  extern __shared__ float sm[];
  float* w = sm;          // P
  float* part = w + P;    // 256
  const int r = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const float* Gbh = G + ((long long)b * H + h) * Lq * Lk;
  for (int c = threadIdx.x; c < P; c += kThreads) w[c] = dband(Gbh, r, c, Lq, Lk, P, mpf);
  __syncthreads();
  const long long o = (long long)(b * Lq + r) * H * dh + h * dh;
  weighted_rows(w, pk + h * dh, ldp, P, dh, part, [&](int d, float y) {
    dqv[o + d] = y;
    dq[o + d] = dqu[o + d] + y;
  });
}

// Backward, key-row pass: dk[j] = Σ_i G[i][j] (q_i + u), dv[j] = Σ_i Pd[i][j] dO_i.
template <typename TI>
__global__ __launch_bounds__(kThreads) void xattn_bwd_kv_kernel(
    const TI* __restrict__ q, int ldq, const TI* __restrict__ dO, int lddo, const float* __restrict__ pbu,
    const float* __restrict__ probs, const float* __restrict__ G, int Lq, int Lk, int H, int dh, unsigned thresh,
    float inv_keep, unsigned long long seed, int use_drop, float* __restrict__ dk, float* __restrict__ dv) {
  extern __shared__ float sm[];
  float* gc = sm;          // Lq: G[:, j]
  float* pc = gc + Lq;     // Lq: Pd[:, j]
  float* part = pc + Lq;   // 256
  const int j = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const long long base = ((long long)b * H + h) * Lq * Lk + j;
  float gsum = 0.f;
  for (int i = threadIdx.x; i < Lq; i += kThreads) {
    const long long e = base + (long long)i * Lk;
    gc[i] = G[e];
    float p = probs[e];
    if (use_drop) p = keep_elem(seed, e, thresh) ? p * inv_keep : 0.f;
    pc[i] = p;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < Lq; i += kThreads) gsum += gc[i];
  float* red = part;  // reused below only after this reduction completes
  gsum = block_reduce(gsum, red, false);
  __syncthreads();
  const long long o = (long long)(b * Lk + j) * H * dh + h * dh;
  // Σ_i G[i][j] (q_i + u) = Σ_i G[i][j] q_i + u Σ_i G[i][j]
  weighted_rows(gc, q + (long long)b * Lq * ldq + h * dh, ldq, Lq, dh, part,
                [&](int d, float y) { dk[o + d] = y + (pbu ? pbu[h * dh + d] * gsum : 0.f); });
  weighted_rows(pc, dO + (long long)b * Lq * lddo + h * dh, lddo, Lq, dh, part,
                [&](int d, float y) { dv[o + d] = y; });
}

// Backward, band-column pass: dpk[c] = Σ_b Σ_r dBD[b][r][c] (q_r + v).
template <typename TI>
__global__ __launch_bounds__(kThreads) void xattn_bwd_pk_kernel(
    const TI* __restrict__ q, int ldq, const float* __restrict__ pbv, const float* __restrict__ G, int B, int Lq,
    int Lk, int H, int dh, int P, int mpf, float* __restrict__ dpk) {
  extern __shared__ float sm[];
  float* w = sm;          // Lq
  float* part = w + Lq;   // 256
  float* red = part + 256;
  const int c = blockIdx.x, h = blockIdx.y;
  const int dl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int nd = (dh + 63) / 64;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};  // dh <= 256
  float wsum = 0.f;
  for (int b = 0; b < B; ++b) {
    const float* Gbh = G + ((long long)b * H + h) * Lq * Lk;
    __syncthreads();
    for (int r = threadIdx.x; r < Lq; r += kThreads) {
      const float x = dband(Gbh, r, c, Lq, Lk, P, mpf);
      w[r] = x;
      wsum += x;
    }
    __syncthreads();
    const TI* qb = q + (long long)b * Lq * ldq + h * dh;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int d = t * 64 + dl;
      if (t < nd && d < dh)
        for (int r = grp; r < Lq; r += 4) acc[t] += w[r] * ld(qb, (long long)r * ldq + d);
    }
  }
  wsum = block_reduce(wsum, red, false);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (t >= nd) break;
    const int d = t * 64 + dl;
    __syncthreads();
    part[grp * 64 + dl] = acc[t];
    __syncthreads();
    if (grp == 0 && d < dh)
      dpk[(long long)c * H * dh + h * dh + d] =
          part[dl] + part[64 + dl] + part[128 + dl] + part[192 + dl] + pbv[h * dh + d] * wsum;
  }
}

unsigned drop_thresh(float p) {
  const double keep = 1.0 - (double)p;
  return (unsigned)fmin(keep * 16777216.0, 16777216.0);
}

template <typename K>
int prep_lds(K kern, size_t lds) {
  if (lds > 160 * 1024) return SBK_ERR_ARG;
  if (sbk::lds_optin((const void*)kern, lds) != hipSuccess) return SBK_ERR_ARG;
  return 0;
}

bool bad_dims(int B, int Lq, int Lk, int H, int dh, int P) {
  return B <= 0 || Lq <= 0 || Lk <= 0 || H <= 0 || dh <= 0 || dh > 256 || P < Lk || Lq > 65535 || Lk > 65535 ||
         H > 65535 || B > 65535 || P > 65535 * 2;
}

template <typename TI>
int xattn_fwd(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, const void* pk, int ldp, int P,
              const float* pbu, const float* pbv, const unsigned char* kpm, const float* am, long long am_sb,
              long long am_sh, int B, int Lq, int Lk, int H, int dh, float scale, int mpf, float p,
              unsigned long long seed, void* out, int ldo, float* probs, float* attn, hipStream_t st) {
  const size_t lds = (size_t)(Lk + dh + 64 + 256) * sizeof(float);
  auto kern = xattn_fwd_kernel<TI>;
  if (int rc = prep_lds(kern, lds)) return rc;
  const int use_drop = p > 0.f;
  if (use_drop && !attn) return SBK_ERR_ARG;
  hipLaunchKernelGGL(kern, dim3(Lq, H, B), dim3(kThreads), lds, st, (const TI*)q, ldq, (const TI*)k, ldk,
                     (const TI*)v, ldv, (const TI*)pk, ldp, P, pbu, pbv, kpm, am, am_sb, am_sh, Lq, Lk, H, dh, scale,
                     mpf, drop_thresh(p), (float)(1.0 / (1.0 - (double)p)), seed, use_drop, (TI*)out, ldo, probs,
                     attn);
  SBK_CHECK_LAUNCH();
  return 0;
}

template <typename TI>
int xattn_bwd(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, const void* pk, int ldp, int P,
              const float* pbu, const float* pbv, const float* probs, const void* dO, int lddo, int B, int Lq, int Lk,
              int H, int dh, float scale, int mpf, float p, unsigned long long seed, float* G, float* dqu, float* dqv,
              float* dq, float* dk, float* dv, float* dpk, hipStream_t st) {
  const unsigned thresh = drop_thresh(p);
  const float inv_keep = (float)(1.0 / (1.0 - (double)p));
  const int use_drop = p > 0.f;
  {
    const size_t lds = (size_t)(Lk + dh + 64 + 256) * sizeof(float);
    auto kern = xattn_bwd_rows_kernel<TI>;
    if (int rc = prep_lds(kern, lds)) return rc;
    hipLaunchKernelGGL(kern, dim3(Lq, H, B), dim3(kThreads), lds, st, (const TI*)k, ldk, (const TI*)v, ldv,
                       (const TI*)dO, lddo, probs, Lq, Lk, H, dh, scale, thresh, inv_keep, seed, use_drop, G,
                       pk ? dqu : dq);
    SBK_CHECK_LAUNCH();
  }
  if (pk) {
    const size_t lds = (size_t)(P + 256) * sizeof(float);
    auto kern = xattn_bwd_qv_kernel<TI>;
    if (int rc = prep_lds(kern, lds)) return rc;
    hipLaunchKernelGGL(kern, dim3(Lq, H, B), dim3(kThreads), lds, st, (const TI*)pk, ldp, P, G, dqu, Lq, Lk, H, dh,
                       mpf, dqv, dq);
    SBK_CHECK_LAUNCH();
  }
  {
    const size_t lds = (size_t)(2 * Lq + 256) * sizeof(float);
    auto kern = xattn_bwd_kv_kernel<TI>;
    if (int rc = prep_lds(kern, lds)) return rc;
    hipLaunchKernelGGL(kern, dim3(Lk, H, B), dim3(kThreads), lds, st, (const TI*)q, ldq, (const TI*)dO, lddo, pbu,
                       probs, G, Lq, Lk, H, dh, thresh, inv_keep, seed, use_drop, dk, dv);
    SBK_CHECK_LAUNCH();
  }
  if (pk) {
    const size_t lds = (size_t)(Lq + 256 + 64) * sizeof(float);
    auto kern = xattn_bwd_pk_kernel<TI>;
    if (int rc = prep_lds(kern, lds)) return rc;
    hipLaunchKernelGGL(kern, dim3(P, H, 1), dim3(kThreads), lds, st, (const TI*)q, ldq, pbv, G, B, Lq, Lk, H, dh, P,
                       mpf, dpk);
    SBK_CHECK_LAUNCH();
  }
  return 0;
}

}  // namespace

SBK_API int sbk_relpos_xattn_fwd(int dtype_bf16, const void* q, int ldq, const void* k, int ldk, const void* v,
                                 int ldv, const void* pk, int ldp, int P, const float* pbu, const float* pbv,
                                 const unsigned char* kpm, const float* am, long long am_sb, long long am_sh, int B,
                                 int Lq, int Lk, int H, int dh, float scale, int mask_pos_future, float p_drop,
                                 unsigned long long seed, void* out, int ldo, float* probs, float* attn,
                                 void* stream) {
  if (!q || !k || !v || (pk && (!pbu || !pbv || ldp < H * dh)) || !out || !probs || bad_dims(B, Lq, Lk, H, dh, P) ||
      p_drop < 0.f || p_drop >= 1.f || ldq < H * dh || ldk < H * dh || ldv < H * dh || ldo < H * dh)
    return SBK_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  return dtype_bf16 ? xattn_fwd<uint16_t>(q, ldq, k, ldk, v, ldv, pk, ldp, P, pbu, pbv, kpm, am, am_sb, am_sh, B, Lq,
                                          Lk, H, dh, scale, mask_pos_future, p_drop, seed, out, ldo, probs, attn, st)
                    : xattn_fwd<float>(q, ldq, k, ldk, v, ldv, pk, ldp, P, pbu, pbv, kpm, am, am_sb, am_sh, B, Lq, Lk,
                                       H, dh, scale, mask_pos_future, p_drop, seed, out, ldo, probs, attn, st);
}

SBK_API int sbk_relpos_xattn_bwd(int dtype_bf16, const void* q, int ldq, const void* k, int ldk, const void* v,
                                 int ldv, const void* pk, int ldp, int P, const float* pbu, const float* pbv,
                                 const float* probs, const void* dO, int lddo, int B, int Lq, int Lk, int H, int dh,
                                 float scale, int mask_pos_future, float p_drop, unsigned long long seed, float* G,
                                 float* dqu, float* dqv, float* dq, float* dk, float* dv, float* dpk, void* stream) {
  if (!q || !k || !v || !probs || !dO || !G || !dq || !dk || !dv ||
      (pk && (!pbu || !pbv || !dqu || !dqv || !dpk || ldp < H * dh)) || bad_dims(B, Lq, Lk, H, dh, P) ||
      p_drop < 0.f || p_drop >= 1.f || ldq < H * dh || ldk < H * dh || ldv < H * dh || lddo < H * dh)
    return SBK_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  return dtype_bf16 ? xattn_bwd<uint16_t>(q, ldq, k, ldk, v, ldv, pk, ldp, P, pbu, pbv, probs, dO, lddo, B, Lq, Lk, H,
                                          dh, scale, mask_pos_future, p_drop, seed, G, dqu, dqv, dq, dk, dv, dpk, st)
                    : xattn_bwd<float>(q, ldq, k, ldk, v, ldv, pk, ldp, P, pbu, pbv, probs, dO, lddo, B, Lq, Lk, H,
                                       dh, scale, mask_pos_future, p_drop, seed, G, dqu, dqv, dq, dk, dv, dpk, st);
}
