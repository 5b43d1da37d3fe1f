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

#include <initializer_list>

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

// No-position forward (pk == nullptr), query-blocked: one workgroup per
// (QB query rows, head, batch).  The per-row kernel above gives every
// score its own thread and walks a key row dimension by dimension, so a
// wave reads 64 different rows element-wise and every query row re-reads
// all of K and V (decoder cross-attention over 376 keys: 1.2-2x torch's
// GEMM-based MHA, profiles/r06u_mha_decoder_timing.log).  Here K and V pass
// through LDS in chunks of XQ_KC rows, read once per QB query rows with
// coalesced loads, the scores of the block stay in LDS (QB x Lk) for the
// softmax, and P·V accumulates per (row, 8 output dims); the LDS rows are
// padded to dh + 4 floats so the dot products read 16 B at a time, the 16
// key rows of a lane group 4 banks apart.  fp32 VALU as above (exact fp32
// operands for the parity path).
constexpr int XQ_QB = 16, XQ_KC = 64, XQ_DMAX = 128, XQ_LKMAX = 1024;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 ld4(const uint16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}
// ROWS x dh of src (row stride ld_src elements, 4-element aligned) -> dst
// (row stride ld_dst floats); rows >= rmax -> 0.  Every load of the thread
// is issued before the first LDS store (a load -> store loop per element
// paid the global latency once per element: the first version of these
// kernels spent most of its time there).
template <int ROWS, typename TI>
__device__ __forceinline__ void xq_stage(float* dst, int ld_dst, const TI* src, long long ld_src, int rmax, int dh) {
  constexpr int PT = (ROWS * (XQ_DMAX / 4) + kThreads - 1) / kThreads;  // float4 per thread at dh = XQ_DMAX
  const int q4 = dh >> 2, total = ROWS * q4;
  float4 v[PT];
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    const int e = threadIdx.x + u * kThreads;
    v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < total) {
      const int r = e / q4, c = (e - r * q4) * 4;
      if (r < rmax) v[u] = ld4(src + (long long)r * ld_src + c);
    }
  }
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    const int e = threadIdx.x + u * kThreads;
    if (e < total) {
      const int r = e / q4, c = (e - r * q4) * 4;
      *reinterpret_cast<float4*>(dst + r * ld_dst + c) = v[u];
    }
  }
}

// POS: the rel-pos band term as well.  Output (i, j) takes band element
// (r, c) = shift_src(i, j); for the common r == i it is (q_i + v)·pk_c with
// c = j - i + Lq - 1, so the (QB + KC - 1) band rows a block-chunk needs are
// staged beside the K chunk (XQ_BR rows from c_base); the wrap rows of the
// reference's rel_shift (r > i: q_len > k_len) read global memory.
constexpr int XQ_BR = XQ_QB + XQ_KC;  // staged band rows per chunk (79 used)

template <int ROWS, typename TI>
__device__ __forceinline__ void xq_stage_rows(float* dst, int ld_dst, const TI* src, long long ld_src, int row0,
                                              int rows_total, int dh) {
  // rows row0 .. row0 + ROWS - 1 of src (rows outside [0, rows_total) -> 0)
  constexpr int PT = (ROWS * (XQ_DMAX / 4) + kThreads - 1) / kThreads;
  const int q4 = dh >> 2, total = ROWS * q4;
  float4 v[PT];
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    const int e = threadIdx.x + u * kThreads;
    v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < total) {
      const int r = e / q4, c = (e - r * q4) * 4, gr = row0 + r;
      if (gr >= 0 && gr < rows_total) v[u] = ld4(src + (long long)gr * ld_src + c);
    }
  }
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    const int e = threadIdx.x + u * kThreads;
    if (e < total) {
      const int r = e / q4, c = (e - r * q4) * 4;
      *reinterpret_cast<float4*>(dst + r * ld_dst + c) = v[u];
    }
  }
}

template <typename TI, bool POS>
__global__ __launch_bounds__(kThreads) void xattn_fwd_qb_kernel(
    const TI* __restrict__ q, int ldq, const TI* __restrict__ k, int ldk, const TI* __restrict__ v, int ldv,
    const TI* __restrict__ pk, int ldp, int P, const float* __restrict__ pbu, const float* __restrict__ pbv, int mpf,
    const unsigned char* __restrict__ kpm, const float* __restrict__ am, long long am_sb, long long am_sh, int Lq,
    int Lk, int H, int dh, float scale, unsigned thresh, float inv_keep, unsigned long long seed, int use_drop,
    TI* __restrict__ out, int ldo, float* __restrict__ probs, float* __restrict__ attn) {
  extern __shared__ float sm[];
  const int DP = dh + 4;                   // padded LDS row (floats): 16-B aligned, rows 4 banks apart
  float* qs = sm;                          // XQ_QB x DP (POS: q + u)
  float* kv = qs + XQ_QB * DP;             // XQ_KC x DP (K chunk, then V chunk)
  float* qv = kv + XQ_KC * DP;             // POS: XQ_QB x DP, q + v
  float* band = qv + (POS ? XQ_QB * DP : 0);  // POS: XQ_BR x DP band rows from c_base
  float* s = band + (POS ? XQ_BR * DP : 0);   // XQ_QB x Lk scores -> probabilities (dropped)
  const int i0 = blockIdx.x * XQ_QB, h = blockIdx.y, b = blockIdx.z;
  const int nq = min(XQ_QB, Lq - i0);
  const int tid = threadIdx.x, ri = tid >> 4, sub = tid & 15;  // row ri, 16 threads per row
  const TI* qblk = q + (long long)(b * Lq + i0) * ldq + h * dh;
  xq_stage<XQ_QB>(qs, DP, qblk, ldq, nq, dh);
  if constexpr (POS) {
    xq_stage<XQ_QB>(qv, DP, qblk, ldq, nq, dh);
    __syncthreads();
    for (int e = tid; e < XQ_QB * dh; e += kThreads) {
      const int r = e / dh, d = e - r * dh;
      qs[r * DP + d] += pbu[h * dh + d];
      qv[r * DP + d] += pbv[h * dh + d];
    }
  }
  const int i = i0 + ri;
  // scores: thread (ri, sub) takes keys j0 + sub + 16 m of each chunk
  for (int j0 = 0; j0 < Lk; j0 += XQ_KC) {
    const int nk = min(XQ_KC, Lk - j0);
    const int cb = j0 - i0 - (XQ_QB - 1) + Lq - 1;  // band row of (i0 + 15, j0) when r == i
    __syncthreads();  // the previous chunk's readers are done (and qs is staged)
    xq_stage<XQ_KC>(kv, DP, k + (long long)(b * Lk + j0) * ldk + h * dh, ldk, nk, dh);
    if constexpr (POS) xq_stage_rows<XQ_BR>(band, DP, pk + h * dh, ldp, cb, P, dh);
    __syncthreads();
    float ac[XQ_KC / 16] = {};
    float bd[XQ_KC / 16] = {};
    int bro[XQ_KC / 16];  // POS: LDS band row of each key (-1: zero term; -2: wrap row, global)
    int wr[XQ_KC / 16], wc[XQ_KC / 16];
    if constexpr (POS) {
#pragma unroll
      for (int m = 0; m < XQ_KC / 16; ++m) {
        const int j = j0 + sub + 16 * m;
        int r = 0, c = -1;
        if (j < Lk && ri < nq) shift_src(i, j, Lq, P, mpf, r, c);
        wr[m] = r;
        wc[m] = c;
        bro[m] = c < 0 ? -1 : (r == i && c - cb >= 0 && c - cb < XQ_BR) ? c - cb : -2;
      }
    }
    const float* qr = qs + ri * DP;
    const float* vr = qv + ri * DP;
    for (int d = 0; d < dh; d += 4) {
      const float4 qd = *reinterpret_cast<const float4*>(qr + d);
      float4 vd;
      if constexpr (POS) vd = *reinterpret_cast<const float4*>(vr + d);
#pragma unroll
      for (int m = 0; m < XQ_KC / 16; ++m) {
        const float4 kd = *reinterpret_cast<const float4*>(kv + (sub + 16 * m) * DP + d);
        ac[m] += qd.x * kd.x + qd.y * kd.y + qd.z * kd.z + qd.w * kd.w;
        if constexpr (POS) {
          const float4 pd = *reinterpret_cast<const float4*>(band + max(bro[m], 0) * DP + d);
          bd[m] += vd.x * pd.x + vd.y * pd.y + vd.z * pd.z + vd.w * pd.w;
        }
      }
    }
    if constexpr (POS) {
#pragma unroll
      for (int m = 0; m < XQ_KC / 16; ++m) {
        if (bro[m] == -1) bd[m] = 0.f;
        if (bro[m] == -2) {  // rel_shift wrap row (r > i): (q_r + v)·pk_c from global memory
          const TI* qrow = q + (long long)(b * Lq + wr[m]) * ldq + h * dh;
          const TI* prow = pk + (long long)wc[m] * ldp + h * dh;
          float t = 0.f;
          for (int d = 0; d < dh; ++d) t += (ld(qrow, d) + pbv[h * dh + d]) * ld(prow, d);
          bd[m] = t;
        }
      }
    }
    const float* am_row = (am && ri < nq) ? am + b * am_sb + h * am_sh + (long long)i * Lk : nullptr;
#pragma unroll
    for (int m = 0; m < XQ_KC / 16; ++m) {
      const int j = j0 + sub + 16 * m;
      if (j >= Lk) continue;
      float sc = (ac[m] + bd[m]) * scale;
      if (am_row) sc += am_row[j];
      if (kpm && kpm[(long long)b * Lk + j]) sc = -INFINITY;
      s[ri * Lk + j] = sc;
    }
  }
  __syncthreads();
  // softmax per row: 16 threads per row (lanes 16 ri' .. of one wave), xor shuffles within the 16
  float mx = -INFINITY;
  for (int j = sub; j < Lk; j += 16) mx = fmaxf(mx, s[ri * Lk + j]);
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 16));
  float sum = 0.f;
  for (int j = sub; j < Lk; j += 16) {
    const float e = expf(s[ri * Lk + j] - mx);  // all -inf: NaN, as the reference's softmax
    s[ri * Lk + j] = e;
    sum += e;
  }
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 16);
  const float inv = 1.f / sum;
  const long long prow = (((long long)b * H + h) * Lq + i0 + ri) * Lk;
  for (int j = sub; j < Lk; j += 16) {
    const float pv = s[ri * Lk + j] * inv;
    float pd = pv;
    if (ri < nq) {
      probs[prow + j] = pv;
      if (use_drop) {
        pd = keep_elem(seed, prow + j, thresh) ? pv * inv_keep : 0.f;
        attn[prow + j] = pd;
      }
    }
    s[ri * Lk + j] = pd;
  }
  // out[ri][8 sub .. 8 sub + 7] (+ 128 per extra pass for dh > 128: not taken, dh <= XQ_DMAX)
  float acc[8] = {};
  const int d0 = 8 * sub;
  for (int j0 = 0; j0 < Lk; j0 += XQ_KC) {
    const int nk = min(XQ_KC, Lk - j0);
    __syncthreads();
    xq_stage<XQ_KC>(kv, DP, v + (long long)(b * Lk + j0) * ldv + h * dh, ldv, nk, dh);
    __syncthreads();
    if (d0 < dh)
      for (int jj = 0; jj < nk; ++jj) {
        const float pj = s[ri * Lk + j0 + jj];
        const float4 va = *reinterpret_cast<const float4*>(kv + jj * DP + d0);
        const float4 vb = *reinterpret_cast<const float4*>(kv + jj * DP + d0 + 4);
        acc[0] += pj * va.x; acc[1] += pj * va.y; acc[2] += pj * va.z; acc[3] += pj * va.w;
        acc[4] += pj * vb.x; acc[5] += pj * vb.y; acc[6] += pj * vb.z; acc[7] += pj * vb.w;
      }
  }
  if (ri < nq && d0 < dh) {
    TI* orow = out + (long long)(b * Lq + i0 + ri) * ldo + h * dh;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (d0 + e < dh) st(orow, d0 + e, acc[e]);
  }
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

// No-position backward row pass, query-blocked like xattn_fwd_qb_kernel:
// dP = dO·Vᵀ over V chunks in LDS, G = P ⊙ (dP - Σ P dP) · scale (written
// to global for the key-row pass), dq = G·K over K chunks in LDS.
template <typename TI>
__global__ __launch_bounds__(kThreads) void xattn_bwd_rows_qb_kernel(
    const TI* __restrict__ k, int ldk, const TI* __restrict__ v, int ldv, const TI* __restrict__ dO, int lddo,
    const float* __restrict__ probs, int Lq, int Lk, int H, int dh, float scale, unsigned thresh, float inv_keep,
    unsigned long long seed, int use_drop, float* __restrict__ G, float* __restrict__ dq) {
  extern __shared__ float sm[];
  const int DP = dh + 4;
  float* ds = sm;                          // XQ_QB x DP: dO rows
  float* kv = ds + XQ_QB * DP;             // XQ_KC x DP: V chunk, then K chunk
  float* g = kv + XQ_KC * DP;              // XQ_QB x Lk: dP, then G
  const int i0 = blockIdx.x * XQ_QB, h = blockIdx.y, b = blockIdx.z;
  const int nq = min(XQ_QB, Lq - i0);
  const int tid = threadIdx.x, ri = tid >> 4, sub = tid & 15;
  xq_stage<XQ_QB>(ds, DP, dO + (long long)(b * Lq + i0) * lddo + h * dh, lddo, nq, dh);
  const long long prow = (((long long)b * H + h) * Lq + i0 + ri) * Lk;
  for (int j0 = 0; j0 < Lk; j0 += XQ_KC) {
    const int nk = min(XQ_KC, Lk - j0);
    __syncthreads();
    xq_stage<XQ_KC>(kv, DP, v + (long long)(b * Lk + j0) * ldv + h * dh, ldv, nk, dh);
    __syncthreads();
    float dp[XQ_KC / 16] = {};
    const float* dr = ds + ri * DP;
    for (int d = 0; d < dh; d += 4) {
      const float4 od = *reinterpret_cast<const float4*>(dr + d);
#pragma unroll
      for (int m = 0; m < XQ_KC / 16; ++m) {
        const float4 vd = *reinterpret_cast<const float4*>(kv + (sub + 16 * m) * DP + d);
        dp[m] += od.x * vd.x + od.y * vd.y + od.z * vd.z + od.w * vd.w;
      }
    }
#pragma unroll
    for (int m = 0; m < XQ_KC / 16; ++m) {
      const int j = j0 + sub + 16 * m;
      if (j >= Lk) continue;
      float x = dp[m];
      if (use_drop && ri < nq) x = keep_elem(seed, prow + j, thresh) ? x * inv_keep : 0.f;
      g[ri * Lk + j] = x;
    }
  }
  __syncthreads();
  float dot = 0.f;
  if (ri < nq)
    for (int j = sub; j < Lk; j += 16) dot += probs[prow + j] * g[ri * Lk + j];
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) dot += __shfl_xor(dot, o, 16);
  for (int j = sub; j < Lk; j += 16) {
    float gv = 0.f;
    if (ri < nq) {
      gv = probs[prow + j] * (g[ri * Lk + j] - dot) * scale;
      G[prow + j] = gv;
    }
    g[ri * Lk + j] = gv;
  }
  float acc[8] = {};
  const int d0 = 8 * sub;
  for (int j0 = 0; j0 < Lk; j0 += XQ_KC) {
    const int nk = min(XQ_KC, Lk - j0);
    __syncthreads();
    xq_stage<XQ_KC>(kv, DP, k + (long long)(b * Lk + j0) * ldk + h * dh, ldk, nk, dh);
    __syncthreads();
    if (d0 < dh)
      for (int jj = 0; jj < nk; ++jj) {
        const float gj = g[ri * Lk + j0 + jj];
        const float4 ka = *reinterpret_cast<const float4*>(kv + jj * DP + d0);
        const float4 kb = *reinterpret_cast<const float4*>(kv + jj * DP + d0 + 4);
        acc[0] += gj * ka.x; acc[1] += gj * ka.y; acc[2] += gj * ka.z; acc[3] += gj * ka.w;
        acc[4] += gj * kb.x; acc[5] += gj * kb.y; acc[6] += gj * kb.z; acc[7] += gj * kb.w;
      }
  }
  if (ri < nq && d0 < dh) {
    float* dqr = dq + (long long)(b * Lq + i0 + ri) * H * dh + h * dh;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (d0 + e < dh) dqr[d0 + e] = acc[e];
  }
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

// Key-row pass, key-blocked (dh <= XQ_DMAX): one workgroup per (XQ_QB key
// rows, head, batch) walks the query rows in chunks of XQ_KC: the G / P
// column slices of its keys (16 consecutive floats of each row) and the q /
// dO rows of the chunk go through LDS, thread (key row, 8 dims) accumulates
// dk and dv.  (The per-key kernel above read each G / P column element by
// element at a stride of Lk: 25 % of a decoder cross-attention's backward.)
template <typename TI>
__global__ __launch_bounds__(kThreads) void xattn_bwd_kv_qb_kernel(
    const TI* __restrict__ q, int ldq, const TI* __restrict__ dO, int lddo, const float* __restrict__ pbu,
    const float* __restrict__ probs, const float* __restrict__ G, int Lq, int Lk, int H, int dh, unsigned thresh,
    float inv_keep, unsigned long long seed, int use_drop, float* __restrict__ dk, float* __restrict__ dv) {
  extern __shared__ float sm[];
  const int DP = dh + 4;
  float* gs = sm;                    // XQ_KC x XQ_QB: G[i][j0 + jj]
  float* ps = gs + XQ_KC * XQ_QB;    // XQ_KC x XQ_QB: Pd
  float* qs = ps + XQ_KC * XQ_QB;    // XQ_KC x DP: q rows
  float* os = qs + XQ_KC * DP;       // XQ_KC x DP: dO rows
  const int j0 = blockIdx.x * XQ_QB, h = blockIdx.y, b = blockIdx.z;
  const int nj = min(XQ_QB, Lk - j0);
  const int tid = threadIdx.x, rj = tid >> 4, sub = tid & 15, d0 = 8 * sub;
  const long long gbase = ((long long)b * H + h) * Lq * Lk + j0;
  float adk[8] = {}, adv[8] = {};
  float gsum = 0.f;
  for (int i0 = 0; i0 < Lq; i0 += XQ_KC) {
    const int ni = min(XQ_KC, Lq - i0);
    __syncthreads();
    for (int e = tid; e < XQ_KC * XQ_QB; e += kThreads) {
      const int ii = e / XQ_QB, jj = e - ii * XQ_QB;
      float gv = 0.f, pv = 0.f;
      if (ii < ni && jj < nj) {
        const long long x = gbase + (long long)(i0 + ii) * Lk + jj;
        gv = G[x];
        pv = probs[x];
        if (use_drop) pv = keep_elem(seed, x, thresh) ? pv * inv_keep : 0.f;
      }
      gs[e] = gv;
      ps[e] = pv;
    }
    xq_stage<XQ_KC>(qs, DP, q + (long long)(b * Lq + i0) * ldq + h * dh, ldq, ni, dh);
    xq_stage<XQ_KC>(os, DP, dO + (long long)(b * Lq + i0) * lddo + h * dh, lddo, ni, dh);
    __syncthreads();
    if (d0 < dh)
      for (int ii = 0; ii < ni; ++ii) {
        const float gj = gs[ii * XQ_QB + rj], pj = ps[ii * XQ_QB + rj];
        gsum += gj;
        const float4 qa = *reinterpret_cast<const float4*>(qs + ii * DP + d0);
        const float4 qb = *reinterpret_cast<const float4*>(qs + ii * DP + d0 + 4);
        const float4 oa = *reinterpret_cast<const float4*>(os + ii * DP + d0);
        const float4 ob = *reinterpret_cast<const float4*>(os + ii * DP + d0 + 4);
        adk[0] += gj * qa.x; adk[1] += gj * qa.y; adk[2] += gj * qa.z; adk[3] += gj * qa.w;
        adk[4] += gj * qb.x; adk[5] += gj * qb.y; adk[6] += gj * qb.z; adk[7] += gj * qb.w;
        adv[0] += pj * oa.x; adv[1] += pj * oa.y; adv[2] += pj * oa.z; adv[3] += pj * oa.w;
        adv[4] += pj * ob.x; adv[5] += pj * ob.y; adv[6] += pj * ob.z; adv[7] += pj * ob.w;
      }
  }
  if (rj < nj && d0 < dh) {
    const long long o = (long long)(b * Lk + j0 + rj) * H * dh + h * dh;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (d0 + e < dh) {
        dk[o + d0 + e] = adk[e] + (pbu ? pbu[h * dh + d0 + e] * gsum : 0.f);
        dv[o + d0 + e] = adv[e];
      }
  }
}

// Band-row pass, blocked (dh <= XQ_DMAX, 16-B aligned pk): one workgroup
// per (XQ_QB band rows, head, batch) walks the band in chunks of XQ_KC
// rows staged through LDS (the per-row kernel above re-read all P rows of
// pk for every band row): w[r][c] = dBD[r][c] of the chunk into LDS, then
// thread (row, 8 dims) accumulates dq_bd = Σ_c w pk_c.
template <typename TI>
__global__ __launch_bounds__(kThreads) void xattn_bwd_qv_qb_kernel(
    const TI* __restrict__ pk, int ldp, int P, const float* __restrict__ G, const float* __restrict__ dqu, int Lq,
    int Lk, int H, int dh, int mpf, float* __restrict__ dqv, float* __restrict__ dq) {
  extern __shared__ float sm[];
  const int DP = dh + 4;
  float* ps = sm;                      // XQ_KC x DP: pk rows of the chunk
  float* w = ps + XQ_KC * DP;          // XQ_QB x XQ_KC: dBD of the chunk
  const int r0 = blockIdx.x * XQ_QB, h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, ri = tid >> 4, sub = tid & 15, d0 = 8 * sub;
  const float* Gbh = G + ((long long)b * H + h) * Lq * Lk;
  float acc[8] = {};
  for (int c0 = 0; c0 < P; c0 += XQ_KC) {
    const int nc = min(XQ_KC, P - c0);
    __syncthreads();
    xq_stage<XQ_KC>(ps, DP, pk + (long long)c0 * ldp + h * dh, ldp, nc, dh);
    for (int e = tid; e < XQ_QB * XQ_KC; e += kThreads) {
      const int rr = e / XQ_KC, cc = e - rr * XQ_KC;
      w[e] = (r0 + rr < Lq && cc < nc) ? dband(Gbh, r0 + rr, c0 + cc, Lq, Lk, P, mpf) : 0.f;
    }
    __syncthreads();
    if (d0 < dh)
      for (int cc = 0; cc < nc; ++cc) {
        const float wc = w[ri * XQ_KC + cc];
        const float4 pa = *reinterpret_cast<const float4*>(ps + cc * DP + d0);
        const float4 pb = *reinterpret_cast<const float4*>(ps + cc * DP + d0 + 4);
        acc[0] += wc * pa.x; acc[1] += wc * pa.y; acc[2] += wc * pa.z; acc[3] += wc * pa.w;
        acc[4] += wc * pb.x; acc[5] += wc * pb.y; acc[6] += wc * pb.z; acc[7] += wc * pb.w;
      }
  }
  if (r0 + ri < Lq && d0 < dh) {
    const long long o = (long long)(b * Lq + r0 + ri) * H * dh + h * dh;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (d0 + e < dh) {
        dqv[o + d0 + e] = acc[e];
        dq[o + d0 + e] = dqu[o + d0 + e] + acc[e];
      }
  }
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

// operands the query-blocked kernels can stage 4 elements at a time
template <typename TI>
bool qb_aligned(std::initializer_list<const void*> ps, std::initializer_list<int> lds, int dh) {
  if (dh > XQ_DMAX || dh % 4) return false;
  for (const void* p : ps)
    if (reinterpret_cast<uintptr_t>(p) % (4 * sizeof(TI))) return false;
  for (int l : lds)
    if (l % 4) return false;
  return true;
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
  const int use_drop = p > 0.f;
  if (use_drop && !attn) return SBK_ERR_ARG;
  const size_t lq = (size_t)((XQ_QB + XQ_KC + (pk ? XQ_QB + XQ_BR : 0)) * (dh + 4) + XQ_QB * Lk) * sizeof(float);
  if (Lk <= XQ_LKMAX && lq <= 160 * 1024 &&
      (pk ? qb_aligned<TI>({q, k, v, pk}, {ldq, ldk, ldv, ldp}, dh) : qb_aligned<TI>({q, k, v}, {ldq, ldk, ldv}, dh))) {
    const dim3 grid((Lq + XQ_QB - 1) / XQ_QB, H, B);
    const unsigned th = drop_thresh(p);
    const float ik = (float)(1.0 / (1.0 - (double)p));
    if (pk) {
      auto kq = xattn_fwd_qb_kernel<TI, true>;
      if (int rc = prep_lds(kq, lq)) return rc;
      hipLaunchKernelGGL(kq, grid, dim3(kThreads), lq, st, (const TI*)q, ldq, (const TI*)k, ldk, (const TI*)v, ldv,
                         (const TI*)pk, ldp, P, pbu, pbv, mpf, kpm, am, am_sb, am_sh, Lq, Lk, H, dh, scale, th, ik,
                         seed, use_drop, (TI*)out, ldo, probs, attn);
    } else {
      auto kq = xattn_fwd_qb_kernel<TI, false>;
      if (int rc = prep_lds(kq, lq)) return rc;
      hipLaunchKernelGGL(kq, grid, dim3(kThreads), lq, st, (const TI*)q, ldq, (const TI*)k, ldk, (const TI*)v, ldv,
                         (const TI*)nullptr, 0, 0, (const float*)nullptr, (const float*)nullptr, 0, kpm, am, am_sb,
                         am_sh, Lq, Lk, H, dh, scale, th, ik, seed, use_drop, (TI*)out, ldo, probs, attn);
    }
    SBK_CHECK_LAUNCH();
    return 0;
  }
  const size_t lds = (size_t)(Lk + dh + 64 + 256) * sizeof(float);
  auto kern = xattn_fwd_kernel<TI>;
  if (int rc = prep_lds(kern, lds)) return rc;
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
  if (Lk <= XQ_LKMAX && qb_aligned<TI>({k, v, dO}, {ldk, ldv, lddo}, dh)) {
    const size_t lq = (size_t)((XQ_QB + XQ_KC) * (dh + 4) + XQ_QB * Lk) * sizeof(float);
    auto kq = xattn_bwd_rows_qb_kernel<TI>;
    if (int rc = prep_lds(kq, lq)) return rc;
    hipLaunchKernelGGL(kq, dim3((Lq + XQ_QB - 1) / XQ_QB, H, B), dim3(kThreads), lq, st, (const TI*)k, ldk,
                       (const TI*)v, ldv, (const TI*)dO, lddo, probs, Lq, Lk, H, dh, scale, thresh, inv_keep, seed,
                       use_drop, G, pk ? dqu : dq);
    SBK_CHECK_LAUNCH();
  } else {
    const size_t lds = (size_t)(Lk + dh + 64 + 256) * sizeof(float);
    auto kern = xattn_bwd_rows_kernel<TI>;
    if (int rc = prep_lds(kern, lds)) return rc;
    hipLaunchKernelGGL(kern, dim3(Lq, H, B), dim3(kThreads), lds, st, (const TI*)k, ldk, (const TI*)v, ldv,
                       (const TI*)dO, lddo, probs, Lq, Lk, H, dh, scale, thresh, inv_keep, seed, use_drop, G,
                       pk ? dqu : dq);
    SBK_CHECK_LAUNCH();
  }
  if (pk && qb_aligned<TI>({pk}, {ldp}, dh)) {
    const size_t lq = (size_t)(XQ_KC * (dh + 4) + XQ_QB * XQ_KC) * sizeof(float);
    auto kq = xattn_bwd_qv_qb_kernel<TI>;
    if (int rc = prep_lds(kq, lq)) return rc;
    hipLaunchKernelGGL(kq, dim3((Lq + XQ_QB - 1) / XQ_QB, H, B), dim3(kThreads), lq, st, (const TI*)pk, ldp, P, G,
                       dqu, Lq, Lk, H, dh, mpf, dqv, dq);
    SBK_CHECK_LAUNCH();
  } else if (pk) {
    const size_t lds = (size_t)(P + 256) * sizeof(float);
    auto kern = xattn_bwd_qv_kernel<TI>;
    if (int rc = prep_lds(kern, lds)) return rc;
    hipLaunchKernelGGL(kern, dim3(Lq, H, B), dim3(kThreads), lds, st, (const TI*)pk, ldp, P, G, dqu, Lq, Lk, H, dh,
                       mpf, dqv, dq);
    SBK_CHECK_LAUNCH();
  }
  if (qb_aligned<TI>({q, dO}, {ldq, lddo}, dh)) {
    const size_t lq = (size_t)(2 * XQ_KC * XQ_QB + 2 * XQ_KC * (dh + 4)) * sizeof(float);
    auto kq = xattn_bwd_kv_qb_kernel<TI>;
    if (int rc = prep_lds(kq, lq)) return rc;
    hipLaunchKernelGGL(kq, dim3((Lk + XQ_QB - 1) / XQ_QB, H, B), dim3(kThreads), lq, st, (const TI*)q, ldq,
                       (const TI*)dO, lddo, pbu, probs, G, Lq, Lk, H, dh, thresh, inv_keep, seed, use_drop, dk, dv);
    SBK_CHECK_LAUNCH();
  } else {
    const size_t lds = (size_t)(2 * Lq + 256) * sizeof(float);
    auto kern = xattn_bwd_kv_kernel<TI>;
    if (int rc = prep_lds(kern, lds)) return rc;
    hipLaunchKernelGGL(kern, dim3(Lk, H, B), dim3(kThreads), lds, st, (const TI*)q, ldq, (const TI*)dO, lddo, pbu,
                       probs, G, Lq, Lk, H, dh, thresh, inv_keep, seed, use_drop, dk, dv);
    SBK_CHECK_LAUNCH();
  }
  if (pk) {  // (a column-blocked variant over 188 workgroups measured 2x slower: 550 vs 276 us)
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
