// MFMA GEMM with fused epilogues for the Conformer projections.
//
//   C[M, N] = epilogue( A[M, K] · W[N, K]^T )
//
// A: activations (row-major, lda), W: nn.Linear weight layout [out][in]
// (K contiguous) — both operands are K-contiguous, so every MFMA fragment is
// one 16-byte LDS read for bf16 (two for f32).  Tiles: 4 waves (2x2), each
// wave owns a (BM/2)x(BN/2) block of 16x16 MFMA tiles; K staged through a
// double-buffered LDS ring (register prefetch of tile k+1 overlaps the MFMAs
// of tile k, one barrier per K tile).
//
// Epilogues (fused so no activation makes an extra HBM round trip):
//   bias, activation (Swish / GLU / LeakyReLU), row mask (padding frames ->
//   0), residual  out = res + alpha * val,  fp32 or bf16 output.
// These implement speechbrain nn.Linear / Conv1d(k=1) sites:
//   attention.py:549-553 (in_proj), :581 (linear_pos), :636 (out_proj),
//   :823-839 (FFN Linear-Swish-Linear), Conformer.py:73-79,105 (pointwise
//   conv + GLU), :87-92 (after_conv Linear), :243,:259 (0.5-scaled residuals),
//   TransformerASR.py:127-135 (custom_src_module Linear).
#include "mfma.h"
#include "gemm256.h"

using namespace sbk;

namespace {

enum Act { ACT_NONE = 0, ACT_SWISH = 1, ACT_GLU = 2, ACT_LRELU = 3, ACT_GELU = 4 };

struct Epi {
  const float* bias;        // [N] (GLU: permuted like W) or null
  int act;
  float slope;              // LeakyReLU negative slope
  const float* res;         // residual [M, ldr] fp32 or null
  int ldr;
  float alpha;              // val scale before residual add
  const uint8_t* rowmask;   // [M]: nonzero -> val = 0
  void* out;
  int ldc;
  int out_bf16;
  // optional row LayerNorm of the stored rows (full-row tiles, BN == N == 256):
  // ln_out = LN(out row; ln_g, ln_b, ln_eps)
  const float* ln_g = nullptr;
  const float* ln_b = nullptr;
  float ln_eps = 0.f;
  void* ln_out = nullptr;
  int ldu = 0;
  int ln_bf16 = 0;
  // batched launches (grid.z): element strides of A, W and out per batch;
  // zdiv > 0 splits the batch index z into (z / zdiv, z % zdiv) with output
  // strides (sCo, sC) — per-(utterance, head) products written straight
  // into the (B*T, H*dh) head-interleaved layout
  long long sA = 0, sW = 0, sC = 0;
  int zdiv = 0;
  long long sCo = 0;
};

// C tile (fp32, row stride CR, in LDS) -> global through the fused epilogue:
// bias, activation (GLU pairs [value16 | gate16] column groups), row mask,
// alpha, fp32 residual; fp32 or bf16 output, 16-/8-B vector stores.
template <int ACT>
__device__ __forceinline__ float epi_act(float x, float slope) {
  if (ACT == ACT_SWISH) return x * (1.0f / (1.0f + __expf(-x)));
  if (ACT == ACT_LRELU) return x >= 0.f ? x : x * slope;
  if (ACT == ACT_GELU) return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
  return x;
}

// Fast path of store_ctile: the whole tile is in range and every pointer /
// leading dimension is 16-B (fp32) or 8-B (bf16) aligned.  Each thread owns
// one fixed output column quad (NT is a multiple of the quads per row), so
// bias is one float4 load; the row loop has a compile-time trip count and is
// fully unrolled, so every LDS read / residual load of the tile is in flight
// at once instead of one dependent round trip per iteration.
template <int BM, int BN, int NT, int ACT, bool GLU>
__device__ __forceinline__ void store_ctile_fast(const float* __restrict__ Cs, const Epi& ep, int m0, int n0,
                                                 int tid) {
  constexpr int CR = BN + 4;
  constexpr int NCOL = GLU ? BN / 2 : BN;
  constexpr int QPR = NCOL / 4;          // column quads per row
  static_assert(NT % QPR == 0, "thread map");
  constexpr int RPI = NT / QPR;          // rows per pass
  constexpr int NPASS = BM / RPI;
  static_assert(BM % RPI == 0, "rows");
  const int o = (tid % QPR) * 4, r0 = tid / QPR;
  const int oc = (GLU ? n0 / 2 : n0) + o;
  // LDS columns of this quad: GLU tiles hold [value16 | gate16] column groups
  const int ca = GLU ? 32 * (o >> 4) + (o & 15) : o;
  float4 ba = make_float4(0.f, 0.f, 0.f, 0.f), bg = ba;
  if (ep.bias) {
    ba = *reinterpret_cast<const float4*>(ep.bias + n0 + ca);
    if (GLU) bg = *reinterpret_cast<const float4*>(ep.bias + n0 + ca + 16);
  }
#pragma unroll
  for (int p = 0; p < NPASS; ++p) {
    const int r = r0 + p * RPI, row = m0 + r;
    const float4 a = *reinterpret_cast<const float4*>(Cs + r * CR + ca);
    float v[4] = {a.x + ba.x, a.y + ba.y, a.z + ba.z, a.w + ba.w};
    if (GLU) {
      const float4 gt = *reinterpret_cast<const float4*>(Cs + r * CR + ca + 16);
      const float gg[4] = {gt.x + bg.x, gt.y + bg.y, gt.z + bg.z, gt.w + bg.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] *= 1.0f / (1.0f + __expf(-gg[e]));
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = epi_act<ACT>(v[e], ep.slope);
    }
    const float sc = (ep.rowmask && ep.rowmask[row]) ? 0.f : ep.alpha;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] *= sc;
    if (ep.res) {
      const float4 rv = *reinterpret_cast<const float4*>(ep.res + (long long)row * ep.ldr + oc);
      v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
    }
    if (ep.out_bf16) {
      uint2 pk;
      pk.x = pack_bf16x2(v[0], v[1]);
      pk.y = pack_bf16x2(v[2], v[3]);
      *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(ep.out) + (long long)row * ep.ldc + oc) = pk;
    } else {
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(ep.out) + (long long)row * ep.ldc + oc) =
          make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

__device__ __forceinline__ bool epi_aligned(const Epi& ep) {
  const uintptr_t m = reinterpret_cast<uintptr_t>(ep.bias) | reinterpret_cast<uintptr_t>(ep.res) |
                      reinterpret_cast<uintptr_t>(ep.out);
  return (m & 15) == 0 && (ep.ldr & 3) == 0 && (ep.ldc & 3) == 0;
}

// Full-row epilogue (BN == N == 256, act none, fp32 out): wave w owns rows
// w*BM/4 .. +BM/4-1, lane l columns 4l .. 4l+3; after the residual stream row
// is stored, its LayerNorm (two wave reductions) is written to ln_out.  This
// removes a separate LayerNorm launch and its HBM re-read (Conformer.py:69-72
// after the attention residual).
template <int BM, int BN, int NT>
__device__ __forceinline__ void store_ctile_rowln(const float* __restrict__ Cs, const Epi& ep, int m0, int M,
                                                  int tid, const float4 (&rres)[BM / 4]) {
  static_assert(BN == 256 && NT == 256, "row-LN epilogue: 256 columns, 4 waves");
  constexpr int CR = BN + 4, RPW = BM / 4;
  const int lane = tid & 63, w = tid >> 6;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 bs = ep.bias ? *reinterpret_cast<const float4*>(ep.bias + 4 * lane) : z4;
  const float4 g4 = *reinterpret_cast<const float4*>(ep.ln_g + 4 * lane);
  const float4 b4 = *reinterpret_cast<const float4*>(ep.ln_b + 4 * lane);
  // all RPW rows at once: independent loads and reductions overlap
  float v[RPW][4], sm[RPW], sq[RPW];
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int r = w * RPW + rr, row = min(m0 + r, M - 1);
    const float4 c = *reinterpret_cast<const float4*>(Cs + r * CR + 4 * lane);
    const float sc = (ep.rowmask && ep.rowmask[row]) ? 0.f : ep.alpha;
    v[rr][0] = (c.x + bs.x) * sc; v[rr][1] = (c.y + bs.y) * sc;
    v[rr][2] = (c.z + bs.z) * sc; v[rr][3] = (c.w + bs.w) * sc;
    v[rr][0] += rres[rr].x; v[rr][1] += rres[rr].y; v[rr][2] += rres[rr].z; v[rr][3] += rres[rr].w;
    sm[rr] = v[rr][0] + v[rr][1] + v[rr][2] + v[rr][3];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) sm[rr] += __shfl_xor(sm[rr], o);
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const float mean = sm[rr] * (1.0f / BN);
    sq[rr] = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) sq[rr] += (v[rr][e] - mean) * (v[rr][e] - mean);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) sq[rr] += __shfl_xor(sq[rr], o);
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int r = w * RPW + rr, row = m0 + r;
    if (row >= M) continue;
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(ep.out) + (long long)row * ep.ldc + 4 * lane) =
        make_float4(v[rr][0], v[rr][1], v[rr][2], v[rr][3]);
    const float mean = sm[rr] * (1.0f / BN);
    const float rstd = 1.0f / sqrtf(sq[rr] * (1.0f / BN) + ep.ln_eps);
    const float y0 = (v[rr][0] - mean) * rstd * g4.x + b4.x, y1 = (v[rr][1] - mean) * rstd * g4.y + b4.y;
    const float y2 = (v[rr][2] - mean) * rstd * g4.z + b4.z, y3 = (v[rr][3] - mean) * rstd * g4.w + b4.w;
    if (ep.ln_bf16) {
      uint2 pk;
      pk.x = pack_bf16x2(y0, y1);
      pk.y = pack_bf16x2(y2, y3);
      *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(ep.ln_out) + (long long)row * ep.ldu + 4 * lane) = pk;
    } else {
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(ep.ln_out) + (long long)row * ep.ldu + 4 * lane) =
          make_float4(y0, y1, y2, y3);
    }
  }
}

template <int BM, int BN, int NT>
__device__ __forceinline__ void store_ctile(const float* __restrict__ Cs, const Epi& ep, int m0, int n0, int M,
                                            int N, int tid) {

  if (m0 + BM <= M && n0 + BN <= N && epi_aligned(ep)) {
    switch (ep.act) {
      case ACT_NONE: store_ctile_fast<BM, BN, NT, ACT_NONE, false>(Cs, ep, m0, n0, tid); return;
      case ACT_SWISH: store_ctile_fast<BM, BN, NT, ACT_SWISH, false>(Cs, ep, m0, n0, tid); return;
      case ACT_GLU: store_ctile_fast<BM, BN, NT, ACT_NONE, true>(Cs, ep, m0, n0, tid); return;
      case ACT_LRELU: store_ctile_fast<BM, BN, NT, ACT_LRELU, false>(Cs, ep, m0, n0, tid); return;
      case ACT_GELU: store_ctile_fast<BM, BN, NT, ACT_GELU, false>(Cs, ep, m0, n0, tid); return;
    }
  }
  constexpr int CR = BN + 4;
  const bool glu = ep.act == ACT_GLU;
  const int ncols = glu ? BN / 2 : BN;       // output columns of this tile
  const int oc0 = glu ? n0 / 2 : n0;         // first output column
  const int nout = glu ? N / 2 : N;
  for (int c = tid; c < BM * (ncols / 4); c += NT) {
    const int r = c / (ncols / 4), o = (c % (ncols / 4)) * 4;
    const int row = m0 + r;
    if (row >= M || oc0 + o >= nout) continue;
    float v[4];
    if (glu) {
      const int q = o >> 4, wi = o & 15;
      const int ca = 32 * q + wi, cg = ca + 16;  // [value16 | gate16] column groups
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float va = Cs[r * CR + ca + e], vg = Cs[r * CR + cg + e];
        if (ep.bias) {
          va += ep.bias[n0 + ca + e];
          vg += ep.bias[n0 + cg + e];
        }
        v[e] = va * (1.0f / (1.0f + __expf(-vg)));
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = Cs[r * CR + o + e];
        if (ep.bias) x += ep.bias[n0 + o + e];
        if (ep.act == ACT_SWISH)
          x = x * (1.0f / (1.0f + __expf(-x)));
        else if (ep.act == ACT_LRELU)
          x = x >= 0.f ? x : x * ep.slope;
        else if (ep.act == ACT_GELU)
          x = 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
        v[e] = x;
      }
    }
    const bool masked = ep.rowmask && ep.rowmask[row];
    const long long oc = oc0 + o;
    const bool full = oc + 3 < nout;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (masked ? 0.f : v[e]) * ep.alpha;
    if (ep.res) {
      const float* rp = ep.res + (long long)row * ep.ldr + oc;
      if (full && ((reinterpret_cast<uintptr_t>(rp) & 15) == 0)) {
        const float4 rv = *reinterpret_cast<const float4*>(rp);
        v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (oc + e < nout) v[e] += rp[e];
      }
    }
    if (ep.out_bf16) {
      bf16_t* op = reinterpret_cast<bf16_t*>(ep.out) + (long long)row * ep.ldc + oc;
      if (full && ((reinterpret_cast<uintptr_t>(op) & 7) == 0)) {
        uint2 pk;
        pk.x = pack_bf16x2(v[0], v[1]);
        pk.y = pack_bf16x2(v[2], v[3]);
        *reinterpret_cast<uint2*>(op) = pk;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (oc + e < nout) op[e] = f32_to_bf16(v[e]);
      }
    } else {
      float* op = reinterpret_cast<float*>(ep.out) + (long long)row * ep.ldc + oc;
      if (full && ((reinterpret_cast<uintptr_t>(op) & 15) == 0)) {
        *reinterpret_cast<float4*>(op) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (oc + e < nout) op[e] = v[e];
      }
    }
  }
}

template <typename T, int BM, int BN, int BK, int NBUF>
__global__ void __launch_bounds__(256) gemm_kernel(const T* __restrict__ A, int lda, const T* __restrict__ W,
                                                   int ldw, int M, int N, int K, Epi ep) {
  using Tr = MT<T>;
  constexpr int VEC = Tr::VEC;
  // LDS row stride (elements): +32 B for bf16 makes the 16-lane ds_read_b128
  // groups of the fragment reads bank-conflict-free (+16 B left 2-way conflicts)
  constexpr int LDSR = BK + (sizeof(T) == 2 ? 2 : 1) * Tr::PAD;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int CPR = BK / VEC;          // 16-B chunks per row
  constexpr int ACH = (BM * CPR + 255) / 256;  // chunks per thread (A; the last pass may be partial)
  constexpr int BCH = (BN * CPR + 255) / 256;  // chunks per thread (B)

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* As = reinterpret_cast<T*>(smem);
  T* Bs = As + NBUF * BM * LDSR;
  if (gridDim.z > 1) {  // batched: this batch's operands and output
    const long long z = blockIdx.z;
    A += z * ep.sA;
    W += z * ep.sW;
    const long long oc = ep.zdiv > 0 ? (z / ep.zdiv) * ep.sCo + (z % ep.zdiv) * ep.sC : z * ep.sC;
    ep.out = reinterpret_cast<char*>(ep.out) + oc * (ep.out_bf16 ? 2 : 4);
  }

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntn = (N + BN - 1) / BN;
  // XCD-aware remap (bijective): workgroups dealt round-robin to the 8 XCDs get
  // consecutive tiles per XCD, so the N-tiles of one A row-panel share an L2.
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile_id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int m0 = (tile_id / ntn) * BM;
  const int n0 = (tile_id % ntn) * BN;
  // full-row (BN == 256) tiles are sbk_gemm_ln's: the residual rows of the
  // row-LN epilogue are fetched here so their latency hides under the K loop
  constexpr bool ROWLN = BN == 256;
  float4 rres[ROWLN ? BM / 4 : 1];
  if constexpr (ROWLN) {
#pragma unroll
    for (int rr = 0; rr < BM / 4; ++rr) {
      const int row = min(m0 + (tid >> 6) * (BM / 4) + rr, M - 1);
      rres[rr] = ep.res ? *reinterpret_cast<const float4*>(ep.res + (long long)row * ep.ldr + 4 * (tid & 63))
                        : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }

  uint4 ra[ACH], rb[BCH];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * 256, r = c / CPR, kc = (c % CPR) * VEC;
      const int gr = m0 + r, gk = k0 + kc;
      ra[i] = (c < BM * CPR && gr < M && gk < K) ? *reinterpret_cast<const uint4*>(A + (long long)gr * lda + gk)
                                                 : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * 256, r = c / CPR, kc = (c % CPR) * VEC;
      const int gr = n0 + r, gk = k0 + kc;
      rb[i] = (c < BN * CPR && gr < N && gk < K) ? *reinterpret_cast<const uint4*>(W + (long long)gr * ldw + gk)
                                                 : make_uint4(0, 0, 0, 0);
    }
  };
  auto sstore = [&](int buf) {
    T* as = As + buf * BM * LDSR;
    T* bs = Bs + buf * BN * LDSR;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * 256, r = c / CPR, kc = (c % CPR) * VEC;
      if (c < BM * CPR) *reinterpret_cast<uint4*>(as + r * LDSR + kc) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * 256, r = c / CPR, kc = (c % CPR) * VEC;
      if (c < BN * CPR) *reinterpret_cast<uint4*>(bs + r * LDSR + kc) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + BK - 1) / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  int cur = 0;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gload((kt + 1) * BK);
    const T* as = As + cur * BM * LDSR + (wm * WM + fr) * LDSR + fk;
    const T* bs = Bs + cur * BN * LDSR + (wn * WN + fr) * LDSR + fk;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      typename Tr::frag fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = Tr::load(as + i * 16 * LDSR + ks * 32);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = Tr::load(bs + j * 16 * LDSR + ks * 32);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) Tr::mma(acc[i][j], fa[i], fb[j]);
    }
    if (NBUF == 2) {
      if (kt + 1 < nk) sstore(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    } else if (kt + 1 < nk) {
      __syncthreads();  // all waves done reading the single buffer
      sstore(0);
      __syncthreads();
    }
  }
  if (NBUF == 1) __syncthreads();

  // ---- epilogue: accumulators -> LDS C tile -> coalesced vector pass ----
  // (the staging ring is free: the last loop iteration ended with a barrier)
  constexpr int CR = BN + 4;  // C tile row stride (floats)
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * WM + i * 16 + 4 * (lane >> 4) + r) * CR + wn * WN + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  if constexpr (ROWLN)
    store_ctile_rowln<BM, BN, 256>(Cs, ep, m0, M, tid, rres);
  else
    store_ctile<BM, BN, 256>(Cs, ep, m0, n0, M, N, tid);
}

template <typename T, int BM, int BN, int BK, int NBUF = 2>
int launch(const void* A, int lda, const void* W, int ldw, int M, int N, int K, const Epi& ep, hipStream_t s,
           int batch = 1) {
  constexpr int LDSR = BK + (sizeof(T) == 2 ? 2 : 1) * MT<T>::PAD;
  size_t lds = (size_t)NBUF * (BM + BN) * LDSR * sizeof(T);
  const size_t cbytes = (size_t)BM * (BN + 4) * 4;  // epilogue C tile
  if (cbytes > lds) lds = cbytes;
  if (lds > 64 * 1024)
    if (hipError_t e = sbk::lds_optin(reinterpret_cast<const void*>(&gemm_kernel<T, BM, BN, BK, NBUF>), lds))
      return (int)e;
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_kernel<T, BM, BN, BK, NBUF>), dim3(grid, 1, batch), dim3(256), lds, s,
                     reinterpret_cast<const T*>(A), lda, reinterpret_cast<const T*>(W), ldw, M, N, K, ep);
  SBK_CHECK_LAUNCH();
  return 0;
}


// LDS-DMA ring GEMM (bf16, K % 64 == 0, K >= 192): 4 waves (2x2), tile BM x BN,
// 64-deep K steps staged global -> LDS by global_load_lds_dwordx4 (full
// 128-B lines, no VGPRs) into a 4-slot ring with 3 steps in flight across one
// raw barrier per step (counted vmcnt; the tail re-loads the last step into a
// dead slot so every step waits on the same count).  The LDS image is
// lane-linear, 16-B chunks XOR-swizzled by (row >> 1) & 7 on the source
// address and on the fragment reads (conflict-free ds_read_b128).  Out-of-
// range rows clamp their source to the last row (results never stored).
template <int BM, int BN>
__global__ void __launch_bounds__(256) gemm_ring_kernel(const bf16_t* __restrict__ A, int lda,
                                                        const bf16_t* __restrict__ W, int ldw, int M, int N, int K,
                                                        Epi ep) {
  constexpr int BK = 64, NB = 4, NT = 256;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int SLOT = (BM + BN) * BK;          // elements per ring slot
  constexpr int GA = BM * BK * 2 / 1024 / 4;    // LDS-DMA pieces per wave per step (A)
  constexpr int GB = BN * BK * 2 / 1024 / 4;    // (B)
  constexpr int GPS = GA + GB;
  static_assert(GA >= 1 && GB >= 1 && GA * 4 * 1024 == BM * BK * 2 && GB * 4 * 1024 == BN * BK * 2, "tile");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int fr = lane & 15, g = lane >> 4;
  const int ntn = (N + BN - 1) / BN;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile_id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int m0 = (tile_id / ntn) * BM;
  const int n0 = (tile_id % ntn) * BN;
  const int nk = K / BK;

  // piece p of a tile covers rows 8p .. 8p+7; lane -> row 8p + lane/8, chunk lane%8
  const int lrow = lane >> 3, lchk = lane & 7;
  auto issue = [&](int kt) __attribute__((always_inline)) {
    bf16_t* dst = ring + (kt % NB) * SLOT;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int p = i * 4 + w, r = p * 8 + lrow;
      const int gr = min(m0 + r, M - 1);
      const bf16_t* src = A + (long long)gr * lda + k0 + ((lchk ^ ((r >> 1) & 7)) << 3);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(dst + p * 8 * BK), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const int p = i * 4 + w, r = p * 8 + lrow;
      const int gr = min(n0 + r, N - 1);
      const bf16_t* src = W + (long long)gr * ldw + k0 + ((lchk ^ ((r >> 1) & 7)) << 3);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(dst + BM * BK + p * 8 * BK), 16, 0, 0);
    }
  };
  issue(0);
  issue(1);
  issue(2);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int kt = 0; kt < nk; ++kt) {
    // this wave's pieces of step kt landed (steps kt+1, kt+2 stay in flight);
    // the barrier publishes every wave's pieces and retires step kt-1's reads
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GPS) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue(min(kt + 3, nk - 1));  // into slot (kt+3)%NB = (kt-1)%NB
    const bf16_t* As = ring + (kt % NB) * SLOT;
    const bf16_t* Bs = As + BM * BK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WM + i * 16 + fr;
        fa[i] = *reinterpret_cast<const bf16x8*>(As + r * BK + (((ks * 4 + g) ^ ((r >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WN + j * 16 + fr;
        fb[j] = *reinterpret_cast<const bf16x8*>(Bs + r * BK + (((ks * 4 + g) ^ ((r >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tail re-loads
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  constexpr int CR = BN + 4;
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * WM + i * 16 + 4 * g + r) * CR + wn * WN + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  store_ctile<BM, BN, NT>(Cs, ep, m0, n0, M, N, tid);
}

template <int BM, int BN>
int launch_ring(const void* A, int lda, const void* W, int ldw, int M, int N, int K, const Epi& ep, hipStream_t s) {
  size_t lds = (size_t)4 * (BM + BN) * 64 * sizeof(bf16_t);
  const size_t cbytes = (size_t)BM * (BN + 4) * 4;
  if (cbytes > lds) lds = cbytes;
  if (hipError_t e = sbk::lds_optin(reinterpret_cast<const void*>(&gemm_ring_kernel<BM, BN>), lds)) return (int)e;
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_ring_kernel<BM, BN>), dim3(grid), dim3(256), lds, s, reinterpret_cast<const bf16_t*>(A),
                     lda, reinterpret_cast<const bf16_t*>(W), ldw, M, N, K, ep);
  SBK_CHECK_LAUNCH();
  return 0;
}


typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int V>
struct IntC {
  static constexpr int value = V;
};

// Deep-prefetch GEMM (bf16): the register-staged double-buffered LDS tile of
// gemm_kernel, but with NPRE = 4 register stages in flight, so a K step's
// global loads were issued 3 steps before they are stored to LDS.  At the
// encoder's K = 256 all of K is requested up front; the shallow pipeline of
// gemm_kernel (load k+1 while computing k) left every step waiting one full
// L2/HBM latency.  Loads are unconditional (rows and K clamp; a ragged K tail
// is zeroed after the load) so the compiler's vmcnt waits stay counted.
template <int BM, int BN, int BK>
__global__ void __launch_bounds__(256) gemm_pf_kernel(const bf16_t* __restrict__ A, int lda,
                                                      const bf16_t* __restrict__ W, int ldw, int M, int N, int K,
                                                      Epi ep) {
  constexpr int NT = 256, LDSR = BK + 16;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int CPR = BK / 8, ACH = BM * CPR / NT, BCH = BN * CPR / NT, CH = ACH + BCH;
  static_assert(ACH >= 1 && BCH >= 1 && ACH * NT == BM * CPR && BCH * NT == BN * CPR, "tile");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Bs = As + 2 * BM * LDSR;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntn = (N + BN - 1) / BN;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile_id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int m0 = (tile_id / ntn) * BM;
  const int n0 = (tile_id % ntn) * BN;
  const int nk = (K + BK - 1) / BK;

  auto gload = [&](int kt, u32x4 (&rs)[CH]) __attribute__((always_inline)) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const bool isA = i < ACH;
      const int c = tid + (isA ? i : i - ACH) * NT, r = c / CPR, kc = (c % CPR) * 8;
      const int gk = k0 + kc;
      const bf16_t* src = isA ? A + (long long)min(m0 + r, M - 1) * lda : W + (long long)min(n0 + r, N - 1) * ldw;
      u32x4 v = *reinterpret_cast<const u32x4*>(src + min(gk, K - 8));
      rs[i] = gk < K ? v : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto sstore = [&](int buf, const u32x4 (&rs)[CH]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const bool isA = i < ACH;
      const int c = tid + (isA ? i : i - ACH) * NT, r = c / CPR, kc = (c % CPR) * 8;
      bf16_t* dst = isA ? As + buf * BM * LDSR : Bs + buf * BN * LDSR;
      *reinterpret_cast<u32x4*>(dst + r * LDSR + kc) = rs[i];
    }
  };
  u32x4 s0[CH], s1[CH], s2[CH], s3[CH];
  auto sset = [&](auto U) -> u32x4(&)[CH] {
    constexpr int u = decltype(U)::value & 3;
    if constexpr (u == 0) return s0;
    else if constexpr (u == 1) return s1;
    else if constexpr (u == 2) return s2;
    else return s3;
  };
  gload(0, s0);
  gload(min(1, nk - 1), s1);
  gload(min(2, nk - 1), s2);
  gload(min(3, nk - 1), s3);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  sstore(0, s0);
  __syncthreads();
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  auto step = [&](int kt, auto U) __attribute__((always_inline)) {
    constexpr int u = decltype(U)::value;
    const bf16_t* as = As + (kt & 1) * BM * LDSR + (wm * WM + fr) * LDSR + fk;
    const bf16_t* bs = Bs + (kt & 1) * BN * LDSR + (wn * WN + fr) * LDSR + fk;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(as + i * 16 * LDSR + ks * 32);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(bs + j * 16 * LDSR + ks * 32);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    sstore((kt + 1) & 1, sset(IntC<u + 1>{}));   // tile kt+1 (requested 3 steps ago; a dummy past the end)
    gload(min(kt + 4, nk - 1), sset(U));          // this set's tile kt is in LDS already
    __syncthreads();
  };
  for (int kt0 = 0; kt0 < nk; kt0 += 4) {
    step(kt0, IntC<0>{});
    if (kt0 + 1 < nk) step(kt0 + 1, IntC<1>{});
    if (kt0 + 2 < nk) step(kt0 + 2, IntC<2>{});
    if (kt0 + 3 < nk) step(kt0 + 3, IntC<3>{});
  }

  constexpr int CR = BN + 4;
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * WM + i * 16 + 4 * (lane >> 4) + r) * CR + wn * WN + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  store_ctile<BM, BN, NT>(Cs, ep, m0, n0, M, N, tid);
}

template <int BM, int BN, int BK>
int launch_pf(const void* A, int lda, const void* W, int ldw, int M, int N, int K, const Epi& ep, hipStream_t s) {
  size_t lds = (size_t)2 * (BM + BN) * (BK + 16) * sizeof(bf16_t);
  const size_t cbytes = (size_t)BM * (BN + 4) * 4;
  if (cbytes > lds) lds = cbytes;
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_pf_kernel<BM, BN, BK>), dim3(grid), dim3(256), lds, s, reinterpret_cast<const bf16_t*>(A),
                     lda, reinterpret_cast<const bf16_t*>(W), ldw, M, N, K, ep);
  SBK_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// The GLU column permutation depends on the wave tile width WN = BN/2; the
// host asks for it here so weights are permuted consistently.
SBK_API int sbk_gemm_glu_group(int dtype_bf16) { (void)dtype_bf16; return 16; }  // [value16 | gate16] groups

// dtype_bf16: A and W are bf16 (else fp32).  tile: 0 auto, 1 = 128x128, 2 = 64x64, 3 = 128x64 (BK 64,
// double-buffered); bf16 only: 4/5/6 = 64x64 / 64x128 / 128x64 with BK 256 single buffer,
// out = res + alpha * (A @ W^T + bias) (rows masked -> 0 before the residual),
// then u = LN(out row) — the attention output projection and the convolution
// module's LayerNorm (Conformer.py:69-72, attention.py:636) in one launch.
// Full-row tiles: N == 256, fp32 out, no activation.
SBK_API int sbk_gemm_ln(int dtype_bf16, const void* A, int lda, const void* W, int ldw, int M, int N, int K,
                        const float* bias, const float* res, int ldr, float alpha, const uint8_t* rowmask, float* out,
                        int ldc, const float* ln_g, const float* ln_b, float ln_eps, void* u, int ldu, int u_bf16,
                        int tile, void* stream) {
  if (M <= 0 || N != 256 || K <= 0 || !ln_g || !ln_b || !u || !out) return SBK_ERR_ARG;
  const int vec = dtype_bf16 ? 8 : 4;
  if ((K % vec) || (lda % vec) || (ldw % vec) || (ldc % 4) || (ldu % 4) || (res && (ldr % 4))) return SBK_ERR_ARG;
  const uintptr_t al = reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(W) |
                       reinterpret_cast<uintptr_t>(bias) | reinterpret_cast<uintptr_t>(res) |
                       reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(ln_g) |
                       reinterpret_cast<uintptr_t>(ln_b) | reinterpret_cast<uintptr_t>(u);
  if (al & 15) return SBK_ERR_ARG;
  Epi ep{bias, ACT_NONE, 0.f, res, ldr, alpha, rowmask, out, ldc, 0};
  ep.ln_g = ln_g;
  ep.ln_b = ln_b;
  ep.ln_eps = ln_eps;
  ep.ln_out = u;
  ep.ldu = ldu;
  ep.ln_bf16 = u_bf16;
  hipStream_t s = (hipStream_t)stream;
  if (dtype_bf16) {
    if (tile == 2) return launch<bf16_t, 64, 256, 32, 2>(A, lda, W, ldw, M, N, K, ep, s);
    if (tile == 1) return launch<bf16_t, 32, 256, 64, 2>(A, lda, W, ldw, M, N, K, ep, s);
    return launch<bf16_t, 32, 256, 32, 2>(A, lda, W, ldw, M, N, K, ep, s);
  }
  return launch<float, 32, 256, 32, 2>(A, lda, W, ldw, M, N, K, ep, s);
}

// 7 = 128x128 BK 128 single buffer, 8 = 64x64 BK 128 double buffer.
SBK_API int sbk_gemm(int dtype_bf16, const void* A, int lda, const void* W, int ldw, int M, int N, int K,
                     const float* bias, int act, float slope, const float* res, int ldr, float alpha,
                     const uint8_t* rowmask, void* out, int ldc, int out_bf16, int tile, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return SBK_ERR_ARG;
  const int vec = dtype_bf16 ? 8 : 4;
  if ((K % vec) || (lda % vec) || (ldw % vec)) return SBK_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(W)) & 15) return SBK_ERR_ARG;
  if (act == ACT_GLU && (N % 32)) return SBK_ERR_ARG;  // whole [a16|gate16] groups
  Epi ep{bias, act, slope, res, ldr, alpha, rowmask, out, ldc, out_bf16};
  hipStream_t s = (hipStream_t)stream;
  // tile 30: the 256 x 256 multi-phase kernel (gemm256.hip), N % 256 == 0,
  // K % 64 == 0; taken by default when it fills the chip (>= 180 tiles) at
  // K >= 256 — config 5's projections: 0.97-1.03 PF/s against 0.67-0.82 for
  // the best of the other tiles (profiles/r05c_g256_shapes.log)
  if (dtype_bf16 && (tile == 30 || tile == 0)) {
    const Gemm256Epi e{bias, act, slope, res, ldr, alpha, rowmask, out, ldc, out_bf16};
    const bool ok = gemm256_supported(M, N, K, lda, ldw, A, W, e);
    if (tile == 30 && !ok) return SBK_ERR_ARG;
    if (ok && (tile == 30 || (K >= 256 && (long long)((M + 255) / 256) * (N / 256) >= 180)))
      return gemm256_launch(A, lda, W, ldw, M, N, K, e, s);
  }
  // tile 2 (64x64x64) measured best for every encoder shape (M = B*T = 12032,
  // scripts/kbench.py gemm); the joint-output projection of the transducer
  // (M = B*T*U1 = 782080, N = 1000, K = 1024) runs 1.5x faster on 128x128x128
  // (scripts/logits_gemm_probe.py: 3.69 -> 2.46 ms, 652 TF/s).
  if (tile == 0) tile = (dtype_bf16 && (long long)M * N >= (32LL << 20) && K >= 512 && N >= 256) ? 7 : 2;
  if (dtype_bf16) {
    switch (tile) {
      case 1: return launch<bf16_t, 128, 128, 64>(A, lda, W, ldw, M, N, K, ep, s);
      case 3: return launch<bf16_t, 128, 64, 64>(A, lda, W, ldw, M, N, K, ep, s);
      case 4: return launch<bf16_t, 64, 64, 256, 1>(A, lda, W, ldw, M, N, K, ep, s);
      case 5: return launch<bf16_t, 64, 128, 256, 1>(A, lda, W, ldw, M, N, K, ep, s);
      case 6: return launch<bf16_t, 128, 64, 256, 1>(A, lda, W, ldw, M, N, K, ep, s);
      case 7: return launch<bf16_t, 128, 128, 128, 1>(A, lda, W, ldw, M, N, K, ep, s);
      case 8: return launch<bf16_t, 64, 64, 128, 2>(A, lda, W, ldw, M, N, K, ep, s);
      case 9: return launch<bf16_t, 64, 64, 32, 2>(A, lda, W, ldw, M, N, K, ep, s);
      case 10: return launch<bf16_t, 128, 64, 32, 2>(A, lda, W, ldw, M, N, K, ep, s);
      case 18: return launch_pf<64, 64, 64>(A, lda, W, ldw, M, N, K, ep, s);
      case 19: return launch_pf<128, 64, 64>(A, lda, W, ldw, M, N, K, ep, s);
      case 20: return launch_pf<64, 128, 64>(A, lda, W, ldw, M, N, K, ep, s);
      case 21: return launch_pf<128, 128, 64>(A, lda, W, ldw, M, N, K, ep, s);
      case 22: return launch_pf<64, 64, 32>(A, lda, W, ldw, M, N, K, ep, s);
      case 17: return launch<bf16_t, 64, 128, 32, 2>(A, lda, W, ldw, M, N, K, ep, s);
      case 11: case 12: case 13: {
        // LDS-DMA ring: K % 64 == 0, K >= 192, 16-B aligned rows
        if ((K % 64) || K < 192 || (lda % 8) || (ldw % 8)) return SBK_ERR_ARG;
        if (tile == 11) return launch_ring<128, 128>(A, lda, W, ldw, M, N, K, ep, s);
        if (tile == 12) return launch_ring<128, 64>(A, lda, W, ldw, M, N, K, ep, s);
        return launch_ring<64, 64>(A, lda, W, ldw, M, N, K, ep, s);
      }
      default: return launch<bf16_t, 64, 64, 64>(A, lda, W, ldw, M, N, K, ep, s);
    }
  }
  switch (tile) {
    case 1: return launch<float, 128, 128, 32>(A, lda, W, ldw, M, N, K, ep, s);
    case 3: return launch<float, 128, 64, 32>(A, lda, W, ldw, M, N, K, ep, s);
    default: return launch<float, 64, 64, 32>(A, lda, W, ldw, M, N, K, ep, s);
  }
}

// Batched C[z] = A[z] · W[z]^T (bf16 or fp32 operands, K-contiguous rows;
// fp32 or bf16 out) for z < batch with element strides sA / sW: the
// per-(b, h) products of the attention backward (dP = dO·V^T, dQ = dS·K, ...)
// and the dropout product drop(P)·V, one launch over grid.z.  Output: batch
// z at (z / zdiv) * sCo + (z % zdiv) * sC when zdiv > 0, else z * sC.
// M, N, K as sbk_gemm (K, lda, ldw multiples of the 16-B vector).
SBK_API int sbk_gemm_batched(int dtype_bf16, const void* A, int lda, long long sA, const void* W, int ldw,
                             long long sW, int M, int N, int K, int batch, void* out, int ldc, long long sC, int zdiv,
                             long long sCo, int out_bf16, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535 || zdiv < 0) return SBK_ERR_ARG;
  const int vec = dtype_bf16 ? 8 : 4;
  if ((K % vec) || (lda % vec) || (ldw % vec) || (sA % vec) || (sW % vec)) return SBK_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(W)) & 15) return SBK_ERR_ARG;
  Epi ep{nullptr, ACT_NONE, 0.f, nullptr, 0, 1.f, nullptr, out, ldc, out_bf16};
  ep.sA = sA;
  ep.sW = sW;
  ep.sC = sC;
  ep.zdiv = zdiv;
  ep.sCo = sCo;
  if (dtype_bf16) return launch<bf16_t, 64, 64, 64>(A, lda, W, ldw, M, N, K, ep, (hipStream_t)stream, batch);
  return launch<float, 64, 64, 32>(A, lda, W, ldw, M, N, K, ep, (hipStream_t)stream, batch);
}
