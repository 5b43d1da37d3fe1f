// Fused Transformer-XL relative-position self-attention (RelPosMHAXL).
//
// Reference: speechbrain/nnet/attention.py:485-639 (RelPosMHAXL.forward),
// rel_shift :468-483.  For query i, key j (T queries = T keys):
//   score[i,j] = ( (q_i + u)·k_j  +  (q_i + v)·p_{T-1-i+j} ) / sqrt(d_model)
//   key-padding -> -inf, softmax over j, out_i = Σ_j P[i,j] v_j
// with p = linear_pos(RelPosEncXL) and rel_shift in closed form
// (out[i,j] = bd[i, T-1-i+j]); the (B,H,T,2T-1) bd tensor the reference
// materialises (145 MB at B=32, T=376) never exists.
//
// Flash-style, transposed formulation (MI355X wave64 + 16x16 MFMA):
//  * workgroup = (b, h, 64 queries), 4 waves x 16 queries; 64-key chunks of
//    K, V^T and the 127 positional rows the chunk needs are staged in LDS
//    with 16-B loads, shared by the 4 waves.
//  * each wave computes S^T = K·Qu^T (4 tiles) — the query sits on the lane,
//    so softmax statistics are per-lane (+2 xor-shuffles) — and
//    G^T = P_band·Qv^T (5 tiles); the rel_shift gather S^T[jj][ii] +=
//    G^T[15-ii+jj][ii] stays inside the lane's column via a 5 KB per-wave
//    LDS scratch.
//  * O^T = V^T·P^T accumulates with P taken straight from the S registers
//    (permuted-k fragments: keys {4g..4g+3, 16+4g..16+4g+3} per 32-key step,
//    V^T read in the same order) — no LDS round trip for P.
//  * online softmax (running max / sum, rescale) when no probabilities are
//    requested; with probabilities (the reference's returned attention map)
//    a stats pass then an exact pass that writes P and accumulates P·V.
// bf16 operands use v_mfma_f32_16x16x32_bf16, fp32 operands exact f32 MFMA
// (mfma.h); softmax and accumulators are fp32.
#include "mfma.h"

using namespace sbk;

namespace {


constexpr int QB = 64;        // queries per workgroup
constexpr int KC = 64;        // keys per chunk
constexpr int PBR = KC + QB;  // positional band rows staged per chunk (127 used)
constexpr int GR = 80;        // G^T rows per wave (79 used)
constexpr int GS = 20;        // G^T scratch row stride (floats): conflict-free writes and shifted reads

template <typename T>
struct VLayout {  // bf16: V row-major + ds_read_tr16 ; fp32: V^T staged transposed
  static constexpr bool TR = sizeof(T) == 2;
};

template <typename T, int DHP>
struct FlashLds {
  // bf16: +32 B row pad makes the 16-lane ds_read_b128 groups of the K / P
  // fragment reads and the ds_read_b64_tr_b16 V reads conflict-free (+16 B
  // left 2-way conflicts); fp32: +16 B
  static constexpr int PAD = sizeof(T) == 2 ? 2 * MT<T>::PAD : MT<T>::PAD;
  static constexpr int KR = DHP + PAD;  // Ks / Ps / V(row-major) row stride
  static constexpr int VR = KC + PAD;   // Vt row stride (fp32 path)
  static constexpr size_t ks = (size_t)KC * KR * sizeof(T);
  static constexpr size_t vt = VLayout<T>::TR ? (size_t)KC * KR * sizeof(T) : (size_t)DHP * VR * sizeof(T);
  static constexpr size_t ps = (size_t)PBR * KR * sizeof(T);
  static constexpr size_t gs = (size_t)4 * GR * GS * 4;
  static constexpr size_t ms = (size_t)(KC + 4) * 4;  // key mask + 'chunk has a masked key' flag
  // The per-wave G^T scratch aliases the K and positional-band tiles, which
  // are dead once every wave's S / G MFMAs have consumed them (one barrier):
  // 66 -> 40 KB per workgroup, three workgroups per CU instead of two, and
  // the 768 workgroups of a B = 32, T = 376 launch fit in one round.
  static_assert(gs <= ks + ps, "G^T scratch fits over Ks + Ps");
  static constexpr size_t bytes = ks + ps + vt + ms;
};

typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

// Out-of-range K / V / positional rows are zeroed at commit.  (Tried:
// committing the clamped loads unmasked — the rows only meet masked scores —
// measured 36 -> 54 us: the compiler then sank the prefetch loads to their
// stores; and head dims >= dh must stay zero when dh is not a multiple of the
// 8-dim Q fragment, whose vector loads then read the next section.)
#define STAGE_SEL(ok, v) sel4((ok), (v))

// component-wise select (a struct-valued ?: takes the operands' addresses and
// sends the staging arrays to scratch)
__device__ __forceinline__ uint4 sel4(bool c, const uint4& a) {
  return make_uint4(c ? a.x : 0u, c ? a.y : 0u, c ? a.z : 0u, c ? a.w : 0u);
}

// A-operand fragment of V^T (rows d = dbase + (lane&15)) for keys
// {k0 + 4g .. k0 + 4g + 3} ∪ {k0 + 16 + 4g .. +3}, read from row-major V in
// LDS with two transposing reads (ds_read_b64_tr_b16): lane 4q+p of each
// 16-lane group addresses row (key) q, columns (d) 4p..4p+3 of the block.
__device__ __forceinline__ bf16x8 vt_frag_tr(const bf16_t* V, int KR, int k0, int dbase, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const bf16_t* a0 = V + (k0 + 4 * g + q) * KR + dbase + 4 * p;
  const bf16_t* a1 = a0 + 16 * KR;
  const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4_t*)(a0));
  const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4_t*)(a1));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// s_memtime marks of the waves of one workgroup, and per workgroup its
// memrealtime / memtime at start and end (probe builds only)
SBK_PROBE_BUFFER(g_att_tl, 4, 64)
SBK_PROBE_BUFFER(g_att_wg, 4096, 4)
#define ATT_TL(i) SBK_PROBE(if (tl_on && lane == 0 && (i) < 64) g_att_tl[w][i] = __builtin_amdgcn_s_memtime();)

template <typename T, int DHP, bool PROBS>
__global__ void __launch_bounds__(256, 2) relpos_flash_kernel(const T* __restrict__ qkv, const T* __restrict__ pk,
                                                           const float* __restrict__ pbu,
                                                           const float* __restrict__ pbv,
                                                           const uint8_t* __restrict__ kpm, int B, int Tn, int H,
                                                           int dh, float scale, T* __restrict__ out,
                                                           float* __restrict__ probs, int vec_ok, int ldp,
                                                           const float* __restrict__ am, long long am_sb,
                                                           long long am_sh) {
  using Tr = MT<T>;
  using L = FlashLds<T, DHP>;
  constexpr int KR = L::KR, VR = L::VR, VEC = Tr::VEC;
  constexpr bool TRV = VLayout<T>::TR;
  constexpr int KS = DHP / 32;   // k-steps over the head dim
  constexpr int NDT = DHP / 16;  // O^T tiles (head-dim rows)
  constexpr int CPR = DHP / VEC; // 16-B chunks per staged row
  constexpr int NKC = KC * CPR / 256;   // K (and V) chunks per thread
  constexpr int NPC = PBR * CPR / 256;  // P-band chunks per thread
  static_assert(KC == 64, "mask staging: one wave per chunk");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* Ks = reinterpret_cast<T*>(smem);
  T* Ps = reinterpret_cast<T*>(smem + L::ks);
  T* Vs = reinterpret_cast<T*>(smem + L::ks + L::ps);
  float* Gs = reinterpret_cast<float*>(smem);  // over Ks + Ps (dead after the S / G MFMAs)
  float* Ms = reinterpret_cast<float*>(smem + L::ks + L::ps + L::vt);
  constexpr bool ALIAS = true;

  const int d_model = H * dh;
  const long long row3 = 3LL * d_model;
  const int nqb = (Tn + QB - 1) / QB;
  // XCD-aware bijective remap: workgroups are dealt round-robin to the 8 XCDs;
  // give each XCD a contiguous run of tiles so the query blocks of one (b, h)
  // share an L2 and its K/V/positional rows are fetched from HBM once.
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int qb = tile % nqb;
  const int bh = tile / nqb;
  const int h = bh % H, b = bh / H;
  const int i0 = qb * QB;
  SBK_PROBE(const bool tl_on = tile == 200 && sizeof(T) == 2 && !PROBS;)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c16 = lane & 15, g = lane >> 4;
  const int i0w = i0 + 16 * w;
  const int my_i = i0w + c16;  // this lane's query
  const T* qkv_b = qkv + (long long)b * Tn * row3 + h * 3 * dh;
  const T* pk_h = pk + h * dh;
  float* Gw = Gs + w * GR * GS;

  // ---- Qu / Qv as B-operand fragments (query on the lane), pre-scaled by
  // scale * log2(e) so scores come out of the MFMAs in the exp2 domain ----
  const float qscale = scale * 1.4426950408889634f;
  typename Tr::frag fqu[KS], fqv[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    float qu[8], qv[8];
    const int d0 = 32 * s + 8 * g;
    if (vec_ok && d0 < dh) {  // 8 consecutive head dims: 16-B (bf16) / 2x16-B (fp32) loads
      const T* qp = qkv_b + (long long)min(my_i, Tn - 1) * row3 + d0;
      float qf[8];
      if constexpr (sizeof(T) == 2) {
        const uint4 q4 = *reinterpret_cast<const uint4*>(qp);
        const uint32_t wv[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) qf[e] = __uint_as_float((wv[e >> 1] >> (16 * (e & 1))) << 16);
      } else {
        const float4 a4 = *reinterpret_cast<const float4*>(qp), b4 = *reinterpret_cast<const float4*>(qp + 4);
        qf[0] = a4.x; qf[1] = a4.y; qf[2] = a4.z; qf[3] = a4.w;
        qf[4] = b4.x; qf[5] = b4.y; qf[6] = b4.z; qf[7] = b4.w;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float q = my_i < Tn ? qf[e] : 0.f;
        qu[e] = my_i < Tn ? (q + pbu[h * dh + d0 + e]) * qscale : 0.f;
        qv[e] = my_i < Tn ? (q + pbv[h * dh + d0 + e]) * qscale : 0.f;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int d = d0 + e;
        if (my_i < Tn && d < dh) {
          const float q = Tr::to_f32(qkv_b[(long long)my_i * row3 + d]);
          qu[e] = (q + pbu[h * dh + d]) * qscale;
          qv[e] = (q + pbv[h * dh + d]) * qscale;
        } else {
          qu[e] = 0.f;
          qv[e] = 0.f;
        }
      }
    }
    fqu[s] = Tr::from8(qu);
    fqv[s] = Tr::from8(qv);
  }

  float m_run = -INFINITY, l_run = 0.f;
  f32x4 acc_o[NDT];
#pragma unroll
  for (int t = 0; t < NDT; ++t) acc_o[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int Tp = (Tn + KC - 1) / KC * KC;
  const int nchunk = Tp / KC;

  // ---- staging: registers (vector path) -> LDS ----
  uint4 rk[NKC], rv[NKC], rp[NPC];
  float rm = 0.f;
  // loads are unconditional (indices clamped into range) and out-of-range
  // values are zeroed at commit: a predicated load would make the compiler
  // wait for it on its own path, serialising the prefetch with the chunk math
  bool okk[NKC], okp[NPC];
  auto fetch = [&](int j0, bool need_v) {
    const int rbase = Tn - QB - i0 + j0;
#pragma unroll
    for (int i = 0; i < NKC; ++i) {
      const int c = tid + 256 * i, r = c / CPR, d = (c % CPR) * VEC, j = j0 + r;
      okk[i] = j < Tn && d < dh;
      const T* src = qkv_b + (long long)min(j, Tn - 1) * row3 + dh + min(d, dh - VEC);
      rk[i] = *reinterpret_cast<const uint4*>(src);
      rv[i] = *reinterpret_cast<const uint4*>(src + (need_v ? dh : 0));  // (stats pass: unused re-read of K)
    }
#pragma unroll
    for (int i = 0; i < NPC; ++i) {
      const int c = tid + 256 * i, rr = c / CPR, d = (c % CPR) * VEC, r = rbase + rr;
      okp[i] = rr < PBR - 1 && r >= 0 && r <= 2 * Tn - 2 && d < dh;
      rp[i] = *reinterpret_cast<const uint4*>(pk_h + (long long)min(max(r, 0), 2 * Tn - 2) * ldp +
                                              min(d, dh - VEC));
    }
    if (tid < KC) {
      const int j = j0 + tid;
      rm = (j < Tn && !(kpm && kpm[(long long)b * Tn + min(j, Tn - 1)])) ? 0.f : -INFINITY;
    }
  };
  auto commit = [&](bool need_v) {
#pragma unroll
    for (int i = 0; i < NKC; ++i) {
      const int c = tid + 256 * i, r = c / CPR, d = (c % CPR) * VEC;
      *reinterpret_cast<uint4*>(Ks + r * KR + d) = STAGE_SEL(okk[i], rk[i]);
      if (need_v) {
        const uint4 vv = STAGE_SEL(okk[i], rv[i]);
        if (TRV) {
          *reinterpret_cast<uint4*>(Vs + r * KR + d) = vv;
        } else {
          const T* ve = reinterpret_cast<const T*>(&vv);
#pragma unroll
          for (int e = 0; e < VEC; ++e) Vs[(d + e) * VR + r] = ve[e];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NPC; ++i) {
      const int c = tid + 256 * i, rr = c / CPR, d = (c % CPR) * VEC;
      *reinterpret_cast<uint4*>(Ps + rr * KR + d) = STAGE_SEL(okp[i], rp[i]);
    }
    if (tid < KC) {  // wave 0 (KC == 64): mask values and the chunk's any-masked flag
      Ms[tid] = rm;
      const bool anym = __any(rm != 0.f);
      if (tid == 0) reinterpret_cast<int*>(Ms)[KC] = anym;
    }
  };
  auto stage_scalar = [&](int j0, bool need_v) {  // unaligned head dims (e.g. d=144, H=4)
    const int rbase = Tn - QB - i0 + j0;
    for (int e = tid; e < KC * DHP; e += 256) {
      const int r = e / DHP, d = e - r * DHP, j = j0 + r;
      const bool ok = j < Tn && d < dh;
      Ks[r * KR + d] = ok ? qkv_b[(long long)j * row3 + dh + d] : Tr::from_f32(0.f);
      if (need_v) {
        const T v = ok ? qkv_b[(long long)j * row3 + 2 * dh + d] : Tr::from_f32(0.f);
        if (TRV)
          Vs[r * KR + d] = v;
        else
          Vs[d * VR + r] = v;
      }
    }
    for (int e = tid; e < PBR * DHP; e += 256) {
      const int rr = e / DHP, d = e - rr * DHP, r = rbase + rr;
      Ps[rr * KR + d] = (rr < PBR - 1 && r >= 0 && r <= 2 * Tn - 2 && d < dh) ? pk_h[(long long)r * ldp + d]
                                                                              : Tr::from_f32(0.f);
    }
    if (tid < KC) {
      const int j = j0 + tid;
      const float mv = (j < Tn && !(kpm && kpm[(long long)b * Tn + j])) ? 0.f : -INFINITY;
      Ms[tid] = mv;
      const bool anym = __any(mv != 0.f);
      if (tid == 0) reinterpret_cast<int*>(Ms)[KC] = anym;
    }
  };

  constexpr int NPASS = PROBS ? 2 : 1;
  for (int pass = 0; pass < NPASS; ++pass) {
    const bool stats_only = PROBS && pass == 0;
    const bool need_v = !stats_only;
    __syncthreads();
    if (vec_ok) {
      fetch(0, need_v);
      commit(need_v);
    } else {
      stage_scalar(0, need_v);
    }
    __syncthreads();
    ATT_TL(0);
    for (int ch = 0; ch < nchunk; ++ch) {
      ATT_TL(1 + 6 * ch);
      const int j0 = ch * KC;
      const bool more = ch + 1 < nchunk;
      if (vec_ok && more) fetch(j0 + KC, need_v);  // next chunk in flight during this chunk's math

      // ---- S^T (keys x queries) and G^T (band rows x queries) ----
      // per 32-wide head-dim step: all 9 fragment reads, then the 9 MFMAs;
      // G^T goes to the scratch only after its last MFMA (no read -> MFMA ->
      // store serialisation per tile)
      f32x4 acc_s[4], acc_g[5];
#pragma unroll
      for (int t = 0; t < 4; ++t) acc_s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 5; ++t) acc_g[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int pofs = 48 - 16 * w;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        typename Tr::frag fk[4], fpb[5];
#pragma unroll
        for (int t = 0; t < 4; ++t) fk[t] = Tr::load(Ks + (16 * t + c16) * KR + 8 * g + 32 * s);
#pragma unroll
        for (int t = 0; t < 5; ++t) fpb[t] = Tr::load(Ps + (pofs + 16 * t + c16) * KR + 8 * g + 32 * s);
#pragma unroll
        for (int t = 0; t < 4; ++t) Tr::mma(acc_s[t], fk[t], fqu[s]);
#pragma unroll
        for (int t = 0; t < 5; ++t) Tr::mma(acc_g[t], fpb[t], fqv[s]);
      }
      if (ALIAS) __syncthreads();  // every wave's Ks / Ps fragment reads are done: the scratch may overwrite them
#pragma unroll
      for (int t = 0; t < 5; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) Gw[(16 * t + 4 * g + r) * GS + c16] = acc_g[t][r];
      // G^T scratch is per wave: its LDS writes only need to have completed
      // (in-order per wave) before the shifted reads, no workgroup barrier
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

      ATT_TL(2 + 6 * ch);
      // ---- scores for this lane's query: keys jj = 16t + 4g + r ----
      // (log2 domain: Qu/Qv carry scale * log2(e), probabilities are exp2)
      const bool masked_chunk = __builtin_amdgcn_readfirstlane(reinterpret_cast<const int*>(Ms)[KC]) != 0;
      float sc[4][4];
      float cmax = -INFINITY;
      // additive attention mask (attn_mask, attention.py:604-611), scaled into
      // the log2 domain of the scores; bool masks arrive as 0 / -inf
      const float* amrow = am ? am + b * am_sb + h * am_sh + (long long)min(my_i, Tn - 1) * Tn : nullptr;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int jj = 16 * t + 4 * g + r;
          float v = acc_s[t][r] + Gw[(15 - c16 + jj) * GS + c16];
          if (masked_chunk) v += Ms[jj];
          if (amrow && j0 + jj < Tn) v += amrow[j0 + jj] * 1.4426950408889634f;
          sc[t][r] = v;
          cmax = fmaxf(cmax, v);
        }
      cmax = fmaxf(cmax, __shfl_xor(cmax, 16));
      cmax = fmaxf(cmax, __shfl_xor(cmax, 32));

      if (stats_only) {
        const float m_new = fmaxf(m_run, cmax);
        const float mref = m_new == -INFINITY ? 0.f : m_new;
        float ls = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) ls += __builtin_amdgcn_exp2f(sc[t][r] - mref);
        ls += __shfl_xor(ls, 16);
        ls += __shfl_xor(ls, 32);
        l_run = l_run * __builtin_amdgcn_exp2f(m_run - mref) + ls;
        m_run = m_new;
      } else {
        float p[4][4];
        if (PROBS) {
          const float mref = m_run == -INFINITY ? 0.f : m_run;
          const float inv = 1.0f / l_run;
          float* prow = probs + (((long long)b * H + h) * Tn + my_i) * Tn;
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int j = j0 + 16 * t + 4 * g + r;
              p[t][r] = __builtin_amdgcn_exp2f(sc[t][r] - mref) * inv;
              if (my_i < Tn && j < Tn) prow[j] = p[t][r];
            }
        } else {
          const float m_new = fmaxf(m_run, cmax);
          const float mref = m_new == -INFINITY ? 0.f : m_new;
          const float alpha = __builtin_amdgcn_exp2f(m_run - mref);
          float ls = 0.f;
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              p[t][r] = __builtin_amdgcn_exp2f(sc[t][r] - mref);
              ls += p[t][r];
            }
          ls += __shfl_xor(ls, 16);
          ls += __shfl_xor(ls, 32);
          l_run = l_run * alpha + ls;
          m_run = m_new;
#pragma unroll
          for (int t = 0; t < NDT; ++t) acc_o[t] *= alpha;
        }
        ATT_TL(3 + 6 * ch);
        // ---- O^T += V^T · P^T  (2 k-steps of 32 keys) ----
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          float pv[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            pv[r] = p[2 * s2][r];
            pv[4 + r] = p[2 * s2 + 1][r];
          }
          const typename Tr::frag fp = Tr::from8(pv);
#pragma unroll
          for (int t = 0; t < NDT; ++t) {
            typename Tr::frag fa;
            if constexpr (TRV) {
              fa = vt_frag_tr(reinterpret_cast<const bf16_t*>(Vs), KR, 32 * s2, 16 * t, lane);
            } else {
              const T* vrow = Vs + (16 * t + c16) * VR + 32 * s2 + 4 * g;
              fa = Tr::load2x4(vrow, vrow + 16);
            }
            Tr::mma(acc_o[t], fa, fp);
          }
        }
      }
      ATT_TL(4 + 6 * ch);
      __syncthreads();  // every wave done with this chunk's Ks / Vs / Ps / Gs
      ATT_TL(5 + 6 * ch);
      if (more) {
        if (vec_ok)
          commit(need_v);
        else
          stage_scalar(j0 + KC, need_v);
        __syncthreads();
      }
    }
  }
  ATT_TL(62);
  // ---- write O (row = this lane's query, cols d = 16t + 4g + r) ----
  if (my_i < Tn) {
    const float inv = PROBS ? 1.0f : 1.0f / l_run;
    T* orow = out + ((long long)b * Tn + my_i) * d_model + h * dh;
#pragma unroll
    for (int t = 0; t < NDT; ++t) {
      const int d = 16 * t + 4 * g;
      if (vec_ok && d + 3 < dh) {  // 4 consecutive head dims: one 8-B (bf16) / 16-B (fp32) store
        if constexpr (sizeof(T) == 2) {
          uint2 pk2;
          pk2.x = pack_bf16x2(acc_o[t][0] * inv, acc_o[t][1] * inv);
          pk2.y = pack_bf16x2(acc_o[t][2] * inv, acc_o[t][3] * inv);
          *reinterpret_cast<uint2*>(orow + d) = pk2;
        } else {
          *reinterpret_cast<float4*>(orow + d) =
              make_float4(acc_o[t][0] * inv, acc_o[t][1] * inv, acc_o[t][2] * inv, acc_o[t][3] * inv);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (d + r < dh) orow[d + r] = Tr::from_f32(acc_o[t][r] * inv);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// The encoder's inference path — bf16, dh = 64, no probabilities — with
// three workgroups per CU.  The kernel above carries the next chunk's K / V /
// band rows in 32 VGPRs (194 in all), so it runs two waves per SIMD: at
// B = 32, T = 376 its 768 workgroups take 1.5 rounds of 512.  Its score
// assembly was also 16 serialised LDS round trips per chunk (a per-chunk
// "any key masked" branch split it into read -> wait -> add steps).
// Here the tiles go global -> LDS by LDS-DMA (global_load_lds_dwordx4: no
// VGPRs, no ds_write) into unpadded 128-B rows whose 16-B chunks are
// XOR-swizzled on the global source address — K and the band:
// chunk ^ ((row >> 1) & 7), conflict-free ds_read_b128 fragments; V:
// chunk ^ (((row >> 1) & 3) << 1), conflict-free ds_read_b64_tr_b16.  G^T goes
// to a query-major scratch with the rel_shift applied on the write (row R of
// query ii lands at position R - (15 - ii); the first / last tile's positions
// outside the chunk's 64 keys clamp onto two spare slots), so the scores are
// four aligned 16-B reads.  Key padding: a 64-bit bitmap of the chunks that
// hold a padded key is built once per workgroup; only those chunks (and the
// last, for keys past Tn) apply a mask, so no wave writes a per-chunk mask row
// the others wait for.  Row max / sum: permlane half-swaps.  Two barriers per
// chunk:
//   A  this chunk's K / band landed in every wave and every wave is past the
//      previous chunk's P·V  -> issue this chunk's V;
//   B  V landed and every wave's S / G fragment reads are done -> read the
//      scratch, then issue the next chunk's K / band, which land under the
//      softmax and P·V.
// Measured (s_memtime / s_memrealtime per workgroup, B = 32, T = 376,
// profiles/r02_att_dma_timeline.log): all 768 workgroups start within 1 us
// (one round, three per CU); a CU's three finish in turn at ~12.5 / 15.3 /
// 17.5 us (oldest-first issue), i.e. the CU is issue / LDS bound, not waiting
// on memory.  Tried and slower: six waves x 16 queries per workgroup with
// double-buffered V and two workgroups per CU (27.5 us: the waves of a second
// workgroup do not always fit beside the first).
// The tiles are distinct __shared__ objects and the other LDS accesses come
// before a DMA is issued, so the compiler's LDS-DMA alias guard (a vmcnt wait
// before an LDS access it cannot tell apart from a DMA in flight) has little
// to wait for.  50 KB of LDS and <= 168 VGPRs: three workgroups per CU.
namespace dmak {
typedef float v2f __attribute__((ext_vector_type(2)));
constexpr int RB = 64;   // bf16 per staged row (dh = 64): 128 B
constexpr int PB = 128;  // band rows staged per chunk (127 used)
constexpr int G2 = 72;   // G scratch row (floats): 18 16-B slots, ≡ 2 mod 4
constexpr int GO = 4;    // scratch index of key 0 (spare slots GO - 1 and GO + KC)
__device__ __forceinline__ int swz_kp(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int swz_v(int row) { return ((row >> 1) & 3) << 1; }
// One LDS-DMA piece (64 lanes x 16 B to lds + 16 * lane), issued from inline
// asm: the compiler then sees no LDS write in flight and puts no alias-guard
// vmcnt wait before the LDS reads of the other tiles (with the builtin it
// waited for the next chunk's K / band before the P·V reads).  dma_barrier's
// vmcnt(0) + s_barrier is what orders the fills and the reads.
__device__ __forceinline__ void dma16(const bf16_t* src, bf16_t* lds) {
  const uint32_t la = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) bf16_t*)lds));
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(la) : "memory", "m0");
}
// The same piece from a wave-uniform base (SGPR pair) plus a per-lane byte
// offset computed once before the chunk loop; m0 (the LDS destination) is a
// precomputed scalar.  The interior chunks issue their DMAs with no VALU
// address arithmetic at all (the clamped form above cost ~75 VALU
// instructions per chunk, 8 of them quarter-rate multiplies, in a kernel
// whose chunk time is VALU issue).
__device__ __forceinline__ void dma16s(const void* sbase, uint32_t voff, uint32_t la) {
  asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(la) : "memory", "m0");
}
__device__ __forceinline__ uint32_t lds_addr(const void* lds) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)lds));
}
// this wave's DMA pieces and LDS accesses done, then the workgroup barrier
__device__ __forceinline__ void dma_barrier() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// V^T A-operand fragment (as vt_frag_tr) from the swizzled V tile;
// swz_v(r + 16) == swz_v(r)
__device__ __forceinline__ bf16x8 vt_frag_swz(const bf16_t* V, int k0, int dbase, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r0 = k0 + 4 * g + q, col = dbase + 4 * p;
  const bf16_t* a0 = V + r0 * RB + ((((col >> 3) ^ swz_v(r0)) << 3) | (col & 7));
  const bf16_t* a1 = a0 + 16 * RB;
  const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4_t*)(a0));
  const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4_t*)(a1));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
}  // namespace dmak

// BAND = false: plain scaled dot-product attention (MultiheadAttention of the
// TransformerEncoder, attention.py:642-779 over nn.MultiheadAttention): no
// positional band, no u / v biases — no band DMA, no G tiles, no scatter,
// 16 KB of LDS; otherwise the same chunk loop.
template <bool BAND>
__global__ void __launch_bounds__(256, 3) relpos_flash_dma_kernel(const bf16_t* __restrict__ qkv,
                                                                  const bf16_t* __restrict__ pk, int ldp,
                                                                  const float* __restrict__ pbu,
                                                                  const float* __restrict__ pbv,
                                                                  const uint8_t* __restrict__ kpm, int Tn, int H,
                                                                  float scale, bf16_t* __restrict__ out) {
  using namespace dmak;
  constexpr int dh = 64;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[KC * RB];
  __shared__ __attribute__((aligned(16))) bf16_t Ps[BAND ? PB * RB : 8];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[KC * RB];
  __shared__ __attribute__((aligned(16))) float Gs[BAND ? 4 * 16 * G2 : 4];
  __shared__ unsigned long long Mb[4];  // per-wave partial bitmaps of the chunks holding a padded key

  const int d_model = H * dh;
  const long long row3 = 3LL * d_model;
  const int nqb = (Tn + QB - 1) / QB;
  const int nwg = gridDim.x, orig = blockIdx.x;  // XCD-aware bijective remap, as above
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int qb = tile % nqb, bh = tile / nqb;
  const int h = bh % H, b = bh / H;
  const int i0 = qb * QB;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15, g = lane >> 4;
  const int my_i = i0 + 16 * w + c16;
  SBK_PROBE(const bool tl_on = tile == 200;)
  const bf16_t* qkv_b = qkv + (long long)b * Tn * row3 + h * 3 * dh;
  const bf16_t* pk_h = pk + h * dh;
  float* gq = Gs + w * 16 * G2 + c16 * G2 + GO;  // this lane's query row of the G scratch, at key 0
  const int lrow = lane >> 3, lchk = lane & 7;   // DMA piece: 8 rows x 8 16-B chunks

  // per-lane byte offsets of the interior-chunk DMA pieces (row stride x row
  // + swizzled 16-B chunk); the chunk's base goes in the scalar operand
  uint32_t offk[2], offv[2], offp[4], lak[2], lav[2], lap[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r0 = 16 * w + 8 * i, row = r0 + lrow;
    offk[i] = (uint32_t)(row * row3 + ((lchk ^ swz_kp(row)) << 3)) * 2u;
    offv[i] = (uint32_t)(row * row3 + ((lchk ^ swz_v(row)) << 3)) * 2u;
    lak[i] = lds_addr(Ks + r0 * RB);
    lav[i] = lds_addr(Vs + r0 * RB);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r0 = 32 * w + 8 * i, rr = r0 + lrow;
    offp[i] = BAND ? (uint32_t)(rr * ldp + ((lchk ^ swz_kp(rr)) << 3)) * 2u : 0u;
    lap[i] = BAND ? lds_addr(Ps + r0 * RB) : 0u;
  }
  auto dma_kp = [&](int j0) {
    const int rbase = Tn - QB - i0 + j0;  // band row 0
    if (j0 + KC <= Tn && (!BAND || (rbase >= 0 && rbase + PB <= 2 * Tn - 1))) {  // no row clamped
      const bf16_t* sk = qkv_b + (long long)j0 * row3 + dh;
#pragma unroll
      for (int i = 0; i < 2; ++i) dma16s(sk, offk[i], lak[i]);
      if constexpr (BAND) {
        const bf16_t* sp = pk_h + (long long)rbase * ldp;
#pragma unroll
        for (int i = 0; i < 4; ++i) dma16s(sp, offp[i], lap[i]);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // K rows 16w .. 16w+15
      const int r0 = 16 * w + 8 * i, row = r0 + lrow;
      dma16(qkv_b + (long long)min(j0 + row, Tn - 1) * row3 + dh + ((lchk ^ swz_kp(row)) << 3), Ks + r0 * RB);
    }
    if constexpr (BAND)
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // band rows 32w .. 32w+31
      const int r0 = 32 * w + 8 * i, rr = r0 + lrow;
      const int pr = min(max(rbase + rr, 0), 2 * Tn - 2);
      dma16(pk_h + (long long)pr * ldp + ((lchk ^ swz_kp(rr)) << 3), Ps + r0 * RB);
    }
  };
  auto dma_v = [&](int j0) {
    if (j0 + KC <= Tn) {
      const bf16_t* sv = qkv_b + (long long)j0 * row3 + 2 * dh;
#pragma unroll
      for (int i = 0; i < 2; ++i) dma16s(sv, offv[i], lav[i]);
      return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r0 = 16 * w + 8 * i, row = r0 + lrow;
      dma16(qkv_b + (long long)min(j0 + row, Tn - 1) * row3 + 2 * dh + ((lchk ^ swz_v(row)) << 3), Vs + r0 * RB);
    }
  };
  ATT_TL(0);
  SBK_PROBE(if (tid == 0 && orig < 4096) {
    g_att_wg[orig][0] = __builtin_amdgcn_s_memrealtime();
    g_att_wg[orig][2] = __builtin_amdgcn_s_memtime();
  })
  dma_kp(0);
  const int nchunk = (Tn + KC - 1) / KC;  // <= 64 (launcher)
  // Key padding: which chunks hold a padded key, as a 64-bit chunk bitmap
  // built once (wave w scans chunks w, w + 4, ...; merged after barrier A of
  // chunk 0).  Chunks without one add no mask at all; keys past Tn are masked
  // arithmetically in the last chunk.  (A per-chunk mask row written by one
  // wave made the other three wait for it at every barrier.)
  {
    unsigned long long bits = 0;
    if (kpm) {
      const uint8_t* kb = kpm + (long long)b * Tn;
      for (int c0 = w; c0 < nchunk; c0 += 8) {
        const int c1 = c0 + 4, ja = c0 * KC + lane, jb = c1 * KC + lane;
        const int ma = kb[min(ja, Tn - 1)];
        const int mb = c1 < nchunk ? (int)kb[min(jb, Tn - 1)] : 0;
        if (__ballot(ja < Tn && ma != 0)) bits |= 1ull << c0;
        if (__ballot(jb < Tn && mb != 0)) bits |= 1ull << c1;
      }
    }
    if (lane == 0) Mb[w] = bits;
  }
  uint32_t mlo = 0, mhi = 0;  // the merged bitmap (wave-uniform)

  // Qu / Qv B-operand fragments, pre-scaled into the exp2 domain
  const float qscale = scale * 1.4426950408889634f;
  bf16x8 fqu[2], fqv[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int d0 = 32 * s + 8 * g;
    const uint4 q4 = *reinterpret_cast<const uint4*>(qkv_b + (long long)min(my_i, Tn - 1) * row3 + d0);
    const uint32_t wv[4] = {q4.x, q4.y, q4.z, q4.w};
    // biases by unconditional vector loads (guarded scalar loads each became
    // a branch and a full wait)
    const f32x4 z4 = f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 bu0 = BAND ? *reinterpret_cast<const f32x4*>(pbu + h * dh + d0) : z4;
    const f32x4 bu1 = BAND ? *reinterpret_cast<const f32x4*>(pbu + h * dh + d0 + 4) : z4;
    const f32x4 bv0 = BAND ? *reinterpret_cast<const f32x4*>(pbv + h * dh + d0) : z4;
    const f32x4 bv1 = BAND ? *reinterpret_cast<const f32x4*>(pbv + h * dh + d0 + 4) : z4;
    float qu[8], qv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float q = __uint_as_float((wv[e >> 1] >> (16 * (e & 1))) << 16);
      const float bu = e < 4 ? bu0[e & 3] : bu1[e & 3], bv = e < 4 ? bv0[e & 3] : bv1[e & 3];
      qu[e] = my_i < Tn ? (q + bu) * qscale : 0.f;
      qv[e] = my_i < Tn ? (q + bv) * qscale : 0.f;
    }
    fqu[s] = MT<bf16_t>::from8(qu);
    fqv[s] = MT<bf16_t>::from8(qv);
  }

  float m_run = -INFINITY, l_run = 0.f;
  f32x4 acc_o[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc_o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int pofs = 48 - 16 * w;
  for (int ch = 0; ch < nchunk; ++ch) {
    const int j0 = ch * KC;
    const bool more = ch + 1 < nchunk;
    dma_barrier();  // A
    ATT_TL(1 + 5 * ch);
    if (ch == 0) {
      const unsigned long long m = Mb[0] | Mb[1] | Mb[2] | Mb[3];
      mlo = __builtin_amdgcn_readfirstlane((uint32_t)m);
      mhi = __builtin_amdgcn_readfirstlane((uint32_t)(m >> 32));
    }
    __builtin_amdgcn_sched_barrier(0);
    dma_v(j0);

    // S^T = K·Qu^T (4 tiles), G^T = P_band·Qv^T (5 tiles)
    f32x4 acc_s[4], acc_g[5];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc_s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 5; ++t) acc_g[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fk[4], fpb[5];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int row = 16 * t + c16;
        fk[t] = *reinterpret_cast<const bf16x8*>(Ks + row * RB + (((4 * s + g) ^ swz_kp(row)) << 3));
      }
      if constexpr (BAND)
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          const int row = pofs + 16 * t + c16;
          fpb[t] = *reinterpret_cast<const bf16x8*>(Ps + row * RB + (((4 * s + g) ^ swz_kp(row)) << 3));
        }
#pragma unroll
      for (int t = 0; t < 4; ++t) acc_s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fk[t], fqu[s], acc_s[t], 0, 0, 0);
      if constexpr (BAND)
#pragma unroll
        for (int t = 0; t < 5; ++t) acc_g[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fpb[t], fqv[s], acc_g[t], 0, 0, 0);
    }
    // rel_shift on the write: row R = 16t + 4g + r -> position R - (15 - c16)
    if constexpr (BAND)
#pragma unroll
      for (int t = 0; t < 5; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int p = 16 * t + 4 * g + r + c16 - 15;
          if (t == 0) p = max(p, -1);
          if (t == 4) p = min(p, KC);
          gq[p] = acc_g[t][r];
        }
    ATT_TL(2 + 5 * ch);
    dma_barrier();  // B
    ATT_TL(3 + 5 * ch);

    // scores for this lane's query, keys jj = 16t + 4g + r (log2 domain)
    f32x4 gv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
      gv[t] = BAND ? *reinterpret_cast<const f32x4*>(gq + 16 * t + 4 * g) : f32x4{0.f, 0.f, 0.f, 0.f};
    const bool chunk_padded = ((ch < 32 ? mlo >> ch : mhi >> (ch - 32)) & 1u) != 0u;
    __builtin_amdgcn_sched_barrier(0);
    if (more) dma_kp(j0 + KC);
    float p[4][4];
    float cmax = -INFINITY;
    // S + G as packed fp32 pairs (v_pk_add_f32: half the instructions of the
    // per-element adds; the chunk loop is VALU-issue bound)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const v2f sg = BAND ? v2f{acc_s[t][r], acc_s[t][r + 1]} + v2f{gv[t][r], gv[t][r + 1]}
                            : v2f{acc_s[t][r], acc_s[t][r + 1]};
        p[t][r] = sg[0];
        p[t][r + 1] = sg[1];
      }
    if (chunk_padded) {  // uniform branch, only in chunks holding a padded key
      const uint8_t* kb = kpm + (long long)b * Tn;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kb[min(j0 + 16 * t + 4 * g + r, Tn - 1)]) p[t][r] = -INFINITY;
    }
    if (j0 + KC > Tn) {  // last chunk: keys past Tn (their staged rows are clamped copies)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (j0 + 16 * t + 4 * g + r >= Tn) p[t][r] = -INFINITY;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) cmax = fmaxf(cmax, p[t][r]);
    cmax = col4_max(cmax);
    const float m_new = fmaxf(m_run, cmax);
    const float mref = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = __builtin_amdgcn_exp2f(m_run - mref);
    // p - m as packed pairs; the row sum as a tree of packed pairs (one
    // serial chain of 16 dependent adds before)
    v2f ls2[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      v2f e[2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const v2f d = v2f{p[t][2 * h2], p[t][2 * h2 + 1]} - v2f{mref, mref};
        e[h2] = v2f{__builtin_amdgcn_exp2f(d[0]), __builtin_amdgcn_exp2f(d[1])};
        p[t][2 * h2] = e[h2][0];
        p[t][2 * h2 + 1] = e[h2][1];
      }
      ls2[t] = e[0] + e[1];
    }
    const v2f lsv = (ls2[0] + ls2[1]) + (ls2[2] + ls2[3]);
    l_run = l_run * alpha + col4_sum(lsv[0] + lsv[1]);
    m_run = m_new;
#pragma unroll
    for (int t = 0; t < 4; ++t) acc_o[t] *= alpha;
    ATT_TL(4 + 5 * ch);
    // O^T += V^T · P^T (2 k-steps of 32 keys, permuted-k fragments as above)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      float pv[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pv[r] = p[2 * s2][r];
        pv[4 + r] = p[2 * s2 + 1][r];
      }
      const bf16x8 fp = MT<bf16_t>::from8(pv);
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc_o[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vt_frag_swz(Vs, 32 * s2, 16 * t, lane), fp, acc_o[t], 0, 0, 0);
    }
    ATT_TL(5 + 5 * ch);
  }
  if (my_i < Tn) {
    const float inv = 1.0f / l_run;
    bf16_t* orow = out + ((long long)b * Tn + my_i) * d_model + h * dh;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      uint2 pk2;
      pk2.x = pack_bf16x2(acc_o[t][0] * inv, acc_o[t][1] * inv);
      pk2.y = pack_bf16x2(acc_o[t][2] * inv, acc_o[t][3] * inv);
      *reinterpret_cast<uint2*>(orow + 16 * t + 4 * g) = pk2;
    }
  }
  ATT_TL(62);
  SBK_PROBE(__syncthreads(); if (tid == 0 && orig < 4096) {
    g_att_wg[orig][1] = __builtin_amdgcn_s_memrealtime();
    g_att_wg[orig][3] = __builtin_amdgcn_s_memtime();
  })
}

int launch_dma(const void* qkv, const void* pk, int ldp, const float* pbu, const float* pbv, const uint8_t* kpm, int B,
               int Tn, int H, float scale, void* out, hipStream_t s) {
  const int grid = B * H * ((Tn + QB - 1) / QB);
  if (pk)
    hipLaunchKernelGGL(relpos_flash_dma_kernel<true>, dim3(grid), dim3(256), 0, s, reinterpret_cast<const bf16_t*>(qkv),
                       reinterpret_cast<const bf16_t*>(pk), ldp, pbu, pbv, kpm, Tn, H, scale,
                       reinterpret_cast<bf16_t*>(out));
  else
    hipLaunchKernelGGL(relpos_flash_dma_kernel<false>, dim3(grid), dim3(256), 0, s, reinterpret_cast<const bf16_t*>(qkv),
                       nullptr, 0, nullptr, nullptr, kpm, Tn, H, scale, reinterpret_cast<bf16_t*>(out));
  SBK_CHECK_LAUNCH();
  return 0;
}

template <typename T, int DHP>
int launch(const void* qkv, const void* pk, int ldp, const float* pbu, const float* pbv, const uint8_t* kpm, int B,
           int Tn, int H, int dh, float scale, void* out, float* probs, hipStream_t s, const float* am = nullptr,
           long long am_sb = 0, long long am_sh = 0) {
  constexpr size_t lds = FlashLds<T, DHP>::bytes;
  static_assert(lds <= 160 * 1024, "LDS budget");
  const int grid = B * H * ((Tn + QB - 1) / QB);
  const int VEC = MT<T>::VEC;
  const int d_model = H * dh;
  const int vec_ok = (dh % VEC == 0) && (d_model % VEC == 0) && (ldp % VEC == 0) &&
                     ((reinterpret_cast<uintptr_t>(qkv) | reinterpret_cast<uintptr_t>(pk) | reinterpret_cast<uintptr_t>(out)) % 16 == 0);
  if (probs)
    hipLaunchKernelGGL((relpos_flash_kernel<T, DHP, true>), dim3(grid), dim3(256), lds, s,
                       reinterpret_cast<const T*>(qkv), reinterpret_cast<const T*>(pk), pbu, pbv, kpm, B, Tn, H, dh,
                       scale, reinterpret_cast<T*>(out), probs, vec_ok, ldp, am, am_sb, am_sh);
  else
    hipLaunchKernelGGL((relpos_flash_kernel<T, DHP, false>), dim3(grid), dim3(256), lds, s,
                       reinterpret_cast<const T*>(qkv), reinterpret_cast<const T*>(pk), pbu, pbv, kpm, B, Tn, H, dh,
                       scale, reinterpret_cast<T*>(out), probs, vec_ok, ldp, am, am_sb, am_sh);
  SBK_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// qkv: (B, T, 3*d) head-interleaved in_proj output [h][q|k|v][dh];
// pk: (2T-1, d) linear_pos output; pbu/pbv: (H*dh) fp32; kpm: (B, T) uint8 or null;
// out: (B, T, d); probs: (B, H, T, T) fp32 or null.
SBK_API int sbk_relpos_attention_ld(int dtype_bf16, const void* qkv, const void* pk, int ldp, const float* pbu,
                                    const float* pbv, const uint8_t* kpm, int B, int Tn, int H, int dh, float scale,
                                    void* out, float* probs, void* stream) {
  if (B <= 0 || Tn <= 0 || H <= 0 || dh <= 0 || dh > 128 || ldp < H * dh || !pk) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  // the encoder's inference path: bf16, dh = 64, no probabilities
  if (dtype_bf16 && dh == 64 && !probs && ldp % 8 == 0 && Tn <= 64 * 64 &&
      ((reinterpret_cast<uintptr_t>(qkv) | reinterpret_cast<uintptr_t>(pk) | reinterpret_cast<uintptr_t>(out)) % 16) == 0)
    return launch_dma(qkv, pk, ldp, pbu, pbv, kpm, B, Tn, H, scale, out, s);
  if (dtype_bf16)
    return dh <= 64 ? launch<bf16_t, 64>(qkv, pk, ldp, pbu, pbv, kpm, B, Tn, H, dh, scale, out, probs, s)
                    : launch<bf16_t, 128>(qkv, pk, ldp, pbu, pbv, kpm, B, Tn, H, dh, scale, out, probs, s);
  return dh <= 64 ? launch<float, 64>(qkv, pk, ldp, pbu, pbv, kpm, B, Tn, H, dh, scale, out, probs, s)
                  : launch<float, 128>(qkv, pk, ldp, pbu, pbv, kpm, B, Tn, H, dh, scale, out, probs, s);
}

// Plain scaled dot-product attention over the same head-interleaved qkv
// (no positional band, no biases): the band-free LDS-DMA kernel; bf16,
// dh = 64, T <= 4096, 16-B aligned operands (else SBK_ERR_ARG: the caller
// takes sbk_relpos_attention_ld with a zero band).
SBK_API int sbk_mha_attention(const void* qkv, const uint8_t* kpm, int B, int Tn, int H, int dh, float scale, void* out,
                              void* stream) {
  if (B <= 0 || Tn <= 0 || H <= 0 || dh != 64 || Tn > 64 * 64 ||
      ((reinterpret_cast<uintptr_t>(qkv) | reinterpret_cast<uintptr_t>(out)) % 16) != 0)
    return SBK_ERR_ARG;
  return launch_dma(qkv, nullptr, 0, nullptr, nullptr, kpm, B, Tn, H, scale, out, (hipStream_t)stream);
}

SBK_API int sbk_relpos_attention(int dtype_bf16, const void* qkv, const void* pk, const float* pbu, const float* pbv,
                                 const uint8_t* kpm, int B, int Tn, int H, int dh, float scale, void* out, float* probs,
                                 void* stream) {
  return sbk_relpos_attention_ld(dtype_bf16, qkv, pk, H * dh, pbu, pbv, kpm, B, Tn, H, dh, scale, out, probs, stream);
}

// sbk_relpos_attention_ld with an additive attention mask am (fp32): score
// (b, h, i, j) += am[b * am_sb + h * am_sh + i * T + j] after the 1/sqrt(d)
// scale, before the key-padding mask and the softmax (attention.py:598-611;
// a bool mask is passed as 0 / -inf).  A 2-D (T, T) mask has am_sb = am_sh
// = 0, a 3-D (B*H, T, T) one am_sb = H*T*T, am_sh = T*T.  General kernel.
SBK_API int sbk_relpos_attention_mask(int dtype_bf16, const void* qkv, const void* pk, int ldp, const float* pbu,
                                      const float* pbv, const uint8_t* kpm, const float* am, long long am_sb,
                                      long long am_sh, int B, int Tn, int H, int dh, float scale, void* out,
                                      float* probs, void* stream) {
  if (B <= 0 || Tn <= 0 || H <= 0 || dh <= 0 || dh > 128 || ldp < H * dh || !am || am_sb < 0 || am_sh < 0)
    return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (dtype_bf16)
    return dh <= 64 ? launch<bf16_t, 64>(qkv, pk, ldp, pbu, pbv, kpm, B, Tn, H, dh, scale, out, probs, s, am, am_sb,
                                         am_sh)
                    : launch<bf16_t, 128>(qkv, pk, ldp, pbu, pbv, kpm, B, Tn, H, dh, scale, out, probs, s, am, am_sb,
                                          am_sh);
  return dh <= 64 ? launch<float, 64>(qkv, pk, ldp, pbu, pbv, kpm, B, Tn, H, dh, scale, out, probs, s, am, am_sb,
                                      am_sh)
                  : launch<float, 128>(qkv, pk, ldp, pbu, pbv, kpm, B, Tn, H, dh, scale, out, probs, s, am, am_sb,
                                       am_sh);
}

SBK_PROBE_EXPORT(sbk_probe_att_tl, g_att_tl)
SBK_PROBE_EXPORT(sbk_probe_att_wg, g_att_wg)

SBK_API long long sbk_relpos_attention_lds(int dtype_bf16, int Tn, int dh) {
  (void)Tn;
  if (dtype_bf16) return dh <= 64 ? (long long)FlashLds<bf16_t, 64>::bytes : (long long)FlashLds<bf16_t, 128>::bytes;
  return dh <= 64 ? (long long)FlashLds<float, 64>::bytes : (long long)FlashLds<float, 128>::bytes;
}
