// Fused Conformer feed-forward block (bf16 MFMA):
//
//   z   = x + alpha * ( act( LN0(x) · W1^T + b1 ) · W2^T + b2 )
//   out = LNp(z)            (optional post-LayerNorm, e.g. norm2)
//   u   = LNn(out)          (optional, bf16/fp32 input of the next consumer)
//
// Reference: speechbrain/lobes/models/transformer/Conformer.py:239-260
// (macaron FFNs: ffn_module = Sequential(LayerNorm, PositionalwiseFeedForward,
// Dropout), 0.5-scaled residuals, norm2 after the second FFN) and
// speechbrain/nnet/attention.py:823-839 (PositionalwiseFeedForward).
//
// Optional projection tail (sbk_ffn_proj): y = u · Wp^T in bf16 — the
// MHSA in_proj of the next block (attention.py:549-553, RelPosMHAXL has no
// in_proj bias) — so u never leaves the CU and the QKV GEMM is no launch of
// its own.
//
// Design (MI355X): one workgroup (8 waves) owns BM = 48 rows for
// the whole block, so neither LN0(x) nor the (BM x H) hidden activation ever
// leaves the CU:
//   prologue : x rows (fp32) -> LayerNorm -> bf16 Xn; its MFMA fragments are
//              then held in VGPRs (96 per lane) for every phase-1 step; b1 -> LDS;
//   per chunk of HC = 256 hidden units (8 K-steps of 64):
//     phase 1: Hc^T = W1[c]·Xn^T  -> +b1, act -> bf16 Hs (LDS);
//     phase 2: acc2^T += W2[:, c]·Hs^T  (accumulators stay in VGPRs);
//   epilogue : +b2, alpha, residual, optional post-LN and next-LN over the
//              full rows (cross-wave reduction through LDS), float4 stores;
//   tail     : (projection) u -> Xn -> VGPR fragments, K1 steps per 256
//              output columns of Wp through the same ring, bf16 stores.
// Weight tiles (256 rows x 64 k = 32 KB) stream L2 -> LDS by LDS-DMA
// (global_load_lds_dwordx4: full 128-B lines, no VGPRs) into a 2-slot ring,
// one tile in flight behind the one being read (counted vmcnt; the last FFN
// steps already fetch the projection's first tiles).  Each wave stages only
// the weight rows it multiplies, so the ring steps need no workgroup barrier.
// The ring image is lane-linear; bank conflicts are removed by XOR-swizzling
// the 16-B chunk index with (row >> 1) & 7 on the global source address and
// on the fragment reads.  HBM traffic per row: D fp32 in + D fp32 out (+ D u
// out, or np bf16 projection outputs).
//
// Measured (M = 12032, H = 1024, s_memtime timeline of one workgroup of 251):
// prologue 10.6k cycles (x rows from HBM in lockstep with every other CU,
// then tile 0), 32 K-steps of ~650-700 cycles (12 MFMAs = 192 issue cycles
// per wave, 2 waves per SIMD; ~110 GB/s of weights into the CU, the DMA
// wait < 80 cycles), +1,400 on each chunk's activation step (Swish on 24
// values per lane: VALU), epilogue 8.3k (18 MB of out/u stores from every CU
// at once: HBM).  H = 2048 adds 0.5 us per K-step, so ~14 us of the 29.6 us
// launch is the fixed prologue/epilogue/launch cost, not the weight stream.
// Tried and slower or equal: 8-wave register-staged ring (48 us), 4 waves
// (69 us), fragment-shaped loads straight to VGPRs (64 us), row-owner waves
// with the hidden chunk in registers (78 us), a shared 3-slot ring with a
// barrier per K-step (42 us), LN'd rows re-read from LDS each step instead
// of VGPRs (36.7 us), a per-XCD rotated chunk order (35.0 us), a 3-slot ring
// with one hidden buffer (37.2 us), a third slot aliased onto Xn after the
// VGPR load (30.3 us), a tile-contiguous weight image (29.3 us).
// Round 2 (layer chain, 58 us): a single-pass row LayerNorm (sum and sum of
// squares in one LDS exchange, affine prefetched) was no faster (58.4 us).
// Round 3: no s_waitcnt vmcnt(0) left outside the last step.  The compiler
// guards a visible LDS access or the first use of a visible global load
// with vmcnt(0) (it does not count LDS-DMA in order), and __syncthreads()
// waits for vmcnt(0): each drained the two weight tiles in flight (and, in
// the tail, the stores).  Hence asm LDS accesses, asm prologue loads with
// one counted wait, LDS-only barriers, the epilogue vectors copied to LDS in
// the prologue, lane offsets recomputed instead of hoisted (spills 13 -> 4),
// and the out / projection stores interleaved into the projection steps
// with counted waits.  s_memtime timeline: 129.5k -> 128.5k cycles, the
// steps unchanged at ~1,030 cycles: a step issues 32 KB of LDS-DMA per CU,
// ~40 B/clk, the per-CU LDS-DMA issue rate (MI355X_MICROARCH ldsdma-fill:
// 16 KiB per 0.154 us), while its 12 MFMAs per wave fill 384 of them.
// Fewer weight bytes per CU need more rows per CU than M / 256 = 47.
#include "mfma.h"

using namespace sbk;

namespace {

enum Act { ACT_NONE = 0, ACT_SWISH = 1, ACT_GLU = 2, ACT_LRELU = 3, ACT_GELU = 4 };

struct FfnArgs {
  const float* x;  // (M, D) fp32
  int M, H;
  const float *g0, *b0;
  float eps0;
  // the launch's weight stream: ST tiles of 256 rows x 64 k (32 KB) in
  // stream order, each row's 16-B chunks pre-swizzled (sbk_ffn_image), so a
  // wave's share of a tile is one contiguous 4 KB run
  const bf16_t* img;
  const float* b1;
  int act;
  float slope;
  const float* b2;
  float alpha;
  const float *gp, *bp;  // post-LN (or null)
  float epsp;
  float* out;  // (M, D) fp32, may alias x
  const float *gn, *bn;  // next-LN (or null)
  float epsn;
  void* u;
  int u_bf16;
  int np;      // projection of next-LN(out): np output columns (0: none)
  bf16_t* yp;  // (M, np) bf16
  // CHAIN: a second FFN block on the first one's output, which stays on chip
  // (the first block's `out` is not written): FFN2 + norm2 of layer i, then
  // FFN1 of layer i+1 with its own LN0, alpha, w1/b1/w2/b2; its result goes
  // to `out`, next-LN and the projection tail as for a single block
  const float *g0b, *b0b;  // null: one block
  float eps0b;
  const float *b1b, *b2b;
  float alphab;
  // LayerNorm statistics over the first d_eff of the D columns (the others
  // are zero-padded channels: D = 256 carrying a d_model < 256 model whose
  // LN gains / biases and weight rows are zero there): inv_n = 1 / d_eff,
  // npad = D - d_eff (each padded zero adds mean^2 to the centred sum)
  float inv_n, npad;
};

__device__ __forceinline__ bf16x8 ld8(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

template <int V>
struct IntC {
  static constexpr int value = V;
};

constexpr int FFN_BM = 48;
constexpr int FFN_PAD = 16;  // LDS row pad (elements): conflict-free b128 reads (8 measured slower)
constexpr int FFN_NW = 8, FFN_NT = FFN_NW * 64;  // 8 waves: LN'd rows fit in VGPRs (2 waves/SIMD)
// Xn / Hs rows: element (row, col) at row * stride + (col ^ ffn_sw(row)), the
// 16-B chunks of rows with bit 2 set swapped in pairs.  The 8-B column stores
// (16 rows fr of one column per ds_write_b64 lane group: MI355X_MICROARCH
// §LDS) were 4-way conflicted at the 544-B pitch — rows fr, fr + 4, fr + 8,
// fr + 12 on one bank pair — and are 2-way with it, the floor for 16-B-aligned
// rows; the b128 fragment reads stay conflict-free.  Counted: 720 of the 942
// conflict cycles per wave (SQ_LDS_BANK_CONFLICT, profiles/r04t_chain_sq_counters.txt).
__device__ __forceinline__ constexpr int ffn_sw(int row) { return ((row >> 2) & 1) << 3; }
static_assert(FFN_NW % 8 == 0, "rows w + FFN_NW * i share bit 2 with w (their swizzle is ffn_sw(w))");
// row-reduction scratch stride (floats): 16-B-aligned rows whose partial
// stores (16 lanes, rows fr) are 2-way and whose b128 reads are conflict-free
// (a stride of NW = 8 made them 4-way and 2-way: 66 conflict cycles per LayerNorm)
constexpr int FFN_RS = 12;

#define FFN_MFMA(A, B, C) __builtin_amdgcn_mfma_f32_16x16x32_bf16((A), (B), (C), 0, 0, 0)

template <int ACT>
__device__ __forceinline__ float act_fn(float v, float slope) {
  if (ACT == ACT_SWISH) return v * __builtin_amdgcn_rcpf(1.0f + __expf(-v));  // bf16 hidden: approx rcp
  if (ACT == ACT_LRELU) return v >= 0.f ? v : v * slope;
  if (ACT == ACT_GELU) return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
  return v;
}

// LDS read the compiler cannot see (it would guard a visible one with
// s_waitcnt vmcnt(0) against the in-flight LDS-DMA tiles, draining stores too)
__device__ __forceinline__ f32x4 lds_f4(const float* p) {
  f32x4 v;
  const uint32_t la = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) float*)p);
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(la) : "memory");
  return v;
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}
__device__ __forceinline__ float lds_f1(const float* p) {
  float v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}
__device__ __forceinline__ void lds_st1(float* p, float v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st4(float* p, f32x4 v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st2(void* p, uint2 v) {
  const unsigned long long u = (unsigned long long)v.x | ((unsigned long long)v.y << 32);
  asm volatile("ds_write_b64 %0, %1" ::"v"(lds_addr(p)), "v"(u) : "memory");
}
// s_waitcnt lgkmcnt(0) that a value read by the asm LDS loads above depends
// on: its uses cannot be scheduled before the wait (the first tie waits, the
// others retire at once)
template <typename V>
__device__ __forceinline__ void tie(V& v) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v));
}
// workgroup barrier on LDS traffic only: __syncthreads() also waits for
// vmcnt(0), i.e. for every LDS-DMA tile and store in flight
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// global load the compiler cannot see: it would follow a visible one's first
// use with s_waitcnt vmcnt(0) (it does not count LDS-DMA in order), draining
// the weight tiles issued after it.  The caller waits (asm) and then vtie()s.
__device__ __forceinline__ f32x4 gld4(const float* p) {
  f32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void vtie(f32x4& v) { asm volatile("" : "+v"(v)); }

// s_waitcnt vmcnt(n) for a wave-uniform n known only at run time
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
  }
}

// Full-row LayerNorm of the epilogue values z (in place).  Lane (w, g, fr)
// holds rows mt*16 + fr, units (w*T2 + j)*16 + 4g + e; row statistics are
// reduced over g by shuffles and over the NW waves through red[BM][FFN_RS]; gam /
// bet are LDS copies.  Every LDS access is explicit (asm) and the barriers
// wait on LDS only, so the weight tiles and stores in flight stay in flight.
// (One barrier per pass with a buffer per pass measured 1.5 us slower per
// chain launch than two barriers over one buffer.)
template <int D, int T2, int MT, int NW>
__device__ __forceinline__ void row_ln(float (&z)[T2][MT][4], float* red, const float* gam, const float* bet, float eps,
                                       int w, int g, int fr, float inv_n, float npad) {
  static_assert(NW == 8, "two b128 reads per row");
  float mean[MT], rstd[MT];
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    float part[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < T2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float dv = pass ? z[j][mt][e] - mean[mt] : z[j][mt][e];
          s += pass ? dv * dv : dv;
        }
      part[mt] = col4_sum(s);
    }
    lds_barrier();  // the previous readers of red are done
    if (g == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) lds_st1(red + (mt * 16 + fr) * FFN_RS + w, part[mt]);
    }
    lds_barrier();
    f32x4 rv[MT][2];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      rv[mt][0] = lds_f4(red + (mt * 16 + fr) * FFN_RS);
      rv[mt][1] = lds_f4(red + (mt * 16 + fr) * FFN_RS + 4);
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      tie(rv[mt][0]);
      tie(rv[mt][1]);
      const float t = (rv[mt][0][0] + rv[mt][0][1]) + (rv[mt][0][2] + rv[mt][0][3]) + (rv[mt][1][0] + rv[mt][1][1]) +
                      (rv[mt][1][2] + rv[mt][1][3]);
      if (pass)
        rstd[mt] = 1.0f / sqrtf((t - npad * mean[mt] * mean[mt]) * inv_n + eps);
      else
        mean[mt] = t * inv_n;
    }
  }
  f32x4 gv[T2], bv[T2];
#pragma unroll
  for (int j = 0; j < T2; ++j) {
    const int d = (w * T2 + j) * 16 + 4 * g;
    gv[j] = lds_f4(gam + d);
    bv[j] = lds_f4(bet + d);
  }
#pragma unroll
  for (int j = 0; j < T2; ++j) {
    tie(gv[j]);
    tie(bv[j]);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) z[j][mt][e] = (z[j][mt][e] - mean[mt]) * rstd[mt] * gv[j][e] + bv[j][e];
  }
}

// A-operand fragments of the LayerNorm'd rows (Xn, bf16, row stride XS)
// into VGPRs for every K-step of a block
template <int K1, int KS, int MT, int XS, int BK>
__device__ __forceinline__ void load_frags(bf16x8 (&xa)[K1][KS][MT], const bf16_t* Xn, int fr, int fk) {
#pragma unroll
  for (int r = 0; r < K1; ++r)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        asm volatile("ds_read_b128 %0, %1"
                     : "=v"(xa[r][ks][mt])
                     : "v"(lds_addr(Xn + (mt * 16 + fr) * XS + r * BK + ks * 32 + fk))
                     : "memory");
#pragma unroll
  for (int r = 0; r < K1; ++r)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) tie(xa[r][ks][mt]);
}


// s_memtime timeline of the waves of workgroup 128 (probe builds only)
SBK_PROBE_BUFFER(g_ffn_tl, 16, 256)
#define FFN_TL(i) SBK_PROBE(if (tl_rec >= 0 && lane == 0) g_ffn_tl[tl_rec][i] = __builtin_amdgcn_s_memtime();)

template <int D, int ACT, bool PROJ, bool CHAIN>
__global__ void __launch_bounds__(FFN_NT) ffn_kernel(FfnArgs a) {
  constexpr int BM = FFN_BM, HC = 256, NW = FFN_NW, NT = FFN_NT;
  constexpr int XS = D + FFN_PAD, HS = HC + FFN_PAD;   // LDS row strides (elements), +32 B pad: conflict-free b128 reads
  constexpr int MT = BM / 16;                // m-tiles (3)
  constexpr int T = 256 / 16 / FFN_NW;       // 16-row weight tiles per wave (HC/16/NW = D/16/NW)
  constexpr int BK = 64;                     // K per step: one 128-B line per weight row
  constexpr int K1 = D / BK, K2 = HC / BK, SPC = K1 + K2;
  constexpr int NB = 2;                      // ring slots: a slot is refilled as soon as its fragments are in VGPRs
  constexpr int TROWS = 256;                 // rows per weight tile (HC for W1, D for W2, 256 output columns of Wp)
  constexpr int GL = TROWS * BK * 2 / 16 / NT;  // LDS-DMA instructions per thread per tile (4)
  static_assert(GL * 8 == T * 16, "each wave stages exactly the weight rows it multiplies");
  constexpr int PER = D / 64;                // LN: floats per lane (4)
  static_assert(PER == 4 && D == 256 && HC / 16 / NW == T && D / 16 / NW == T, "shape");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);          // NB x TROWS x BK (linear 128-B rows)
  bf16_t* Xn = ring + NB * TROWS * BK;                      // BM x XS
  bf16_t* Hs = Xn + BM * XS;                                // 2 x BM x HS
  float* b1s = reinterpret_cast<float*>(Hs + 2 * BM * HS);  // H (CHAIN: 2 H, block A then B)
  float* red = b1s + (CHAIN ? 2 : 1) * a.H;                 // BM x FFN_RS row partials
  // epilogue vectors, copied to LDS in the prologue so that no global load
  // (and its in-order vmcnt wait behind the weight tiles) sits between blocks
  float* prm = red + BM * FFN_RS;                           // P_* x D
  enum { P_B2 = 0, P_GP, P_BP, P_G0B, P_B0B, P_B2B, P_GN, P_BN, P_N };
  static_assert(P_N == NW, "one parameter row per wave");

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, g = lane >> 4, fk = (8 * g) ^ ffn_sw(fr);  // chunk g of the swizzled rows mt*16 + fr
  const int m0 = blockIdx.x * BM;
  const int NCH = a.H / HC;
  const int S = NCH * SPC;                              // K-steps of one FFN block
  const int SF = CHAIN ? 2 * S : S;                     // FFN K-steps (blocks A, B)
  const int SP = PROJ ? (a.np / TROWS) * K1 : 0;        // projection K-steps (image tiles after the FFN ones)
  const int ST = SF + SP;
  SBK_PROBE(const int tl_rec = blockIdx.x == 128 ? w : -1;)
  FFN_TL(0);

  // ---- weight tile s -> ring slot (LDS-DMA, 1 KB = 8 rows per wave-instruction)
  // lane L of instruction i writes row R0 + L/8, 16-B chunk L%8 (linear image)
  // and fetches source chunk (L%8) ^ ((row >> 1) & 7): the read side applies
  // the same involution.  Steps S.. are the projection's (256 columns of Wp
  // by 64 k per tile, column block after column block).
  auto issue = [&](int s, int slot) __attribute__((always_inline)) {
    // tile s of the image: wave w's 4 KB (its 32 rows, lane-linear) by GL
    // pieces of 1 KB from one base address and immediate offsets, which the
    // instruction applies to the global and the LDS address alike (one m0
    // per tile; the per-piece address arithmetic and tile-index logic of a
    // strided source cost ~100 scalar and vector instructions per step)
    const bf16_t* src = a.img + (long long)s * (TROWS * BK) + w * (GL * 512) + lane * 8;
    bf16_t* dst = ring + slot * (TROWS * BK) + w * (GL * 512);
    const auto gs = (const __attribute__((address_space(1))) void*)src;
    const auto ls = (__attribute__((address_space(3))) void*)dst;
    static_assert(GL == 4, "four 1-KB pieces per wave and tile");
    __builtin_amdgcn_global_load_lds(gs, ls, 16, 0, 0);
    __builtin_amdgcn_global_load_lds(gs, ls, 16, 1024, 0);
    __builtin_amdgcn_global_load_lds(gs, ls, 16, 2048, 0);
    __builtin_amdgcn_global_load_lds(gs, ls, 16, 3072, 0);
  };
  // ---- prologue.  Every HBM read of the launch is issued here, before the
  // weight stream: the residual x values of this lane's epilogue outputs
  // (held in VGPRs through the main loop; rows clamped, masked at the end) and
  // the x rows of the LayerNorm, so their latency overlaps the first weight
  // tiles instead of being paid again after the last MFMA.
  constexpr int NRW = (BM + NW - 1) / NW;    // LN rows per wave
  f32x4 xres[T][MT];
#pragma unroll
  for (int j = 0; j < T; ++j)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int row = min(m0 + mt * 16 + fr, a.M - 1);
      xres[j][mt] = gld4(a.x + (long long)row * D + (w * T + j) * 16 + 4 * g);
    }
  f32x4 xv[NRW];
#pragma unroll
  for (int i = 0; i < NRW; ++i) {
    const int rr = w + i * NW, row = min(m0 + rr, a.M - 1);
    xv[i] = gld4(a.x + (long long)row * D + lane * PER);
  }
  f32x4 g04 = gld4(a.g0 + lane * PER), b04 = gld4(a.b0 + lane * PER);
  // wave w loads parameter row w (null rows are never read); lane-quads of b1 / b1b
  const float* psrc = w == P_B2 ? a.b2 : w == P_GP ? a.gp : w == P_BP ? a.bp : w == P_G0B ? a.g0b
                    : w == P_B0B ? a.b0b : w == P_B2B ? a.b2b : w == P_GN ? a.gn : a.bn;
  f32x4 pv = f32x4{0.f, 0.f, 0.f, 0.f}, b1v = pv, b1bv = pv;
  if (psrc) pv = gld4(psrc + lane * PER);
  const bool b1t = tid * 4 < a.H;
  if (b1t) b1v = gld4(a.b1 + tid * 4);
  if (CHAIN && b1t) b1bv = gld4(a.b1b + tid * 4);
  issue(0, 0);
  issue(1, 1);
  // every load above has landed; the two tiles stay in flight
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NB * GL) : "memory");
#pragma unroll
  for (int j = 0; j < T; ++j)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) vtie(xres[j][mt]);
#pragma unroll
  for (int i = 0; i < NRW; ++i) vtie(xv[i]);
  vtie(g04);
  vtie(b04);
  vtie(pv);
  vtie(b1v);
  vtie(b1bv);

  // LayerNorm of the workgroup's rows -> Xn (bf16); b1 -> LDS
#pragma unroll
  for (int i = 0; i < NRW; ++i) {
    const int rr = w + i * NW;
    if (rr >= BM) break;
    const bool live = m0 + rr < a.M;
    const float v[4] = {live ? xv[i][0] : 0.f, live ? xv[i][1] : 0.f, live ? xv[i][2] : 0.f, live ? xv[i][3] : 0.f};
    const float mean = wave_sum_v(v[0] + v[1] + v[2] + v[3]) * a.inv_n;
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) q += (v[e] - mean) * (v[e] - mean);
    const float rstd = 1.0f / sqrtf((wave_sum_v(q) - a.npad * mean * mean) * a.inv_n + a.eps0);
    uint2 pk;
    pk.x = pack_bf16x2((v[0] - mean) * rstd * g04[0] + b04[0], (v[1] - mean) * rstd * g04[1] + b04[1]);
    pk.y = pack_bf16x2((v[2] - mean) * rstd * g04[2] + b04[2], (v[3] - mean) * rstd * g04[3] + b04[3]);
    lds_st2(Xn + rr * XS + ((lane * PER) ^ ffn_sw(w)), pk);  // rr = w + i * NW, NW % 8 == 0
  }
  static_assert(2048 <= NT * 4, "b1 in one float4 per thread");
  if (psrc) lds_st4(prm + w * D + lane * PER, pv);
  if (b1t) lds_st4(b1s + tid * 4, b1v);
  if (CHAIN && b1t) lds_st4(b1s + a.H + tid * 4, b1bv);

  f32x4 acc1[T][MT], acc2[T][MT];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      acc1[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc2[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

  // ---- main loop.  Every wave stages (LDS-DMA) and reads only its own weight
  // rows, so the 2-slot ring needs no workgroup barrier: a slot takes tile
  // s+2 as soon as the wave's fragments of tile s are in VGPRs.  Barriers
  // remain only where waves share data: Xn (before the loop) and the hidden
  // chunk Hs (written at r == K1-1, read from r == K1; double-buffered by
  // chunk parity).  The LayerNorm'd rows are the A operand of every phase-1
  // step: their fragments stay in VGPRs for the whole launch (96 VGPRs).
  // (Tried and slower: fragments of step s+1 read under the MFMAs of step s —
  // 8 waves 40.8 us, 16 waves spill; weights streamed straight into VGPRs
  // with 4 steps in flight instead of LDS-DMA — 45 us at 8 or 16 waves.)
  FFN_TL(1);
  lds_barrier();
  bf16x8 xa[K1][BK / 32][MT];
  load_frags<K1, BK / 32, MT, XS, BK>(xa, Xn, fr, fk);
  // one K-step: tile s landed -> this wave's fragments (phase 1: the held Xn
  // fragments of k-step r; phase 2: the hidden chunk Hc at k-step r) -> the
  // slot takes tile s+NB -> 12 MFMAs into acc1 / acc2
  auto step = [&](int s, int r, bool ph2, const bf16_t* Hc, bool bar, auto&& post) __attribute__((always_inline)) {
    // this wave's rows of tile s landed (tile s+1 stays in flight)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL * (NB - 1)) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (bar) __builtin_amdgcn_s_barrier();
    if (s < 96) FFN_TL(2 + 2 * s);
    const bf16_t* tile = ring + (s % NB) * TROWS * BK;
    bf16x8 fw[BK / 32][T], fa[BK / 32][MT];
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const int row = w * (T * 16) + t * 16 + fr;
        fw[ks][t] = ld8(tile + row * BK + (((ks * 4 + g) ^ ((row >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        fa[ks][mt] = ph2 ? ld8(Hc + (mt * 16 + fr) * HS + r * BK + ks * 32 + fk) : xa[ph2 ? 0 : r][ks][mt];
    }
    // once this step's fragments are in VGPRs its slot takes tile s+2 (tail:
    // the projection's first tiles, or a harmless reload of the last tile)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    issue(min(s + NB, ST - 1), s % NB);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks)
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          if (ph2)
            acc2[t][mt] = FFN_MFMA(fw[ks][t], fa[ks][mt], acc2[t][mt]);
          else
            acc1[t][mt] = FFN_MFMA(fw[ks][t], fa[ks][mt], acc1[t][mt]);
        }
    // (a sched_barrier here, keeping the MFMAs above the next step's tile
    // wait instead of letting the scheduler sink most of them below it,
    // measured equal: 55.4-56.4 vs 53.8-56.6 us, profiles/r04i_chain_time.log)
    post();  // VALU work that rides under this step's MFMAs (after its DMA issue)
    if (s < 96) FFN_TL(3 + 2 * s);
  };
  auto none = []() __attribute__((always_inline)) {};
  // hidden tiles i = t*MT + mt in [i0, i1) of acc1 -> +b1, act -> Hn (4
  // consecutive units per lane, one 8-B store); acc1 tiles zeroed.  b1 and Hn
  // by explicit ds_read / ds_write: compiler-visible LDS accesses here get an
  // s_waitcnt vmcnt(0) (alias guard against the in-flight LDS-DMA tiles),
  // draining the weight stream
  auto act_tiles = [&](int i0, int i1, const float* b1c, bf16_t* Hn) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < T; ++t) {
      if ((t + 1) * MT <= i0 || t * MT >= i1) continue;
      const int n = w * (T * 16) + t * 16 + 4 * g;
      f32x4 bb;
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(bb) : "v"(lds_addr(b1c + n)) : "memory");
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int i = t * MT + mt;
        if (i < i0 || i >= i1) continue;
        const f32x4 v = acc1[t][mt];
        uint2 pk;
        pk.x = pack_bf16x2(act_fn<ACT>(v[0] + bb[0], a.slope), act_fn<ACT>(v[1] + bb[1], a.slope));
        pk.y = pack_bf16x2(act_fn<ACT>(v[2] + bb[2], a.slope), act_fn<ACT>(v[3] + bb[3], a.slope));
        const unsigned long long pv = (unsigned long long)pk.x | ((unsigned long long)pk.y << 32);
        asm volatile("ds_write_b64 %0, %1" ::"v"(lds_addr(Hn + (mt * 16 + fr) * HS + (n ^ ffn_sw(fr)))), "v"(pv) : "memory");
        acc1[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  for (int stage = 0; stage < (CHAIN ? 2 : 1); ++stage) {
  if (CHAIN && stage == 1) {
    FFN_TL(197);
    // ---- between the blocks: A's rows z = x + alpha (acc2 + b2) -> post-LN
    // (norm2) are B's residual (held in xres) and, through B's LN0, its
    // phase-1 operand (Xn -> VGPR fragments); nothing goes to HBM
    float z[T][MT][4];
#pragma unroll
    for (int j = 0; j < T; ++j) {
      const int d = (w * T + j) * 16 + 4 * g;
      f32x4 bb = lds_f4(prm + P_B2 * D + d);
      tie(bb);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const f32x4 xr = xres[j][mt];
        z[j][mt][0] = xr[0] + a.alpha * (acc2[j][mt][0] + bb[0]);
        z[j][mt][1] = xr[1] + a.alpha * (acc2[j][mt][1] + bb[1]);
        z[j][mt][2] = xr[2] + a.alpha * (acc2[j][mt][2] + bb[2]);
        z[j][mt][3] = xr[3] + a.alpha * (acc2[j][mt][3] + bb[3]);
        acc1[j][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc2[j][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    FFN_TL(200);
    if (a.gp) row_ln<D, T, MT, NW>(z, red, prm + P_GP * D, prm + P_BP * D, a.epsp, w, g, fr, a.inv_n, a.npad);
    FFN_TL(201);
#pragma unroll
    for (int j = 0; j < T; ++j)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) xres[j][mt] = f32x4{z[j][mt][0], z[j][mt][1], z[j][mt][2], z[j][mt][3]};
    row_ln<D, T, MT, NW>(z, red, prm + P_G0B * D, prm + P_B0B * D, a.eps0b, w, g, fr, a.inv_n, a.npad);
    FFN_TL(202);
#pragma unroll
    for (int j = 0; j < T; ++j) {
      const int d = (w * T + j) * 16 + 4 * g;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        uint2 pk;
        pk.x = pack_bf16x2(z[j][mt][0], z[j][mt][1]);
        pk.y = pack_bf16x2(z[j][mt][2], z[j][mt][3]);
        lds_st2(Xn + (mt * 16 + fr) * XS + (d ^ ffn_sw(fr)), pk);
      }
    }
    lds_barrier();
    FFN_TL(203);
    load_frags<K1, BK / 32, MT, XS, BK>(xa, Xn, fr, fk);
    FFN_TL(198);
  }
  const float* b1st = b1s + stage * a.H;  // this block's b1 (LDS)
  for (int c = 0; c < NCH; ++c) {
    const int s0 = stage * S + c * SPC;
#pragma unroll
    for (int r = 0; r < K1; ++r) step(s0 + r, r, false, nullptr, false, none);
    // hidden chunk -> +b1, act -> Hc; phase 2 reads it after the next step's
    // barrier.  The buffer written here was last read in chunk c-2, before
    // every wave passed chunk c-1's first phase-2 barrier.
    bf16_t* Hc = Hs + (c & 1) * BM * HS;
    act_tiles(0, T * MT, b1st + c * HC, Hc);
#pragma unroll
    for (int p = 0; p < K2; ++p) step(s0 + K1 + p, p, true, Hc, p == 0, none);
  }
  }  // stage
  if (!PROJ) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // retire the tail reloads
  FFN_TL(194);

  // ---- epilogue: lane holds rows m = mt*16 + fr, units d = (w*T + j)*16 + 4g .. +3
  // (CHAIN: the parameters of block B, which has no post-LN)
  const float* b2f = prm + (CHAIN ? P_B2B : P_B2) * D;
  const float alphaf = CHAIN ? a.alphab : a.alpha;
  const bool postln = !CHAIN && a.gp;
  float z[T][MT][4];
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const int d = (w * T + j) * 16 + 4 * g;
    f32x4 bb = lds_f4(b2f + d);
    tie(bb);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const f32x4 xr = xres[j][mt];
      z[j][mt][0] = xr[0] + alphaf * (acc2[j][mt][0] + bb[0]);
      z[j][mt][1] = xr[1] + alphaf * (acc2[j][mt][1] + bb[1]);
      z[j][mt][2] = xr[2] + alphaf * (acc2[j][mt][2] + bb[2]);
      z[j][mt][3] = xr[3] + alphaf * (acc2[j][mt][3] + bb[3]);
    }
  }
  FFN_TL(195);
  if (postln) row_ln<D, T, MT, NW>(z, red, prm + P_GP * D, prm + P_BP * D, a.epsp, w, g, fr, a.inv_n, a.npad);
  if (PROJ) {
    // the out rows wait in LDS (over the hidden-chunk buffers, free once the
    // row_ln barriers have passed) until the last weight tile has landed: a
    // store is counted by vmcnt like the LDS-DMA tiles, so a store issued
    // before a tile wait would hold that wait for its HBM write
    float* Zo = reinterpret_cast<float*>(Hs);  // BM x ZS fp32
    constexpr int ZS = D + 4;
    static_assert(BM * ZS * 4 <= 2 * BM * HS * 2, "out rows fit over Hs");
#pragma unroll
    for (int j = 0; j < T; ++j)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) xres[j][mt] = f32x4{z[j][mt][0], z[j][mt][1], z[j][mt][2], z[j][mt][3]};
    // u = next-LN(out) -> Xn (bf16) -> VGPR fragments, the A operand of the projection
    row_ln<D, T, MT, NW>(z, red, prm + P_GN * D, prm + P_BN * D, a.epsn, w, g, fr, a.inv_n, a.npad);
    FFN_TL(204);
#pragma unroll
    for (int j = 0; j < T; ++j) {
      const int d = (w * T + j) * 16 + 4 * g;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        lds_st4(Zo + (mt * 16 + fr) * ZS + d, xres[j][mt]);
        uint2 pk;
        pk.x = pack_bf16x2(z[j][mt][0], z[j][mt][1]);
        pk.y = pack_bf16x2(z[j][mt][2], z[j][mt][3]);
        lds_st2(Xn + (mt * 16 + fr) * XS + (d ^ ffn_sw(fr)), pk);
      }
    }
    lds_barrier();
    FFN_TL(205);
    // ---- projection y = u . Wp^T (bf16), 256 output columns per K1 steps.
    // Stores go out T per step during the first MT steps of every column
    // block, each right after that step's DMA issue: the out rows in block 0,
    // block nc-1's y rows in block nc (the last block's after the loop).  A
    // tile wait counts the stores younger than its tile, so a store only has
    // to land before the wait two steps on instead of holding the next one
    // (a store counts in vmcnt like the LDS-DMA tiles).  Workgroups with rows
    // past M store unconditionally-counted nothing: their stores come at the
    // block ends / the end and their waits assume none younger.  No reloads
    // past ST-1.
    static_assert(MT <= K1, "stores of a column block fit in its steps");
    const int ncp = a.np / TROWS;
    const bool full = m0 + BM <= a.M;
    uint2 yq[T][MT];  // the previous column block's y (bf16)
    for (int nc = 0; nc < ncp; ++nc) {
#pragma unroll
      for (int r = 0; r < K1; ++r) {
        const int s = SF + nc * K1 + r;
        // stores of the two steps before (k(x) = T if step x stored)
        const int kprev1 = (r >= 1 ? (r - 1 < MT) : (K1 - 1 < MT)) ? T : 0;
        const int kprev2 = (r >= 2 ? (r - 2 < MT) : (K1 + r - 2 < MT)) ? T : 0;
        const int k1 = (r >= 1 || nc > 0) ? kprev1 : 0, k2 = (r >= 2 || nc > 0) ? kprev2 : 0;
        vm_wait((s + 1 < ST ? GL : 0) + (full ? k1 + k2 : 0));
        const bf16_t* tile = ring + (s % NB) * TROWS * BK;
        // fragment offsets from an opaque lane id (hoisted, they spill)
        int ln;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
        const int lfr = ln & 15, lg = ln >> 4;
        bf16x8 fw[BK / 32][T];
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks)
#pragma unroll
          for (int t = 0; t < T; ++t) {
            const int row = w * (T * 16) + t * 16 + lfr;
            fw[ks][t] = ld8(tile + row * BK + (((ks * 4 + lg) ^ ((row >> 1) & 7)) << 3));
          }
        // the A operand from Xn each step (not held in VGPRs here: the
        // registers go to the deferred stores instead)
        bf16x8 fx[BK / 32][MT];
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const uint32_t la = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) bf16_t*)(
                Xn + (mt * 16 + fr) * XS + r * BK + ks * 32 + fk));
            asm volatile("ds_read_b128 %0, %1" : "=v"(fx[ks][mt]) : "v"(la) : "memory");
          }
        f32x4 ov[T];
        if (r < MT && full && nc == 0) {
#pragma unroll
          for (int j = 0; j < T; ++j) ov[j] = lds_f4(Zo + (r * 16 + lfr) * ZS + (w * T + j) * 16 + 4 * lg);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (s + NB < ST) issue(s + NB, s % NB);
        asm volatile("" ::: "memory");  // the stores stay behind the DMA issue (the counts above)
        if (r < MT && full) {
          const long long row = m0 + r * 16 + lfr;
          if (nc == 0) {
#pragma unroll
            for (int j = 0; j < T; ++j)
              *reinterpret_cast<f32x4*>(a.out + row * D + (w * T + j) * 16 + 4 * lg) = ov[j];
          } else {
#pragma unroll
            for (int t = 0; t < T; ++t)
              *reinterpret_cast<uint2*>(a.yp + row * a.np + (nc - 1) * TROWS + w * (T * 16) + t * 16 + 4 * lg) = yq[t][r];
          }
        }
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks)
#pragma unroll
          for (int t = 0; t < T; ++t)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
              acc1[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[ks][t], fx[ks][mt], acc1[t][mt], 0, 0, 0);
      }
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const f32x4 v = acc1[t][mt];
          yq[t][mt].x = pack_bf16x2(v[0], v[1]);
          yq[t][mt].y = pack_bf16x2(v[2], v[3]);
          acc1[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
          const int row = m0 + mt * 16 + (ln & 15);
          if ((!full || nc == ncp - 1) && row < a.M)
            *reinterpret_cast<uint2*>(a.yp + (long long)row * a.np + nc * TROWS + w * (T * 16) + t * 16 + 4 * (ln >> 4)) =
                yq[t][mt];
        }
    }
    FFN_TL(206);
    if (!full) {
      f32x4 ov[T][MT];
#pragma unroll
      for (int j = 0; j < T; ++j)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) ov[j][mt] = lds_f4(Zo + (mt * 16 + fr) * ZS + (w * T + j) * 16 + 4 * g);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int j = 0; j < T; ++j)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int row = m0 + mt * 16 + fr;
          if (row < a.M) *reinterpret_cast<f32x4*>(a.out + (long long)row * D + (w * T + j) * 16 + 4 * g) = ov[j][mt];
        }
    }
    SBK_PROBE(asm volatile("s_waitcnt vmcnt(0)" ::: "memory");)  // the end mark includes the store drain
    FFN_TL(196);
    return;
  }
  // all residual reads of x are done before out (which may alias x) is written
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const int d = (w * T + j) * 16 + 4 * g;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int row = m0 + mt * 16 + fr;
      if (row < a.M)
        *reinterpret_cast<float4*>(a.out + (long long)row * D + d) =
            make_float4(z[j][mt][0], z[j][mt][1], z[j][mt][2], z[j][mt][3]);
    }
  }
  if (a.gn) {
    row_ln<D, T, MT, NW>(z, red, prm + P_GN * D, prm + P_BN * D, a.epsn, w, g, fr, a.inv_n, a.npad);
#pragma unroll
    for (int j = 0; j < T; ++j) {
      const int d = (w * T + j) * 16 + 4 * g;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int row = m0 + mt * 16 + fr;
        if (row >= a.M) continue;
        if (a.u_bf16) {
          uint2 pk;
          pk.x = pack_bf16x2(z[j][mt][0], z[j][mt][1]);
          pk.y = pack_bf16x2(z[j][mt][2], z[j][mt][3]);
          *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(a.u) + (long long)row * D + d) = pk;
        } else {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.u) + (long long)row * D + d) =
              make_float4(z[j][mt][0], z[j][mt][1], z[j][mt][2], z[j][mt][3]);
        }
      }
    }
  }
  FFN_TL(196);
}

template <int D>
size_t ffn_lds(int H, bool chain) {
  // 2-slot weight ring, Xn, two hidden-chunk buffers, b1 (two with CHAIN), the row-reduction scratch,
  // the epilogue parameter rows
  return ((size_t)2 * 256 * 64 + (size_t)FFN_BM * (D + FFN_PAD) + (size_t)2 * FFN_BM * (256 + FFN_PAD)) *
             sizeof(bf16_t) +
         (size_t)(chain ? 2 : 1) * H * 4 + (size_t)FFN_RS * FFN_BM * 4 + (size_t)FFN_NW * D * 4;
}

template <int D, int ACT, bool PROJ, bool CHAIN>
int launch_ffn_act(const FfnArgs& a, size_t lds, hipStream_t s) {
  // > 64 KB dynamic LDS: opted in per device, raised when a launch (a larger H) needs more
  if (hipError_t e = sbk::lds_optin(reinterpret_cast<const void*>(&ffn_kernel<D, ACT, PROJ, CHAIN>), lds))
    return (int)e;
  hipLaunchKernelGGL((ffn_kernel<D, ACT, PROJ, CHAIN>), dim3((a.M + FFN_BM - 1) / FFN_BM), dim3(FFN_NT), lds, s, a);
  return 0;
}

template <int D, bool PROJ, bool CHAIN>
int launch_ffn(const FfnArgs& a, hipStream_t s) {
  const size_t lds = ffn_lds<D>(a.H, CHAIN);
  if (lds > 160 * 1024) return SBK_ERR_ARG;
  switch (a.act) {
    case ACT_SWISH: return launch_ffn_act<D, ACT_SWISH, PROJ, CHAIN>(a, lds, s);
    case ACT_LRELU: return launch_ffn_act<D, ACT_LRELU, PROJ, CHAIN>(a, lds, s);
    case ACT_GELU: return launch_ffn_act<D, ACT_GELU, PROJ, CHAIN>(a, lds, s);
    case ACT_NONE: return launch_ffn_act<D, ACT_NONE, PROJ, CHAIN>(a, lds, s);
    default: return SBK_ERR_ARG;
  }
}

int ffn_dispatch(const FfnArgs& a, hipStream_t s) {
  const bool proj = a.np > 0, chain = a.g0b != nullptr;
  if (chain) return proj ? launch_ffn<256, true, true>(a, s) : launch_ffn<256, false, true>(a, s);
  return proj ? launch_ffn<256, true, false>(a, s) : launch_ffn<256, false, false>(a, s);
}

// ---- the weight-stream image.  Tile s (256 rows x 64 k, 32 KB) in the order
// ffn_kernel streams them: per FFN block (A, then B for a chain) and hidden
// chunk c of 256 units: K1 = D / 64 tiles of W1 rows c*256.. (k over D), then
// 4 tiles of W2 (all D rows, k over the chunk's units); then the projection:
// per 256 output columns nc, K1 tiles of Wp rows nc*256.. .  Row r of a tile
// holds its 8 chunks of 8 k in the order j' -> source chunk j' ^ ((r >> 1) & 7)
// (the ring's bank swizzle, applied here once instead of on every load).
struct ImgSrc {
  const bf16_t *w1, *w2, *w1b, *w2b, *wp;
  int D, H, ntile_blk, ntile_ffn, chain;
};

__device__ __forceinline__ void img_tile_src(const ImgSrc& q, int s, const bf16_t** mat, int* ld, int* row0,
                                             int* k0) {
  const int K1 = q.D / 64, SPC = K1 + 4;
  if (s >= q.ntile_ffn) {  // projection
    const int pj = s - q.ntile_ffn, nc = pj / K1, r = pj - nc * K1;
    *mat = q.wp; *ld = q.D; *row0 = nc * 256; *k0 = r * 64;
    return;
  }
  const bool sb = s >= q.ntile_blk;
  const int sl = sb ? s - q.ntile_blk : s, c = sl / SPC, r = sl - c * SPC;
  if (r < K1) {
    *mat = sb ? q.w1b : q.w1; *ld = q.D; *row0 = c * 256; *k0 = r * 64;
  } else {
    *mat = sb ? q.w2b : q.w2; *ld = q.H; *row0 = 0; *k0 = c * 256 + (r - K1) * 64;
  }
}

__global__ void __launch_bounds__(256) ffn_image_kernel(ImgSrc q, int ntile, bf16_t* __restrict__ img) {
  const long long n = (long long)ntile * 256 * 8;  // 16-B chunks
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int s = (int)(i >> 11), rem = (int)(i & 2047), r = rem >> 3, jp = rem & 7;
    const bf16_t* mat;
    int ld, row0, k0;
    img_tile_src(q, s, &mat, &ld, &row0, &k0);
    const int j = jp ^ ((r >> 1) & 7);
    *reinterpret_cast<uint4*>(img + i * 8) =
        *reinterpret_cast<const uint4*>(mat + (long long)(row0 + r) * ld + k0 + 8 * j);
  }
}

int ffn_tiles(int D, int H, int np, int chain) {
  const int per_blk = (H / 256) * (D / 64 + 4);
  return (chain ? 2 : 1) * per_blk + (np / 256) * (D / 64);
}

}  // namespace

SBK_PROBE_EXPORT(sbk_probe_ffn_tl, g_ffn_tl)

SBK_API int sbk_ffn_supported(int D, int H) { return D == 256 && H > 0 && H % 256 == 0 && H <= 2048; }

SBK_API long long sbk_ffn_image_elems(int D, int H, int np, int chain) {
  if (!sbk_ffn_supported(D, H) || np < 0 || np % 256) return -1;
  return (long long)ffn_tiles(D, H, np, chain) * 256 * 64;
}

SBK_API int sbk_ffn_image(const void* w1, const void* w2, const void* w1b, const void* w2b, const void* wp, int D,
                          int H, int np, void* img, void* stream) {
  const int chain = w1b != nullptr;
  if (!sbk_ffn_supported(D, H) || !w1 || !w2 || !img || (chain && !w2b) || np < 0 || np % 256 || (np > 0) != (wp != nullptr))
    return SBK_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(w1) | reinterpret_cast<uintptr_t>(w2) | reinterpret_cast<uintptr_t>(w1b) |
       reinterpret_cast<uintptr_t>(w2b) | reinterpret_cast<uintptr_t>(wp) | reinterpret_cast<uintptr_t>(img)) & 15)
    return SBK_ERR_ARG;
  ImgSrc q;
  q.w1 = reinterpret_cast<const bf16_t*>(w1); q.w2 = reinterpret_cast<const bf16_t*>(w2);
  q.w1b = reinterpret_cast<const bf16_t*>(w1b); q.w2b = reinterpret_cast<const bf16_t*>(w2b);
  q.wp = reinterpret_cast<const bf16_t*>(wp);
  q.D = D; q.H = H; q.chain = chain;
  q.ntile_blk = (H / 256) * (D / 64 + 4);
  q.ntile_ffn = (chain ? 2 : 1) * q.ntile_blk;
  const int nt = ffn_tiles(D, H, np, chain);
  const long long chunks = (long long)nt * 2048;
  hipLaunchKernelGGL(ffn_image_kernel, dim3((unsigned)std::min<long long>((chunks + 255) / 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, q, nt, reinterpret_cast<bf16_t*>(img));
  SBK_CHECK_LAUNCH();
  return 0;
}

namespace {
int ffn_check(const float* x, int M, int D, int H, const float* g0, const float* b0, const void* img,
              long long img_elems, int chain, const float* b1, int act, const float* b2, const float* gp,
              const float* bp, float* out, const float* gn, const float* bn, void* u, int np, void* yp) {
  if (M <= 0 || !sbk_ffn_supported(D, H) || !g0 || !b0 || !img || !b1 || !b2 || !out) return SBK_ERR_ARG;
  // the image must be the one sbk_ffn_image built for this (D, H, np, chain):
  // the kernel streams exactly that many tiles from it
  if (np < 0 || np % 256 || img_elems != sbk_ffn_image_elems(D, H, np, chain)) return SBK_ERR_ARG;
  if (act == ACT_GLU || act < 0 || act > ACT_GELU || (gn && !u && np == 0)) return SBK_ERR_ARG;
  // projection tail: y = next-LN(out) . Wp^T, whole 256-column blocks; it
  // replaces the u output
  if (np < 0 || np % 256 || (np > 0 && (!gn || !bn || u || !yp))) return SBK_ERR_ARG;
  // float4 loads of rows and LayerNorm parameters, 16-B image pieces
  const uintptr_t al = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(g0) |
                       reinterpret_cast<uintptr_t>(b0) | reinterpret_cast<uintptr_t>(b1) |
                       reinterpret_cast<uintptr_t>(b2) | reinterpret_cast<uintptr_t>(gp) |
                       reinterpret_cast<uintptr_t>(bp) | reinterpret_cast<uintptr_t>(out) |
                       reinterpret_cast<uintptr_t>(gn) | reinterpret_cast<uintptr_t>(bn) |
                       reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(img) | reinterpret_cast<uintptr_t>(yp);
  return (al & 15) ? SBK_ERR_ARG : 0;
}
}  // namespace

SBK_API int sbk_ffn_proj(const float* x, int M, int D, int d_eff, int H, const float* g0, const float* b0, float eps0,
                         const void* img, long long img_elems, const float* b1, int act, float slope, const float* b2,
                         float alpha, const float* gp, const float* bp, float epsp, float* out, const float* gn,
                         const float* bn, float epsn, void* u, int u_bf16, int np, void* yp, void* stream) {
  if (ffn_check(x, M, D, H, g0, b0, img, img_elems, 0, b1, act, b2, gp, bp, out, gn, bn, u, np, yp) || d_eff <= 0 ||
      d_eff > D)
    return SBK_ERR_ARG;
  FfnArgs a;
  a.inv_n = 1.0f / (float)d_eff; a.npad = (float)(D - d_eff);
  a.x = x; a.M = M; a.H = H;
  a.g0 = g0; a.b0 = b0; a.eps0 = eps0;
  a.img = reinterpret_cast<const bf16_t*>(img); a.b1 = b1; a.act = act; a.slope = slope;
  a.b2 = b2; a.alpha = alpha;
  a.gp = gp; a.bp = bp; a.epsp = epsp;
  a.out = out;
  a.gn = gn; a.bn = bn; a.epsn = epsn; a.u = u; a.u_bf16 = u_bf16;
  a.np = np; a.yp = reinterpret_cast<bf16_t*>(yp);
  a.g0b = nullptr; a.b0b = nullptr; a.eps0b = 0.f; a.b1b = nullptr; a.b2b = nullptr; a.alphab = 0.f;
  const int rc = ffn_dispatch(a, (hipStream_t)stream);
  if (rc) return rc;
  SBK_CHECK_LAUNCH();
  return 0;
}

// Two consecutive FFN blocks in one launch (the second on the first's
// output, which never leaves the CU): block A (g0 .. gp: e.g. FFN2 + norm2 of
// Conformer layer i) then block B (g0b .. alphab: FFN1 of layer i+1, no
// post-LN), then next-LN / projection tail as sbk_ffn_proj.  out receives
// block B's output only.  img: sbk_ffn_image of (w1, w2, w1b, w2b, wp).
SBK_API int sbk_ffn_chain(const float* x, int M, int D, int d_eff, int H, int act, float slope, const float* g0,
                          const float* b0,
                          float eps0, const float* b1, const float* b2, float alpha, const float* gp, const float* bp,
                          float epsp, const float* g0b, const float* b0b, float eps0b, const float* b1b,
                          const float* b2b, float alphab, float* out, const float* gn, const float* bn, float epsn,
                          void* u, int u_bf16, const void* img, long long img_elems, int np, void* yp,
                          void* stream) {
  if (!g0b || !b0b || !b1b || !b2b) return SBK_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(g0b) | reinterpret_cast<uintptr_t>(b0b) | reinterpret_cast<uintptr_t>(b1b) |
       reinterpret_cast<uintptr_t>(b2b)) & 15)
    return SBK_ERR_ARG;
  if (ffn_check(x, M, D, H, g0, b0, img, img_elems, 1, b1, act, b2, gp, bp, out, gn, bn, u, np, yp) || d_eff <= 0 ||
      d_eff > D)
    return SBK_ERR_ARG;
  FfnArgs a;
  a.inv_n = 1.0f / (float)d_eff; a.npad = (float)(D - d_eff);
  a.x = x; a.M = M; a.H = H;
  a.g0 = g0; a.b0 = b0; a.eps0 = eps0;
  a.img = reinterpret_cast<const bf16_t*>(img); a.b1 = b1; a.act = act; a.slope = slope;
  a.b2 = b2; a.alpha = alpha;
  a.gp = gp; a.bp = bp; a.epsp = epsp;
  a.out = out;
  a.gn = gn; a.bn = bn; a.epsn = epsn; a.u = u; a.u_bf16 = u_bf16;
  a.np = np; a.yp = reinterpret_cast<bf16_t*>(yp);
  a.g0b = g0b; a.b0b = b0b; a.eps0b = eps0b;
  a.b1b = b1b; a.b2b = b2b; a.alphab = alphab;
  const int rc = ffn_dispatch(a, (hipStream_t)stream);
  if (rc) return rc;
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_ffn(const float* x, int M, int D, int d_eff, int H, const float* g0, const float* b0, float eps0,
                    const void* img, long long img_elems, const float* b1, int act, float slope, const float* b2,
                    float alpha, const float* gp, const float* bp, float epsp, float* out, const float* gn,
                    const float* bn, float epsn, void* u, int u_bf16, void* stream) {
  return sbk_ffn_proj(x, M, D, d_eff, H, g0, b0, eps0, img, img_elems, b1, act, slope, b2, alpha, gp, bp, epsp, out, gn, bn,
                      epsn, u, u_bf16, 0, nullptr, stream);
}
