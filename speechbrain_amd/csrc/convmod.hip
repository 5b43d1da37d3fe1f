// Fused Conformer convolution module (bf16 MFMA), one launch per layer:
//
//   u   = LN0(x)                                   (ConvolutionModule.layer_norm)
//   g   = GLU(u · W1^T + b1)                       (bottleneck: 1x1 Conv1d d->2d + GLU)
//   c   = depthwise_conv_k(g) + bc                 (conv, zero padding, causal or centred)
//   v   = Swish(LN1(c))                            (after_conv[0..1])
//   out = x + rowmask0(v · W2^T + b2)              (after_conv[2], masked_fill_, residual)
//
// Reference: speechbrain/lobes/models/transformer/Conformer.py:54-115
// (ConvolutionModule) and :254-255 (x + convolution_module(x, conv_mask)).
//
// Design (MI355X): a workgroup (16 waves) owns CM_BM = 48 consecutive frames
// of ONE utterance; B * ceil(T / 48) = 256 workgroups at B = 32, T = 376 —
// one per CU.  The k - 1 halo frames the depthwise conv needs are recomputed
// through LN0 and the GLU GEMM (78 rows for 48 outputs), so no intermediate
// leaves the CU: u, g and v live in LDS (u and v share a buffer), x is read
// once (plus the halo) and out written once.  This replaces four launches
// (LN, GLU GEMM, dwconv+LN+Swish, projection GEMM) and the HBM round trips of
// g and v.
//   phase 0: x rows (78) -> LN0 -> bf16 U (LDS); rows outside [0, T) -> 0
//   phase 1: G = GLU(U W1p^T + b1p): wave w owns permuted weight rows
//            32w .. 32w+31 = GLU group w, so value and gate of a channel land
//            in the same lane; frames outside [0, T) -> 0
//            (the conv's zero padding)
//   phase 2: thread (channel c, quarter h) slides a 31-tap register window
//            down G for 12 frames into an fp32 LDS tile; then one wave per frame:
//            LN1 over the channels (4 per lane), Swish -> bf16 V (LDS, over U)
//            (per-frame wave sums in the conv's thread map cost 34 us: 48
//            dependent cross-lane reductions per wave)
//   phase 3: Y = V W2^T (wave w: 16 output units x 48 frames) + b2, row mask,
//            + x (fp32), float4 stores
// Phase -1's out_proj fragments are loaded straight from global (L2-resident)
// into VGPRs up front; the phase-1 (256 KB) and phase-3 (128 KB) weights
// stream L2 -> LDS by LDS-DMA through a 4-slot ring of 16-row x 32-k pieces
// (one per wave and slice, each wave staging only the rows it multiplies)
// in the buffers the phase does not use, three slices in flight.
// Round 3 (s_memtime, profiles/r03_convmod_pre_timeline.log): 67k -> 55k
// cycles per workgroup, 33.4 -> 28.5 us per launch.  Phase 1 went 17k ->
// 11.5k (the register prefetch one K-step ahead waited on L2 latency every
// step); phase 3 8-10k -> 3-5k (its bias / key-mask bytes now load ahead of
// the ring instead of after it); the bf16-output sigmoids use the hardware
// reciprocal (an IEEE divide per element before, and the GLU's branches).
// What remains: phase -1 (all 251 workgroups pull 120 KB of o / x rows —
// 1.67x the output rows for the conv halo — plus 128 KB of out_proj weights
// at once: ~15k cycles to the last wave's data) and phase 1 at ~22 B/clk of
// weights with every wave re-reading all 80 U rows from LDS (LDS bound:
// 144 KB of LDS traffic per K-slice).
#include "mfma.h"

using namespace sbk;

namespace {

constexpr int CM_D = 256;          // d_model (channels)
constexpr int CM_BM = 48;          // output frames per workgroup
constexpr int CM_KMAX = 31;        // max depthwise taps
constexpr int CM_ROWS = 80;        // staged frames (BM + K - 1 <= 78, padded to 5 m-tiles)
constexpr int CM_MT1 = CM_ROWS / 16;
constexpr int CM_MT3 = CM_BM / 16;
constexpr int CM_NW = 16, CM_NT = CM_NW * 64;
constexpr int CM_S = CM_D + 16;    // LDS row stride (elements): conflict-free b128 fragment reads
// U / G rows: element (row, col) at row * CM_S + (col ^ cm_sw(row)), the 16-B
// chunks of rows with bit 2 set swapped in pairs.  The 8-B column stores of
// the GLU epilogue and LN0 (16 rows fr of one column per lane group) were
// 4-way conflicted at a 544-B pitch (rows fr, fr + 4, fr + 8, fr + 12 on one
// bank pair) and are 2-way with it — 2-way is the floor for 16-B-aligned
// rows; the fragment reads stay conflict-free.
__device__ __forceinline__ constexpr int cm_sw(int row) { return ((row >> 2) & 1) << 3; }
static_assert(CM_NW % 8 == 0, "rows w + CM_NW * i share bit 2 with w (their swizzle is cm_sw(w))");

struct ConvModArgs {
  const float* x;  // (B*T, D) fp32 residual stream
  float* out;      // (B*T, D) fp32 (must not alias x: neighbours read the halo)
  int B, T, K, padL;
  const float *g0, *b0;
  float eps0;
  const bf16_t* w1;  // (2D, D) GLU-permuted [value16 | gate16] row groups
  const float* b1;   // (2D) permuted like w1
  const float* wc;   // (K, D) depthwise taps, tap-major (host-transposed once)
  const float* bc;   // (D) or null
  const float *g1, *b1n;
  float eps1;
  const bf16_t* w2;  // (D, D)
  const float* b2;   // (D) or null
  const uint8_t* kpm;  // (B*T) padding mask or null
  // optional attention output projection applied first (PRE): the module's
  // input is x + o · wo^T + bo (attention.py:636 and the MHSA residual,
  // Conformer.py:247-252), never materialised outside the workgroup
  const bf16_t* o;   // (B*T, D) attention output (heads concatenated)
  const bf16_t* wo;  // (D, D) out_proj weight
  const float* bo;   // (D) or null
  // LayerNorm statistics over the first d_eff channels (the rest zero-padded,
  // as in ffn.hip): inv_n = 1 / d_eff, npad = D - d_eff
  float inv_n, npad;
};

// s_memtime phase marks of the waves of workgroup 100 (probe builds only)
SBK_PROBE_BUFFER(g_cm_tl, 16, 8)
#define CM_TL(i) \
  SBK_PROBE(if (blockIdx.x == 100 && (threadIdx.x & 63) == 0) g_cm_tl[threadIdx.x >> 6][i] = __builtin_amdgcn_s_memtime();)

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations, not for its outstanding global loads (a __syncthreads() fence
// would drain the weight / residual loads issued ahead of their phase).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ bf16x8 ld8g(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// Weight streams (phases 1 and 3) go L2 -> LDS by LDS-DMA pieces (64 lanes x
// 16 B) issued from inline asm: the compiler sees no LDS write in flight (no
// alias-guard waits on the LDS reads) and the ring waits are explicit
// counted vmcnt.  A wave stages exactly the weight rows it multiplies, so a
// slot needs no workgroup barrier.  A row of a K-slice is 32 bf16 = 64 B, its
// four 16-B chunks XOR-swizzled by cm_q((row >> 2) & 3): the 16 lanes of
// each ds_read_b128 lane group (MI355X_MICROARCH §LDS: lanes {0-3, 12-15,
// 20-27}, {4-11, 16-19, 28-31}, ... — rows fr of chunk g and of chunk g ^ 1)
// then cover all 64 banks.  (The former (row >> 2) & 3 assumed 16 contiguous
// lanes: 2-way conflicts on every fragment read, 96 of the 226 conflict
// cycles per wave that SQ_LDS_BANK_CONFLICT counted.)
// (m0 is a reserved register: the clobber is advisory.  This kernel has no
// other m0 user — every m0 write in its ISA is this one — so nothing the
// compiler keeps in m0 can be overwritten.)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void cm_dma(const bf16_t* src, bf16_t* lds) {
  const uint32_t la = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) bf16_t*)lds));
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(la) : "memory", "m0");
}
#pragma clang diagnostic pop
// 16 rows of a row-major (., CM_D) bf16 weight (src: the first row at k0), k0 ..
// k0 + 31, into 16 slot rows of 64 B at dst (one piece)
// row quad q -> chunk XOR 0, 2, 3, 1: quads {0, 3} of chunk g and {1, 2} of
// chunk g ^ 1 (one lane group) land on four distinct chunks
__device__ __forceinline__ int cm_q(int q) { return ((((q ^ (q >> 1)) & 1) << 1) | (q >> 1)) & 3; }
__device__ __forceinline__ void cm_dma16(const bf16_t* src, bf16_t* dst, int lane) {
  const int r = lane >> 2, lc = (lane & 3) ^ cm_q((r >> 2) & 3);
  cm_dma(src + (long long)r * CM_D + 8 * lc, dst);
}
// fragment of slot row `row`, logical chunk g (8 consecutive k)
__device__ __forceinline__ bf16x8 cm_frag(const bf16_t* slot, int row, int g) {
  return *reinterpret_cast<const bf16x8*>(slot + row * 32 + 8 * (g ^ cm_q((row >> 2) & 3)));
}
// s_waitcnt vmcnt(n), n = 0, 1, 2 known only at run time (wave-uniform)
__device__ __forceinline__ void cm_vmwait(int n) {
  if (n >= 2)
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (n == 1)
    asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// global load the compiler cannot see (so its first use gets no vmcnt(0)
// behind the DMA pieces issued after it); the caller waits (asm) and ties
__device__ __forceinline__ f32x4 cm_gld4(const float* p) {
  f32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void cm_tie(f32x4& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ int cm_gldu8(const uint8_t* p) {
  int v;
  asm volatile("global_load_ubyte %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

template <bool PRE>
__global__ void __launch_bounds__(CM_NT) conv_module_kernel(ConvModArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* Us = reinterpret_cast<bf16_t*>(smem);  // CM_ROWS x CM_S (U, later V)
  bf16_t* Gs = Us + CM_ROWS * CM_S;              // CM_ROWS x CM_S
  float* Cv = reinterpret_cast<float*>(Gs + CM_ROWS * CM_S);  // CM_BM x CM_D fp32 conv output

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, g = lane >> 4, fk = 8 * g;
  const int fks = fk ^ cm_sw(fr);  // fk in the swizzled U / G rows mt*16 + fr
  const int nblk = (a.T + CM_BM - 1) / CM_BM;
  // (an XCD-aware remap that put an utterance's consecutive tiles — which
  // share halo rows — on one XCD measured equal: 30.4-30.5 vs 30.4-30.8 us,
  // profiles/r04m_conv_xcd.log)
  const int tile = blockIdx.x;
  const int b = tile / nblk, t0 = (tile % nblk) * CM_BM;
  const int f0 = t0 - a.padL;  // frame of staged row 0
  const int nrows = CM_BM + a.K - 1;
  const long long ubase = (long long)b * a.T;
  CM_TL(0);
  // first K-step of the phase-1 weights and of the phase-3 weights and the
  // residual rows are issued up front: their latency overlaps phases 0-2
  constexpr int T1 = 2;                  // phase-1 tiles per wave: (value, gate) of GLU group w
  constexpr int T3 = CM_D / 16 / CM_NW;  // phase-3 output tiles per wave (1)
  // Weight rings.  A slot holds one 16-row x 32-k piece per wave (16 KB).
  // Phase 1 streams 16 slices (8 K-slices x the value / gate tile) through
  // four slots — two in Gs, two in the front of Cv, all free while the GLU
  // GEMM runs — three slices in flight; phase 3 streams 8 K-slices through
  // the same four (Gs is free after phase 2a, Cv after phase 2b).
  constexpr int KSL = CM_D / 32, P1S = KSL * T1, SLOT = CM_NW * 16 * 32;
  bf16_t* p1slot[4] = {Gs, Gs + SLOT, reinterpret_cast<bf16_t*>(Cv), reinterpret_cast<bf16_t*>(Cv) + SLOT};
  bf16_t* const* p3slot = p1slot;  // Gs slots from phase 2b on, the Cv ones from phase 3 on
  static_assert(2 * SLOT * 2 <= CM_ROWS * CM_S * 2 && 2 * SLOT * 2 <= CM_BM * CM_D * 4, "ring slots fit");
  auto issue_p1 = [&](int q) __attribute__((always_inline)) {  // slice q: K-slice q / 2, tile q % 2
    cm_dma16(a.w1 + (long long)(w * 32 + 16 * (q & 1)) * CM_D + 32 * (q >> 1), p1slot[q & 3] + w * 16 * 32, lane);
  };
  auto issue_p3 = [&](int ks) __attribute__((always_inline)) {
    cm_dma16(a.w2 + (long long)(w * 16) * CM_D + 32 * ks, p3slot[ks & 3] + w * 16 * 32, lane);
  };

  // PRE: x_att of this lane's phase-3 outputs (units w*16 + 4g .., frames
  // t0 + mt*16 + fr), moved across lanes from phase -1's staged-row layout
  float4 xres[CM_MT3];
  if constexpr (PRE) {
    // ---- phase -1: x_att = x + o wo^T + bo over the staged frames, LN0 -> U
    // every load first (o rows, x rows, wo fragments), then o rows -> Gs
    // (free until phase 1); frames outside [0, T) stage zeros
    constexpr int OC = (CM_ROWS * (CM_D / 8) + CM_NT - 1) / CM_NT;  // 16-B o chunks per thread
    uint4 ov[OC];
#pragma unroll
    for (int i = 0; i < OC; ++i) {
      const int c = min(tid + i * CM_NT, CM_ROWS * (CM_D / 8) - 1);
      const int r = c / (CM_D / 8), ch = c - r * (CM_D / 8);
      const int fc = min(max(f0 + r, 0), a.T - 1);
      ov[i] = *reinterpret_cast<const uint4*>(a.o + (ubase + fc) * CM_D + ch * 8);
    }
    // LN0 affine -> LDS (threads < 128, one float4 each; read after LN0's barrier)
    // LN0's scratch (partials, statistics, affine) sits past the phase-1
    // ring slot that Cv also holds, so that slot can fill during LN0
    float* lnscr = Cv + CM_NW * 32 * 32 / 2;  // 32 KB in (bf16 slot -> float offset)
    static_assert(CM_NW * 32 * 32 / 2 + 2 * CM_ROWS * (CM_NW + 4) + 2 * CM_ROWS + 2 * CM_D <= CM_BM * CM_D,
                  "LN0 scratch fits beside the ring slot");
    float* gb0s = lnscr + 2 * CM_ROWS * (CM_NW + 4) + 2 * CM_ROWS;  // [g0 | b0], past LN0's partials / statistics
    const float4 gbv = tid < CM_D / 2 ? *reinterpret_cast<const float4*>((tid < CM_D / 4 ? a.g0 : a.b0) +
                                                                         4 * (tid % (CM_D / 4)))
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
    // wave w: units w*16 .. +15 (one tile) of all CM_MT1 frame tiles;
    // D[unit 4g + e][frame mt*16 + fr]
    const int u0 = w * 16 + 4 * g;
    float4 xv[CM_MT1];
#pragma unroll
    for (int mt = 0; mt < CM_MT1; ++mt) {
      const int f = min(max(f0 + mt * 16 + fr, 0), a.T - 1);
      xv[mt] = *reinterpret_cast<const float4*>(a.x + (ubase + f) * CM_D + u0);
    }
    const float4 bo4 = a.bo ? *reinterpret_cast<const float4*>(a.bo + u0) : make_float4(0.f, 0.f, 0.f, 0.f);
    // the wo fragments issued with the row loads (L2: their latency overlaps
    // the HBM rows' instead of following the o staging)
    const bf16_t* wrowo = a.wo + (long long)(w * 16 + fr) * CM_D + fk;
    bf16x8 fwo[CM_D / 32];
#pragma unroll
    for (int kk = 0; kk < CM_D / 32; ++kk) fwo[kk] = ld8g(wrowo + kk * 32);
#pragma unroll
    for (int i = 0; i < OC; ++i) {
      const int c = tid + i * CM_NT;
      if (c < CM_ROWS * (CM_D / 8)) {
        const int r = c / (CM_D / 8), ch = c - r * (CM_D / 8), f = f0 + r;
        const bool live = r < nrows && f >= 0 && f < a.T;
        *reinterpret_cast<uint4*>(Gs + r * CM_S + ((ch * 8) ^ cm_sw(r))) = live ? ov[i] : uint4{0u, 0u, 0u, 0u};
      }
    }
    if (tid < CM_D / 2) *reinterpret_cast<float4*>(gb0s + 4 * tid) = gbv;
    CM_TL(6);
    lds_barrier();
    f32x4 acc[CM_MT1];
#pragma unroll
    for (int mt = 0; mt < CM_MT1; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < CM_D / 32; ++kk)
#pragma unroll
      for (int mt = 0; mt < CM_MT1; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            fwo[kk], *reinterpret_cast<const bf16x8*>(Gs + (mt * 16 + fr) * CM_S + kk * 32 + fks), acc[mt], 0, 0, 0);
    float xa[CM_MT1][4];
#pragma unroll
    for (int mt = 0; mt < CM_MT1; ++mt) {
      xa[mt][0] = xv[mt].x + (acc[mt][0] + bo4.x);
      xa[mt][1] = xv[mt].y + (acc[mt][1] + bo4.y);
      xa[mt][2] = xv[mt].z + (acc[mt][2] + bo4.z);
      xa[mt][3] = xv[mt].w + (acc[mt][3] + bo4.w);
    }
    // phase 3's residual: output frame mt*16 + fr is staged row mt*16 + fr +
    // padL, held (same units) by lane (fr + padL) % 16 of tile (mt*16 + fr +
    // padL) / 16: two lane permutes per value and a select
    {
      const int q = a.padL >> 4, rr = a.padL & 15;  // q <= 1 (K <= 31)
      const int src = ((lane & 0x30) + ((fr + rr) & 15)) << 2;
      const bool hi = fr + rr >= 16;
#pragma unroll
      for (int mt = 0; mt < CM_MT3; ++mt) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo_v = q == 0 ? xa[mt][e] : xa[mt + 1][e];
          const float hi_v = q == 0 ? xa[mt + 1][e] : xa[mt + 2][e];
          const float lo = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(lo_v)));
          const float hv = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(hi_v)));
          v[e] = hi ? hv : lo;
        }
        xres[mt] = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    CM_TL(7);
    // LN0 over the 256 units of each frame: 4 per lane, 4 lanes per wave
    // (col4), 16 waves through LDS (Cv: free until phase 2)
    // Sum and sum of squares in one pass (one barrier; var = E[x^2] - mean^2
    // in fp32 on the residual stream), the affine from LDS.
    // Partials laid out [row][wave] (+4 pad) so a row's 16 wave partials are
    // four 16-B reads: with [wave][row] every wave issued 160 ds_read_b32
    // here, and the CU's LDS pipe spent ~11k cycles on them.
    constexpr int RS = CM_NW + 4;  // row stride (floats), 16-B aligned
    float* red = lnscr;            // [CM_ROWS][RS] sums, then [CM_ROWS][RS] squares
    float mean[CM_MT1], rstd[CM_MT1];
#pragma unroll
    for (int mt = 0; mt < CM_MT1; ++mt) {
      const float ps = col4_sum((xa[mt][0] + xa[mt][1]) + (xa[mt][2] + xa[mt][3]));
      const float pq = col4_sum((xa[mt][0] * xa[mt][0] + xa[mt][1] * xa[mt][1]) +
                                (xa[mt][2] * xa[mt][2] + xa[mt][3] * xa[mt][3]));
      if (g == 0) {
        red[(mt * 16 + fr) * RS + w] = ps;
        red[CM_ROWS * RS + (mt * 16 + fr) * RS + w] = pq;
      }
    }
    lds_barrier();
    // every wave is past its phase -1 reads of Gs: the phase-1 weight ring's
    // first three slices land (Gs, the free front of Cv) under the statistics
    // exchange and the LN0 application
    issue_p1(0);
    issue_p1(1);
    issue_p1(2);
    // final statistics once per row (lanes of waves 0-1: row = 64 w + lane),
    // not redundantly in all 16 waves: the LN0 phase is VALU-issue bound
    // (4 waves per SIMD), and the 16-way sums were a third of its VALU work
    float* stat = red + 2 * CM_ROWS * RS;  // [CM_ROWS] mean, [CM_ROWS] rstd (inside Cv, before gb0s)
    if (w < (CM_ROWS + 63) / 64 && w * 64 + lane < CM_ROWS) {
      const int row = w * 64 + lane;
      float t = 0.f, t2 = 0.f;
#pragma unroll
      for (int k4 = 0; k4 < CM_NW / 4; ++k4) {
        const float4 a4 = *reinterpret_cast<const float4*>(red + row * RS + 4 * k4);
        const float4 q4 = *reinterpret_cast<const float4*>(red + CM_ROWS * RS + row * RS + 4 * k4);
        t += a4.x;
        t += a4.y;
        t += a4.z;
        t += a4.w;
        t2 += q4.x;
        t2 += q4.y;
        t2 += q4.z;
        t2 += q4.w;
      }
      const float mu = t * a.inv_n;  // padded channels are zero: they add nothing to t or t2
      stat[row] = mu;
      stat[CM_ROWS + row] = 1.0f / sqrtf(fmaxf(t2 * a.inv_n - mu * mu, 0.f) + a.eps0);
    }
    lds_barrier();
    const float4 g04 = *reinterpret_cast<const float4*>(gb0s + u0);
    const float4 b04 = *reinterpret_cast<const float4*>(gb0s + CM_D + u0);
#pragma unroll
    for (int mt = 0; mt < CM_MT1; ++mt) {
      mean[mt] = stat[mt * 16 + fr];
      rstd[mt] = stat[CM_ROWS + mt * 16 + fr];
      const int r = mt * 16 + fr, f = f0 + r;
      const bool live = r < nrows && f >= 0 && f < a.T;
      uint2 pk = make_uint2(0u, 0u);
      if (live) {
        pk.x = pack_bf16x2((xa[mt][0] - mean[mt]) * rstd[mt] * g04.x + b04.x, (xa[mt][1] - mean[mt]) * rstd[mt] * g04.y + b04.y);
        pk.y = pack_bf16x2((xa[mt][2] - mean[mt]) * rstd[mt] * g04.z + b04.z, (xa[mt][3] - mean[mt]) * rstd[mt] * g04.w + b04.w);
      }
      *reinterpret_cast<uint2*>(Us + r * CM_S + (u0 ^ cm_sw(fr))) = pk;
    }
  } else {
  // ---- phase 0: LN0 of the staged frames -> U (bf16) ----
  // all of the wave's row loads are issued before the first reduction
  {
    constexpr int RPW = CM_ROWS / CM_NW;  // rows per wave (5)
    const float4 g04 = *reinterpret_cast<const float4*>(a.g0 + lane * 4);
    const float4 b04 = *reinterpret_cast<const float4*>(a.b0 + lane * 4);
    float4 xv[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int r = w + i * CM_NW, f = min(max(f0 + r, 0), a.T - 1);
      xv[i] = *reinterpret_cast<const float4*>(a.x + (ubase + f) * CM_D + lane * 4);
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int r = w + i * CM_NW, f = f0 + r;
      const bool live = r < nrows && f >= 0 && f < a.T;
      const float v[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
      const float mean = wave_sum_v(v[0] + v[1] + v[2] + v[3]) * a.inv_n;
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) q += (v[e] - mean) * (v[e] - mean);
      const float rstd = 1.0f / sqrtf((wave_sum_v(q) - a.npad * mean * mean) * a.inv_n + a.eps0);
      uint2 pk = make_uint2(0u, 0u);
      if (live) {
        pk.x = pack_bf16x2((v[0] - mean) * rstd * g04.x + b04.x, (v[1] - mean) * rstd * g04.y + b04.y);
        pk.y = pack_bf16x2((v[2] - mean) * rstd * g04.z + b04.z, (v[3] - mean) * rstd * g04.w + b04.w);
      }
      *reinterpret_cast<uint2*>(Us + r * CM_S + ((lane * 4) ^ cm_sw(w))) = pk;  // r = w + 16 i
    }
  }
  }
  if constexpr (!PRE) {  // phase 0's loads are consumed: no wait for them lands behind these
    issue_p1(0);
    issue_p1(1);
    issue_p1(2);
  }
  lds_barrier();
  CM_TL(1);

  // ---- phase 1: G = GLU(U W1p^T + b1p) over CM_ROWS frames ----
  {
    f32x4 acc[T1][CM_MT1];
#pragma unroll
    for (int t = 0; t < T1; ++t)
#pragma unroll
      for (int mt = 0; mt < CM_MT1; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 fa[CM_MT1];  // U fragments of the K-slice, shared by its two tiles
#pragma unroll
    for (int q = 0; q < P1S; ++q) {
      const int ks = q >> 1, t = q & 1;
      // this slice landed; the (up to two) slices issued after it stay in flight
      cm_vmwait(P1S - 1 - q < 2 ? P1S - 1 - q : 2);
      const bf16x8 fw = cm_frag(p1slot[q & 3], w * 16 + fr, g);
      if (t == 0) {
#pragma unroll
        for (int mt = 0; mt < CM_MT1; ++mt)
          fa[mt] = *reinterpret_cast<const bf16x8*>(Us + (mt * 16 + fr) * CM_S + ks * 32 + fks);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (q + 3 < P1S) issue_p1(q + 3);  // into the slot of slice q - 1, whose fragment is in VGPRs
#pragma unroll
      for (int mt = 0; mt < CM_MT1; ++mt)
        acc[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw, fa[mt], acc[t][mt], 0, 0, 0);
    }
    lds_barrier();  // every wave's ring reads are done before G overwrites Gs
    // GLU epilogue: lane holds frames mt*16 + fr, units 4g..4g+3 of each
    // tile; tiles (0, 1) = (value, gate) of channel group w
    {
      const int ch = w * 16 + 4 * g;                 // output channels ch .. ch + 3
      const int pa = w * 32 + 4 * g, pg = pa + 16;   // permuted rows of value / gate
      const float4 ba = *reinterpret_cast<const float4*>(a.b1 + pa);
      const float4 bg = *reinterpret_cast<const float4*>(a.b1 + pg);
      const float bav[4] = {ba.x, ba.y, ba.z, ba.w}, bgv[4] = {bg.x, bg.y, bg.z, bg.w};
#pragma unroll
      for (int mt = 0; mt < CM_MT1; ++mt) {
        const int r = mt * 16 + fr, f = f0 + r;
        const bool live = r < nrows && f >= 0 && f < a.T;
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float va = acc[0][mt][e] + bav[e], vg = acc[1][mt][e] + bgv[e];
          // bf16 output: the approximate reciprocal (1 ulp) is far below its rounding
          const float sg = va * __builtin_amdgcn_rcpf(1.0f + __expf(-vg));
          o[e] = live ? sg : 0.f;
        }
        uint2 pk;
        pk.x = pack_bf16x2(o[0], o[1]);
        pk.y = pack_bf16x2(o[2], o[3]);
        *reinterpret_cast<uint2*>(Gs + r * CM_S + (ch ^ cm_sw(fr))) = pk;
      }
    }
  }
  lds_barrier();
  CM_TL(2);

  float4 xr[T3][CM_MT3];
  static_assert(T3 == 1, "phase 3: one 16-unit tile per wave (the units of phase -1)");
#pragma unroll
  for (int t = 0; t < T3; ++t)
#pragma unroll
    for (int mt = 0; mt < CM_MT3; ++mt) {
      const int f = min(t0 + mt * 16 + fr, a.T - 1);
      // the residual: x, or (PRE) x_att from phase -1
      if constexpr (PRE)
        xr[t][mt] = xres[mt];
      else
        xr[t][mt] = *reinterpret_cast<const float4*>(a.x + (ubase + f) * CM_D + w * 16 * T3 + t * 16 + 4 * g);
    }

  // ---- phase 2: depthwise conv (register window) -> fp32 tile; LN1 -> Swish -> V (over U) ----
  {
    // 2a: thread (channel c, quarter h) slides the taps down its channel for
    // 12 frames, two taps per v_dot2c_f32_bf16 (bf16 operands, fp32
    // accumulation: Conv1d under bf16 autocast, which this kernel serves):
    // tap pair j = (2j, 2j+1) against the window pair (g[i+2j], g[i+2j+1]),
    // an even-aligned pair E for even frames i and an odd-aligned one O for
    // odd frames.  (fp32 FMAs, one tap per instruction: 8.5k cycles of the
    // 58k per workgroup, VALU-bound at 4 waves per SIMD.)
    const int c = tid & (CM_D - 1), h = tid >> 8;  // channel, quarter of the frames
    constexpr int NF = CM_BM / (CM_NT / CM_D);
    constexpr int NP = (CM_KMAX + 1) / 2;          // tap pairs (tap 31 is zero)
    float wk[2 * NP];
#pragma unroll
    // unconditional loads (clamped address + select): a guarded load compiled
    // to a branch and a full wait per element, serialising the 31 tap loads
    // and the 43 window reads
    for (int k = 0; k < 2 * NP; ++k) {  // (K, D): coalesced
      const float v = a.wc[min(k, a.K - 1) * CM_D + c];
      wk[k] = k < a.K ? v : 0.f;
    }
    const float bias = a.bc ? a.bc[c] : 0.f;
    static_assert((CM_NT / CM_D) * NF + 2 * NP - 1 <= CM_ROWS, "every window row is staged");
    static_assert(NF % 2 == 0, "frame pairs");
    typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
    bf2 tp[NP], ev[NF / 2 + NP - 1], od[NF / 2 + NP - 1];
    // the tap pairs first (the fp32 taps die here: 128 VGPRs at 4 waves per SIMD)
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      tp[j] = __builtin_bit_cast(bf2, pack_bf16x2(wk[2 * j], wk[2 * j + 1]));
      asm volatile("" : "+v"(tp[j]));
    }
    // row h * NF + k: its swizzle is cm_sw(k) ^ cm_sw(h * NF) (NF = 12: h * NF ≡ 0 or 4 mod 8), so
    // two per-lane column bases and a compile-time choice per row
    static_assert(NF % 4 == 0, "h * NF keeps bits 0-1 of the row");
    const int cx = c ^ cm_sw(h * NF);
    const unsigned short* Gu0 = reinterpret_cast<const unsigned short*>(Gs) + h * NF * CM_S + cx;
    const unsigned short* Gu1 = reinterpret_cast<const unsigned short*>(Gs) + h * NF * CM_S + (cx ^ 8);
    auto gu = [&](int k) __attribute__((always_inline)) { return (uint32_t)(cm_sw(k) ? Gu1 : Gu0)[k * CM_S]; };
    uint32_t g0 = gu(0);
#pragma unroll
    for (int r = 0; r < NF / 2 + NP - 1; ++r) {
      const uint32_t g1 = gu(2 * r + 1), g2 = gu(2 * r + 2);
      ev[r] = __builtin_bit_cast(bf2, g0 | (g1 << 16));
      od[r] = __builtin_bit_cast(bf2, g1 | (g2 << 16));
      g0 = g2;
    }
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      float s = bias;
#pragma unroll
      for (int j = 0; j < NP; ++j) s = __builtin_amdgcn_fdot2_f32_bf16(tp[j], (i & 1) ? od[i / 2 + j] : ev[i / 2 + j], s, false);
      Cv[(h * NF + i) * CM_D + c] = s;
    }
  }
  lds_barrier();
  CM_TL(3);
  f32x4 bb2 = f32x4{0.f, 0.f, 0.f, 0.f};
  int km[CM_MT3] = {};
  {
    // 2b: one wave per frame, 4 channels per lane.  Gs is free: the phase-3
    // weight ring's first two slices land under this phase (the LN1 affine
    // is loaded first and waited for by count, ahead of them)
    f32x4 g14 = cm_gld4(a.g1 + lane * 4), b14 = cm_gld4(a.b1n + lane * 4);
    // and phase 3's epilogue operands (its bias and key-padding bytes), which
    // after the ring would each cost a dependent global round trip
    if (a.b2) bb2 = cm_gld4(a.b2 + w * 16 * T3 + 4 * g);
    if (a.kpm) {
#pragma unroll
      for (int mt = 0; mt < CM_MT3; ++mt) km[mt] = cm_gldu8(a.kpm + ubase + min(t0 + mt * 16 + fr, a.T - 1));
    }
    issue_p3(0);
    issue_p3(1);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    cm_tie(g14);
    cm_tie(b14);
    cm_tie(bb2);
#pragma unroll
    for (int mt = 0; mt < CM_MT3; ++mt) asm volatile("" : "+v"(km[mt]));
    const float gm[4] = {g14[0], g14[1], g14[2], g14[3]}, bt[4] = {b14[0], b14[1], b14[2], b14[3]};
    // the wave's CM_BM / CM_NW frames side by side: their four cross-lane
    // reduction chains interleave instead of running back to back
    constexpr int FPW = CM_BM / CM_NW;
    float v[FPW][4], mean[FPW], rstd[FPW];
#pragma unroll
    for (int u = 0; u < FPW; ++u) {
      const float4 v4 = *reinterpret_cast<const float4*>(Cv + (w + u * CM_NW) * CM_D + lane * 4);
      v[u][0] = v4.x; v[u][1] = v4.y; v[u][2] = v4.z; v[u][3] = v4.w;
    }
#pragma unroll
    for (int u = 0; u < FPW; ++u) mean[u] = wave_sum_v((v[u][0] + v[u][1]) + (v[u][2] + v[u][3])) * a.inv_n;
#pragma unroll
    for (int u = 0; u < FPW; ++u) {
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) q += (v[u][e] - mean[u]) * (v[u][e] - mean[u]);
      rstd[u] = q;
    }
#pragma unroll
    for (int u = 0; u < FPW; ++u)
      rstd[u] = 1.0f / sqrtf((wave_sum_v(rstd[u]) - a.npad * mean[u] * mean[u]) * a.inv_n + a.eps1);
#pragma unroll
    for (int u = 0; u < FPW; ++u) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float z = (v[u][e] - mean[u]) * rstd[u] * gm[e] + bt[e];
        v[u][e] = z * __builtin_amdgcn_rcpf(1.0f + __expf(-z));  // bf16 output (as the GLU above)
      }
      uint2 pk;
      pk.x = pack_bf16x2(v[u][0], v[u][1]);
      pk.y = pack_bf16x2(v[u][2], v[u][3]);
      *reinterpret_cast<uint2*>(Us + (w + u * CM_NW) * CM_S + ((lane * 4) ^ cm_sw(w))) = pk;  // CM_NW % 8 == 0
    }
  }
  lds_barrier();
  CM_TL(4);

  // ---- phase 3: out = x + rowmask0(V W2^T + b2) ----
  {
    f32x4 acc[T3][CM_MT3];
#pragma unroll
    for (int t = 0; t < T3; ++t)
#pragma unroll
      for (int mt = 0; mt < CM_MT3; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    issue_p3(2);  // Cv is free: the LN1 statistics are read
#pragma unroll
    for (int ks = 0; ks < KSL; ++ks) {
      cm_vmwait(KSL - 1 - ks < 2 ? KSL - 1 - ks : 2);  // this slice landed (up to two after it in flight)
      const bf16x8 fw = cm_frag(p3slot[ks & 3], w * 16 + fr, g);
      bf16x8 fa[CM_MT3];
#pragma unroll
      for (int mt = 0; mt < CM_MT3; ++mt)
        fa[mt] = *reinterpret_cast<const bf16x8*>(Us + (mt * 16 + fr) * CM_S + ks * 32 + fks);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (ks + 3 < KSL) issue_p3(ks + 3);
#pragma unroll
      for (int mt = 0; mt < CM_MT3; ++mt)
        acc[0][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw, fa[mt], acc[0][mt], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < T3; ++t) {
      const int d = w * 16 * T3 + t * 16 + 4 * g;
      const f32x4 bb = bb2;
#pragma unroll
      for (int mt = 0; mt < CM_MT3; ++mt) {
        const int f = t0 + mt * 16 + fr;
        if (f >= a.T) continue;
        const bool m = km[mt] != 0;
        const float4 xv = xr[t][mt];
        float4 o;
        o.x = xv.x + (m ? 0.f : acc[t][mt][0] + bb[0]);
        o.y = xv.y + (m ? 0.f : acc[t][mt][1] + bb[1]);
        o.z = xv.z + (m ? 0.f : acc[t][mt][2] + bb[2]);
        o.w = xv.w + (m ? 0.f : acc[t][mt][3] + bb[3]);
        *reinterpret_cast<float4*>(a.out + (ubase + f) * CM_D + d) = o;
      }
    }
  }
  CM_TL(5);
}

constexpr size_t conv_module_lds() {
  return (size_t)2 * CM_ROWS * CM_S * sizeof(bf16_t) + (size_t)CM_BM * CM_D * sizeof(float);
}

}  // namespace

SBK_PROBE_EXPORT(sbk_probe_cm_tl, g_cm_tl)

SBK_API int sbk_conv_module_supported(int D, int K) { return D == CM_D && K >= 1 && K <= CM_KMAX; }

SBK_API int sbk_conv_module_pre(const float* x, const void* o, const void* wo, const float* bo, float* out, int B,
                                int T, int D, int d_eff, const float* ln0_w, const float* ln0_b, float eps0, const void* w1p,
                                const float* b1p, const float* wc, const float* bc, int K, int causal,
                                const float* ln1_w, const float* ln1_b, float eps1, const void* w2, const float* b2,
                                const unsigned char* kpm, void* stream) {
  if (B <= 0 || T <= 0 || !sbk_conv_module_supported(D, K) || !x || !out || x == out || d_eff <= 0 || d_eff > D)
    return SBK_ERR_ARG;
  if (o && (causal ? K - 1 : (K - 1) / 2) > 31) return SBK_ERR_ARG;  // phase -1 lane map: padL < 32
  if (!ln0_w || !ln0_b || !w1p || !b1p || !wc || !ln1_w || !ln1_b || !w2) return SBK_ERR_ARG;
  const uintptr_t al = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out) |
                       reinterpret_cast<uintptr_t>(ln0_w) | reinterpret_cast<uintptr_t>(ln0_b) |
                       reinterpret_cast<uintptr_t>(w1p) | reinterpret_cast<uintptr_t>(b1p) |
                       reinterpret_cast<uintptr_t>(w2) | reinterpret_cast<uintptr_t>(b2);
  if (al & 15) return SBK_ERR_ARG;
  if ((o == nullptr) != (wo == nullptr) ||
      ((reinterpret_cast<uintptr_t>(o) | reinterpret_cast<uintptr_t>(wo) | reinterpret_cast<uintptr_t>(bo)) & 15))
    return SBK_ERR_ARG;
  ConvModArgs a;
  a.x = x; a.out = out; a.B = B; a.T = T; a.K = K; a.padL = causal ? K - 1 : (K - 1) / 2;
  a.g0 = ln0_w; a.b0 = ln0_b; a.eps0 = eps0;
  a.w1 = reinterpret_cast<const bf16_t*>(w1p); a.b1 = b1p;
  a.wc = wc; a.bc = bc;
  a.g1 = ln1_w; a.b1n = ln1_b; a.eps1 = eps1;
  a.w2 = reinterpret_cast<const bf16_t*>(w2); a.b2 = b2;
  a.kpm = reinterpret_cast<const uint8_t*>(kpm);
  a.o = reinterpret_cast<const bf16_t*>(o); a.wo = reinterpret_cast<const bf16_t*>(wo); a.bo = bo;
  a.inv_n = 1.0f / (float)d_eff; a.npad = (float)(D - d_eff);
  const long long grid = (long long)B * ((T + CM_BM - 1) / CM_BM);
  if (grid > 0x7fffffffLL) return SBK_ERR_ARG;
  constexpr size_t lds = conv_module_lds();
  static_assert(lds <= 160 * 1024, "LDS budget");
  for (const void* k : {reinterpret_cast<const void*>(&conv_module_kernel<false>),
                        reinterpret_cast<const void*>(&conv_module_kernel<true>)})
    if (hipError_t e = sbk::lds_optin(k, lds)) return (int)e;
  if (o)
    hipLaunchKernelGGL(conv_module_kernel<true>, dim3((unsigned)grid), dim3(CM_NT), lds, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(conv_module_kernel<false>, dim3((unsigned)grid), dim3(CM_NT), lds, (hipStream_t)stream, a);
  SBK_CHECK_LAUNCH();
  return 0;
}

SBK_API int sbk_conv_module(const float* x, float* out, int B, int T, int D, int d_eff, const float* ln0_w,
                            const float* ln0_b,
                            float eps0, const void* w1p, const float* b1p, const float* wc, const float* bc, int K,
                            int causal, const float* ln1_w, const float* ln1_b, float eps1, const void* w2,
                            const float* b2, const unsigned char* kpm, void* stream) {
  return sbk_conv_module_pre(x, nullptr, nullptr, nullptr, out, B, T, D, d_eff, ln0_w, ln0_b, eps0, w1p, b1p, wc, bc, K,
                             causal, ln1_w, ln1_b, eps1, w2, b2, kpm, stream);
}
