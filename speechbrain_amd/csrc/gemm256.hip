// Large-tile MFMA GEMM: 256 x 256 output per workgroup, the MI355X-native
// main loop for the big regular projections — bf16 (v_mfma_f32_16x16x32_bf16)
// and MXFP8 (block-scaled v_mfma_scale_f32_32x32x64_f8f6f4, e4m3 operands
// with one E8M0 scale per 32 contraction elements).  Config 5's
// TransformerEncoder FFN / attention projections (Transformer.py:376-486,
// attention.py:642-778,823-839) and the wav2vec2 convs as GEMMs.
//
//   C[M, N] = epilogue( A[M, K] · W[N, K]^T ),  K-contiguous operands
//   (nn.Linear [out][in] weights), N % 256 == 0; K % 64 (bf16) or
//   K % 128 (MXFP8) == 0.  Every K-tile is 128 bytes of each row.
//
// Structure (cdna_hip_programming.md §5, the 256² multi-phase template):
//  * 8 waves (2 along M x 4 along N), each owning a 128 x 64 block
//    (128 VGPRs of f32 accumulators).
//  * A K-tile is four 16-KB half-tiles (A rows 0-127 / 128-255, W rows
//    0-127 / 128-255; MXFP8 adds the rows' scale dwords), each a lane-linear
//    LDS image filled by LDS-DMA (global_load_lds_dwordx4, 2 pieces of 1 KB
//    per wave) with the 16-B chunk index XOR-swizzled by (row >> 1) & 7 on
//    the SOURCE address, so both fragment shapes (16 rows x 16 B for bf16,
//    32 rows x 2 x 16 B for MXFP8) read conflict-free.
//  * Two K-tile buffers.  Every K-tile runs as 4 phases, one per 64 x 32
//    quadrant of the wave's block (16 bf16 / 4 MXFP8 MFMAs each), 2 LDS-DMA
//    pieces of the next tiles per phase (schedule at the loop); each phase:
//    reads and DMA -> raw s_barrier -> MFMAs at s_setprio(1) -> s_barrier,
//    with waves 4-7 one barrier behind waves 0-3 (one wave of each group per
//    SIMD: one reads while its partner multiplies).  The DMA is inline asm
//    (the compiler sees no LDS write in flight and puts no alias vmcnt(0)
//    before the fragment reads) and the waits are counted, never 0 inside
//    the loop.
//  * Workgroup -> tile map: bijective XCD remap (each XCD walks a contiguous
//    range of tiles), then row panels in groups of 8 so the 32 concurrent
//    tiles of an XCD share A and W panels in its L2.
//  * Epilogue: each wave stages its 128 x 64 block through LDS (64 rows at a
//    time) and stores whole vectors with bias, activation, row mask, alpha
//    and fp32 residual applied; fp32, bf16 or (MXFP8) e4m3 + block scales.
#include <type_traits>

#include "gemm256.h"
#include "mfma.h"
#include "mx.h"

using namespace sbk;

namespace {

enum { G_NONE = 0, G_SWISH = 1, G_LRELU = 3, G_GELU = 4 };

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NT = 512;
constexpr int HALF = 128 * 128;        // bytes of a half-tile (128 rows x 128 B)
constexpr int SCB = 2 * 256 * 4;       // MXFP8: A + W scale dwords of a K-tile
constexpr int CS_STRIDE = 68;          // epilogue C rows (floats)
constexpr int EPI_BYTES = 8 * 64 * CS_STRIDE * 4;
template <bool MX>
constexpr int kbuf() { return 4 * HALF + (MX ? SCB : 0); }
template <bool MX>
constexpr int lds_bytes() { return 2 * kbuf<MX>() > EPI_BYTES ? 2 * kbuf<MX>() : EPI_BYTES; }

// one 1-KB LDS-DMA piece: lane l's 16 source bytes land at lds_wave + 16 l
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_wave) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_wave) : "memory", "m0");
}
// a dword piece: lane l's 4 bytes land at lds_wave + 4 l (exec-masked lanes write nothing)
__device__ __forceinline__ void dma4(const void* src, uint32_t lds_wave) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(lds_wave) : "memory", "m0");
}

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)p);
}

// GELU(x) = x Φ(x), Φ(x) = (1 + erf(x / √2)) / 2 (torch.nn.GELU, the
// TransformerEncoder's activation), with erfc(z) = y(t) e^{-z²},
// t = 1 / (1 + p z), y a degree-5 polynomial (Abramowitz & Stegun 7.1.26,
// |error| <= 1.5e-7 on erf): h = erfc(|x| / √2) / 2 and GELU = x (1 - h) for
// x >= 0, x h below (no cancellation in the negative tail).  ~15 VALU
// instructions against ~40 for erff; the epilogue of the FFN up-projection
// (98 M values per config-5 layer) was VALU-issue bound on it.  This kernel's
// outputs are bf16 or e4m3, far coarser than the approximation.
__device__ __forceinline__ float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  const float y = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                           0.254829592f);
  const float h = 0.5f * y * __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);
  return x * (x >= 0.f ? 1.0f - h : h);
}

// the same on a pair (v_pk_fma / v_pk_mul for everything but the two
// transcendentals): the FFN1 epilogue's GELU ran on scalar VALU at a cost of
// ~29 us of config 5's 217-us MXFP8 up-projection
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v gelu_fast2(f2v x) {
  const f2v z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  const f2v d = z * 0.3275911f + 1.0f;
  const f2v t = f2v{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  f2v y = t * 1.061405429f - 1.453152027f;
  y = y * t + 1.421413741f;
  y = y * t - 0.284496736f;
  y = y * t + 0.254829592f;
  y = y * t;
  const f2v q = (z * z) * -1.4426950408889634f;
  const f2v h = (0.5f * y) * f2v{__builtin_amdgcn_exp2f(q[0]), __builtin_amdgcn_exp2f(q[1])};
  const f2v one_h = 1.0f - h;
  return x * f2v{x[0] >= 0.f ? one_h[0] : h[0], x[1] >= 0.f ? one_h[1] : h[1]};
}

template <int ACT>
__device__ __forceinline__ float act_f(float x, float slope) {
  if (ACT == G_SWISH) return x * (1.0f / (1.0f + __expf(-x)));
  if (ACT == G_LRELU) return x >= 0.f ? x : x * slope;
  if (ACT == G_GELU) return gelu_fast(x);
  return x;
}

struct G256 {
  const uint8_t* A;
  const uint8_t* SA;          // MXFP8: scales, byte (row, k / 32)
  long long lda, ldsa;        // bytes
  long long rpb, a_bs, s_bs;  // A row m = (m / rpb, m % rpb) at A + (m / rpb) * a_bs + (m % rpb) * lda
  const uint8_t* W;
  const uint8_t* SW;
  long long ldw, ldsw;        // bytes
  int M, N, K;                // K in elements
  Gemm256Epi ep;
  int out_mode;               // 0 fp32, 1 bf16, 2 MXFP8 (MX only)
  uint8_t* out_scales;
  long long ldso;
  // split-K tail (launch_t): ksplit 2 = workgroups 2s and 2s + 1 take the two
  // K halves of tile tile_base + s and store raw fp32 partials to part
  // (tile-local 256 x 256, one per workgroup); 0 = whole tiles
  int ksplit, tile_base;
  float* part;
};

// tile index (the launch order) -> (row tile, column tile): bijective XCD
// remap (workgroup i runs on XCD i % 8; each XCD walks a contiguous range),
// then row panels in groups of 8 walked column by column
__device__ __forceinline__ void tile_of(int orig, int ntn, int ntm, int& tm, int& tn) {
  const int nwg = ntn * ntm, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  constexpr int GM = 8;  // row panels per group; a group is walked column by column
  const int gsz = GM * ntn, grp = wg / gsz, first = grp * GM, gm = min(GM, ntm - first);
  const int in = wg - grp * gsz;
  tm = first + in % gm;
  tn = in / gm;
}

template <bool MX, int ACT, int OUT>
__global__ void __launch_bounds__(NT, 1) gemm256_kernel(G256 p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int KB = kbuf<MX>();
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;

  // ---- tile of this workgroup (and, split, its K half)
  const bool split = OUT == 0 && p.ksplit == 2;
  const int half = split ? (int)(blockIdx.x & 1) : 0;
  int tm, tn;
  tile_of(split ? p.tile_base + (int)(blockIdx.x >> 1) : (int)blockIdx.x, p.N >> 8, (p.M + 255) >> 8, tm, tn);
  const int m0 = tm << 8, n0 = tn << 8;
  int nk = MX ? p.K >> 7 : p.K >> 6;
  const int kt0 = half ? nk >> 1 : 0;  // first K-tile (every K-tile is 128 B of a row)
  if (split) nk = half ? nk - (nk >> 1) : nk >> 1;

  // ---- DMA sources: half-tile piece j = 2w + i covers rows 8j .. 8j+7 of the
  // half; lane -> row 8j + (lane >> 3), physical chunk lane & 7 holding logical
  // chunk (lane & 7) ^ ((row >> 1) & 7)
  const uint8_t* asrc[2][2];
  const uint8_t* wsrc[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = h * 128 + (2 * w + i) * 8 + (lane >> 3);
      const int pch = (lane & 7) ^ ((r >> 1) & 7);
      const long long m = min(m0 + r, p.M - 1), b = m / p.rpb;
      asrc[h][i] = p.A + b * p.a_bs + (m - b * p.rpb) * p.lda + pch * 16 + kt0 * 128;
      wsrc[h][i] = p.W + (long long)(n0 + r) * p.ldw + pch * 16 + kt0 * 128;
    }
  // MXFP8 scale pieces: the 512 scale dwords of a K-tile (A rows 0-255, W
  // rows 0-255) are 8 pieces of 64 rows, one per wave: wave w moves A rows
  // 64w + lane (w < 4) or W rows 64(w - 4) + lane, issued with phase 0's DMA
  const uint8_t* ssrc = nullptr;
  if (MX) {
    const int r = (w & 3) * 64 + lane;
    if (w < 4) {
      const long long m = min(m0 + r, p.M - 1), b = m / p.rpb;
      ssrc = p.SA + b * p.s_bs + (m - b * p.rpb) * p.ldsa;
    } else {
      ssrc = p.SW + (long long)(n0 + r) * p.ldsw;
    }
    ssrc += kt0 * 4;
  }
  const uint32_t lds0 = lds_u32(smem);
  auto issue_a1 = [&](int kt, int buf, int h) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      dma16(asrc[h][i] + kt * 128, __builtin_amdgcn_readfirstlane(lds0 + buf * KB + h * HALF + (2 * w + i) * 1024));
  };
  auto issue_w1 = [&](int kt, int buf, int h) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      dma16(wsrc[h][i] + kt * 128,
            __builtin_amdgcn_readfirstlane(lds0 + buf * KB + (2 + h) * HALF + (2 * w + i) * 1024));
  };
  // scale dwords: A rows at 4*HALF + 4 r, W rows at 4*HALF + 1024 + 4 r
  auto issue_s = [&](int kt, int buf) __attribute__((always_inline)) {
    if (MX) dma4(ssrc + kt * 4, __builtin_amdgcn_readfirstlane(lds0 + buf * KB + 4 * HALF + w * 256));
  };

  // ---- fragments and MFMAs
  // bf16: 16x16x32, acc[8 m-tiles][4 n-tiles] f32x4; per quadrant fa[4][2 ks], fb[2][2 ks]
  // MXFP8: 32x32x64, acc[4][2] f32x16; per quadrant fa[2][2 ks], fb[1][2 ks] (i32x8) + scale dwords
  using acc_t = typename std::conditional<MX, f32x16, f32x4>::type;
  using frag_t = typename std::conditional<MX, i32x8, bf16x8>::type;
  constexpr int AM = MX ? 4 : 8, AN = MX ? 2 : 4;   // accumulator tiles
  constexpr int QM = AM / 2, QN = AN / 2;           // per quadrant
  acc_t acc[AM][AN];
#pragma unroll
  for (int i = 0; i < AM; ++i)
#pragma unroll
    for (int j = 0; j < AN; ++j) acc[i][j] = acc_t{};
  frag_t fa[QM][2], fb0[QN][2], fb1[QN][2];
  uint32_t sa[QM], sb0[QN], sb1[QN];
  const int fr = MX ? (lane & 31) : (lane & 15), fq = MX ? (lane >> 5) : (lane >> 4);
  auto rd16 = [](const uint8_t* base, int r, int c) __attribute__((always_inline)) {
    return *reinterpret_cast<const int4*>(base + r * 128 + 16 * (c ^ ((r >> 1) & 7)));
  };
  auto read_frag = [&](const uint8_t* base, int r, int ks) __attribute__((always_inline)) {
    frag_t f;
    if constexpr (MX) {
      const int4 x0 = rd16(base, r, 4 * ks + fq), x1 = rd16(base, r, 4 * ks + 2 + fq);
      f = i32x8{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    } else {
      const int4 x = rd16(base, r, 4 * ks + fq);
      f = __builtin_bit_cast(bf16x8, x);
    }
    return f;
  };
  // A quadrant qm of this wave: half wm, local rows qm*64 + mt*(16|32) + fr
  auto read_a = [&](const uint8_t* buf, int qm) __attribute__((always_inline)) {
    const uint8_t* base = buf + wm * HALF;
#pragma unroll
    for (int mt = 0; mt < QM; ++mt) {
      const int r = qm * 64 + mt * (MX ? 32 : 16) + fr;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fa[mt][ks] = read_frag(base, r, ks);
      if (MX) sa[mt] = reinterpret_cast<const uint32_t*>(buf + 4 * HALF)[wm * 128 + r];
    }
  };
  // W quadrant qn: half wn >> 1, local rows (wn & 1)*64 + qn*32 + nt*(16|32) + fr
  auto read_b = [&](frag_t (&fb)[QN][2], uint32_t (&sb)[QN], const uint8_t* buf, int qn)
      __attribute__((always_inline)) {
    const uint8_t* base = buf + (2 + (wn >> 1)) * HALF;
#pragma unroll
    for (int nt = 0; nt < QN; ++nt) {
      const int r = (wn & 1) * 64 + qn * 32 + nt * (MX ? 32 : 16) + fr;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fb[nt][ks] = read_frag(base, r, ks);
      if (MX) sb[nt] = reinterpret_cast<const uint32_t*>(buf + 4 * HALF + 1024)[(wn >> 1) * 128 + r];
    }
  };
  auto mfma_q = [&](const frag_t (&fb)[QN][2], const uint32_t (&sb)[QN], int qm, int qn)
      __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mt = 0; mt < QM; ++mt)
#pragma unroll
        for (int nt = 0; nt < QN; ++nt) {
          acc_t& c = acc[qm * QM + mt][qn * QN + nt];
          if constexpr (MX) {
            // lane half fq supplies the scale of block 2*ks + fq of its row
            const int sh = 8 * (2 * ks + fq);
            c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[mt][ks], fb[nt][ks], c, 0, 0, 0,
                                                                (int)((sa[mt] >> sh) & 0xFF), 0,
                                                                (int)((sb[nt] >> sh) & 0xFF));
          } else {
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt][ks], fb[nt][ks], c, 0, 0, 0);
          }
        }
    // pin the quadrant's MFMAs ahead of the phase barrier (the compiler would
    // otherwise sink independent MFMAs to later phases)
#pragma unroll
    for (int mt = 0; mt < QM; ++mt)
#pragma unroll
      for (int nt = 0; nt < QN; ++nt) asm volatile("" : "+v"(acc[qm * QM + mt][qn * QN + nt]));
    __builtin_amdgcn_s_setprio(0);
  };
  auto barrier = []() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // retire everything but the youngest half-tile issue (2 pieces)
  auto wait_but_one_half = []() __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  };

  // ---- prologue: tile 0 and W0(1); retire tile 0 on every wave, then one
  // barrier before any read.  Waves 4-7 then take one extra barrier: from
  // here on they run one barrier (half a phase) behind waves 0-3.
  issue_a1(0, 0, 0);
  issue_a1(0, 0, 1);
  issue_w1(0, 0, 0);
  issue_w1(0, 0, 1);
  issue_s(0, 0);
  if (nk > 1) {
    issue_w1(1, 1, 0);
    wait_but_one_half();
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  barrier();
  if (wm) barrier();

  // Per K-tile t (buffer t & 1), with both W fragment sets kept in VGPRs the
  // W slot is last read in phase 1 and the A slot in phase 2.  Under the
  // stagger a slot last read in phase p may be refilled from phase p + 2 on,
  // and data must be waited for in the phase before its first read:
  //   p0: read A[q0], W[q0]   DMA W1(t+1), A0(t+1) (+ MXFP8 scales of t+1)
  //   p1: read W[q1]          DMA A1(t+1)
  //   p2: read A[q1]
  //   p3: (no reads)          DMA W0(t+2); vmcnt retires tile t+1
  // (W0(t+1) was issued in phase 3 of t-1.)
  for (int t = 0; t < nk; ++t) {
    const uint8_t* buf = smem + (t & 1) * KB;
    const bool nx = t + 1 < nk, nx2 = t + 2 < nk;
    const int ob = (t + 1) & 1;
    // phase 0
    read_a(buf, 0);
    read_b(fb0, sb0, buf, 0);
    if (nx) {
      issue_w1(t + 1, ob, 1);
      issue_a1(t + 1, ob, 0);
      issue_s(t + 1, ob);  // the scale region was last read in phase 2 of t-1
    }
    barrier();
    mfma_q(fb0, sb0, 0, 0);
    barrier();
    // phase 1
    read_b(fb1, sb1, buf, 1);
    if (nx) issue_a1(t + 1, ob, 1);
    barrier();
    mfma_q(fb1, sb1, 0, 1);
    barrier();
    // phase 2
    read_a(buf, 1);
    barrier();
    mfma_q(fb1, sb1, 1, 1);
    barrier();
    // phase 3
    if (nx2) {
      issue_w1(t + 2, t & 1, 0);
      wait_but_one_half();
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier();
    mfma_q(fb0, sb0, 1, 0);
    barrier();
  }
  if (!wm) barrier();  // the stagger's matching barrier

  // ---- epilogue: per wave, 64 accumulator rows at a time through its own
  // LDS region (fp32, row stride CS_STRIDE), then 16 column quads x 4 rows per
  // pass of whole-vector stores
  __syncthreads();
  float* cs = reinterpret_cast<float*>(smem) + w * (64 * CS_STRIDE);
  const int ocol = (lane & 15) * 4;  // column quad within the wave's 64
  const int gcol = n0 + wn * 64 + ocol;
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (p.ep.bias) bv = *reinterpret_cast<const float4*>(p.ep.bias + gcol);
#pragma unroll
  for (int hm = 0; hm < 2; ++hm) {
    if constexpr (MX) {
      // 32x32 C/D: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            cs[(mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * fq) * CS_STRIDE + nt * 32 + fr] = acc[hm * 2 + mt][nt][r];
    } else {
      // 16x16 C/D: col = lane & 15, row = 4 (lane >> 4) + r
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r) cs[(mt * 16 + fq * 4 + r) * CS_STRIDE + nt * 16 + fr] = acc[hm * 4 + mt][nt][r];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's stores before its reads
    // residual / row-mask loads of 8 passes at a time first (rows clamped, so
    // no branch serialises them), then the LDS reads, math and stores
#pragma unroll
    for (int pg = 0; pg < 2; ++pg) {
      float4 rv[8];
      float scv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int row = min(m0 + wm * 128 + hm * 64 + (pg * 8 + q) * 4 + (lane >> 4), p.M - 1);
        rv[q] = p.ep.res ? *reinterpret_cast<const float4*>(p.ep.res + (long long)row * p.ep.ldr + gcol)
                         : make_float4(0.f, 0.f, 0.f, 0.f);
        scv[q] = (p.ep.rowmask && p.ep.rowmask[row]) ? 0.f : p.ep.alpha;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int rl = (pg * 8 + q) * 4 + (lane >> 4);
        const int row = m0 + wm * 128 + hm * 64 + rl;
        const float4 a = *reinterpret_cast<const float4*>(cs + rl * CS_STRIDE + ocol);
        const float sc = scv[q];
        float v0, v1, v2, v3;
        if constexpr (ACT == G_GELU) {
          const f2v g0 = gelu_fast2(f2v{a.x + bv.x, a.y + bv.y}) * sc, g1 = gelu_fast2(f2v{a.z + bv.z, a.w + bv.w}) * sc;
          v0 = g0[0]; v1 = g0[1]; v2 = g1[0]; v3 = g1[1];
        } else {
          v0 = act_f<ACT>(a.x + bv.x, p.ep.slope) * sc; v1 = act_f<ACT>(a.y + bv.y, p.ep.slope) * sc;
          v2 = act_f<ACT>(a.z + bv.z, p.ep.slope) * sc; v3 = act_f<ACT>(a.w + bv.w, p.ep.slope) * sc;
        }
        if (p.ep.res) {  // (no +0 when there is none: a -0 stays -0, as in the other kernels)
          v0 += rv[q].x;
          v1 += rv[q].y;
          v2 += rv[q].z;
          v3 += rv[q].w;
        }
        if (OUT == 2) {
          // MXFP8 output: amax over the 8 lanes (32 columns) of a block, e4m3
          // dword per lane, the block's scale byte from its first lane
          const float am = group_max<8>(fmaxf(fmaxf(fabsf(v0), fabsf(v1)), fmaxf(fabsf(v2), fabsf(v3))));
          const int sbyte = mx_scale_byte(am);
          const float is = mx_inv_scale(sbyte);
          if (row < p.M) {
            *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(p.ep.out) + (long long)row * p.ep.ldc + gcol) =
                pack4_e4m3(v0 * is, v1 * is, v2 * is, v3 * is);
            if ((lane & 7) == 0) p.out_scales[(long long)row * p.ldso + (gcol >> 5)] = (uint8_t)sbyte;
          }
        } else if (row < p.M) {
          if (OUT == 1) {
            uint2 pk;
            pk.x = pack_bf16x2(v0, v1);
            pk.y = pack_bf16x2(v2, v3);
            *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.ep.out) + (long long)row * p.ep.ldc + gcol) = pk;
          } else if (split) {  // the partial, tile-local (the launch passes no bias / residual / mask, alpha 1)
            *reinterpret_cast<float4*>(p.part + (long long)blockIdx.x * 65536 + (row - m0) * 256 + (gcol - n0)) =
                make_float4(v0, v1, v2, v3);
          } else {
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.ep.out) + (long long)row * p.ep.ldc + gcol) =
                make_float4(v0, v1, v2, v3);
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next half overwrites
  }
}

// Split-K tail, second step: out = epilogue(P0 + P1) for tile tile_base + s,
// P0 / P1 the two K halves' fp32 partials (one add, so the sum does not
// depend on which half finished first).  One workgroup per (tile, 16-row
// band), a float4 column quad per thread; the epilogue is gemm256_kernel's
// (bias, activation, row mask, alpha, fp32 residual, fp32 out).
template <int ACT>
__global__ void __launch_bounds__(256) splitk_epi_kernel(G256 p) {
  const int s = blockIdx.x >> 4, band = blockIdx.x & 15;
  int tm, tn;
  tile_of(p.tile_base + s, p.N >> 8, (p.M + 255) >> 8, tm, tn);
  const int m0 = tm << 8, n0 = tn << 8;
  const int c = 4 * (threadIdx.x & 63), gcol = n0 + c;
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (p.ep.bias) bv = *reinterpret_cast<const float4*>(p.ep.bias + gcol);
  const float* p0 = p.part + (long long)(2 * s) * 65536;
  const float* p1 = p0 + 65536;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rl = band * 16 + 4 * i + (threadIdx.x >> 6), row = m0 + rl;
    if (row >= p.M) continue;  // (not stored by the partial launch either)
    const float4 x0 = *reinterpret_cast<const float4*>(p0 + rl * 256 + c);
    const float4 x1 = *reinterpret_cast<const float4*>(p1 + rl * 256 + c);
    const float4 a = make_float4(x0.x + x1.x, x0.y + x1.y, x0.z + x1.z, x0.w + x1.w);
    const float sc = (p.ep.rowmask && p.ep.rowmask[row]) ? 0.f : p.ep.alpha;
    float v0, v1, v2, v3;
    if constexpr (ACT == G_GELU) {
      const f2v g0 = gelu_fast2(f2v{a.x + bv.x, a.y + bv.y}) * sc, g1 = gelu_fast2(f2v{a.z + bv.z, a.w + bv.w}) * sc;
      v0 = g0[0]; v1 = g0[1]; v2 = g1[0]; v3 = g1[1];
    } else {
      v0 = act_f<ACT>(a.x + bv.x, p.ep.slope) * sc; v1 = act_f<ACT>(a.y + bv.y, p.ep.slope) * sc;
      v2 = act_f<ACT>(a.z + bv.z, p.ep.slope) * sc; v3 = act_f<ACT>(a.w + bv.w, p.ep.slope) * sc;
    }
    if (p.ep.res) {
      const float4 r = *reinterpret_cast<const float4*>(p.ep.res + (long long)row * p.ep.ldr + gcol);
      v0 += r.x;
      v1 += r.y;
      v2 += r.z;
      v3 += r.w;
    }
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.ep.out) + (long long)row * p.ep.ldc + gcol) =
        make_float4(v0, v1, v2, v3);
  }
}

// compute units of the current device (cached; the split-K tail rule)
int cu_count() {
  static int n = 0;
  if (n <= 0) {
    int d = 0, c = 0;
    if (hipGetDevice(&d) == hipSuccess && hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess &&
        c > 0)
      n = c;
    else
      return 256;
  }
  return n;
}

// Split-K tail (MXFP8, fp32 out): with one 256 x 256 workgroup per CU, the
// tiles past the last full round run as a partial round (config 5's N =
// 1024 projections: 376 tiles on 256 CUs, 120 in the second round).  When
// that tail fills at most half the CUs and K has >= 16 K-tiles, each tail
// tile runs as two workgroups over the K halves (a full round of half-length
// tiles) plus splitk_epi_kernel.  Returns the tail tile count, 0 = no split.
int split_tail(int M, int N, int K) {
  if (M <= 0 || N <= 0 || (N & 255) || (K & 127)) return 0;
  const int nt = (N >> 8) * ((M + 255) >> 8), cus = cu_count(), tail = nt % cus;
  return (nt > cus && tail > 0 && 2 * tail <= cus && (K >> 7) >= 16) ? tail : 0;
}

template <bool MX, int ACT, int OUT>
int launch_t(const G256& p, hipStream_t s, float* ws, long long ws_floats) {
  // > 64 KB of dynamic LDS: opted in per device
  if (hipError_t e = sbk::lds_optin(reinterpret_cast<const void*>(&gemm256_kernel<MX, ACT, OUT>), lds_bytes<MX>()))
    return (int)e;
  const int grid = (p.N >> 8) * ((p.M + 255) >> 8);
  if constexpr (MX && OUT == 0) {
    const int tail = ws ? split_tail(p.M, p.N, p.K) : 0;
    if (tail && ws_floats >= 2LL * tail * 65536) {
      if (hipError_t e = sbk::lds_optin(reinterpret_cast<const void*>(&gemm256_kernel<true, G_NONE, 0>),
                                        lds_bytes<true>()))
        return (int)e;
      G256 q = p;  // whole tiles: the first grid - tail of the launch order
      q.ksplit = 0;
      hipLaunchKernelGGL((gemm256_kernel<MX, ACT, OUT>), dim3(grid - tail), dim3(NT), lds_bytes<MX>(), s, q);
      SBK_CHECK_LAUNCH();
      G256 h = p;  // the tail's K halves: raw partials
      h.ep.bias = nullptr;
      h.ep.res = nullptr;
      h.ep.rowmask = nullptr;
      h.ep.alpha = 1.f;
      h.ep.act = G_NONE;
      h.ksplit = 2;
      h.tile_base = grid - tail;
      h.part = ws;
      hipLaunchKernelGGL((gemm256_kernel<true, G_NONE, 0>), dim3(2 * tail), dim3(NT), lds_bytes<true>(), s, h);
      SBK_CHECK_LAUNCH();
      G256 f = p;  // the tail's epilogue
      f.tile_base = grid - tail;
      f.part = ws;
      hipLaunchKernelGGL((splitk_epi_kernel<ACT>), dim3(16 * tail), dim3(256), 0, s, f);
      SBK_CHECK_LAUNCH();
      return 0;
    }
  }
  G256 q = p;
  q.ksplit = 0;
  hipLaunchKernelGGL((gemm256_kernel<MX, ACT, OUT>), dim3(grid), dim3(NT), lds_bytes<MX>(), s, q);
  SBK_CHECK_LAUNCH();
  return 0;
}

template <bool MX, int OUT>
int launch_o(const G256& p, hipStream_t s, float* ws = nullptr, long long ws_floats = 0) {
  switch (p.ep.act) {
    case G_NONE: return launch_t<MX, G_NONE, OUT>(p, s, ws, ws_floats);
    case G_SWISH:
      if constexpr (MX) return SBK_ERR_ARG;
      else return launch_t<MX, G_SWISH, OUT>(p, s, ws, ws_floats);
    case G_LRELU: return launch_t<MX, G_LRELU, OUT>(p, s, ws, ws_floats);
    case G_GELU: return launch_t<MX, G_GELU, OUT>(p, s, ws, ws_floats);
    default: return SBK_ERR_ARG;
  }
}

bool epi_ok(const Gemm256Epi& ep) {
  if (ep.act != G_NONE && ep.act != G_SWISH && ep.act != G_LRELU && ep.act != G_GELU) return false;
  const uintptr_t al = reinterpret_cast<uintptr_t>(ep.bias) | reinterpret_cast<uintptr_t>(ep.res) |
                       reinterpret_cast<uintptr_t>(ep.out);
  return !(al & 15) && !(ep.ldr & 3) && !(ep.ldc & 3);
}

}  // namespace

bool gemm256_supported(int M, int N, int K, long long lda, long long ldw, const void* A, const void* W,
                       const Gemm256Epi& ep) {
  if (M <= 0 || N <= 0 || K <= 0 || (N & 255) || (K & 63) || (lda & 7) || (ldw & 7)) return false;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(W)) & 15) return false;
  return epi_ok(ep);
}

int gemm256_launch(const void* A, long long lda, const void* W, long long ldw, int M, int N, int K,
                   const Gemm256Epi& ep, hipStream_t s) {
  if (!gemm256_supported(M, N, K, lda, ldw, A, W, ep)) return SBK_ERR_ARG;
  G256 p{reinterpret_cast<const uint8_t*>(A), nullptr, lda * 2, 0, (long long)M, 0, 0,
         reinterpret_cast<const uint8_t*>(W), nullptr, ldw * 2, 0, M, N, K, ep, ep.out_bf16 ? 1 : 0, nullptr, 0};
  return ep.out_bf16 ? launch_o<false, 1>(p, s) : launch_o<false, 0>(p, s);
}

bool mx256_supported(int M, int N, int K, long long lda, long long ldsa, long long rpb, long long a_bs,
                     long long s_bs, long long ldw, long long ldsw, const void* A, const void* SA, const void* W,
                     const void* SW, const Gemm256Epi& ep, int out_mode, const void* out_scales) {
  if (M <= 0 || N <= 0 || K <= 0 || (N & 255) || (K & 127) || rpb <= 0) return false;
  if ((lda | a_bs | ldw) & 15) return false;
  if ((ldsa | s_bs | ldsw) & 3) return false;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(W)) & 15) return false;
  if ((reinterpret_cast<uintptr_t>(SA) | reinterpret_cast<uintptr_t>(SW)) & 3) return false;
  if (ep.act == G_SWISH || out_mode < 0 || out_mode > 2) return false;
  if (out_mode == 2 && (!out_scales || (ep.ldc & 15) || (reinterpret_cast<uintptr_t>(ep.out) & 15))) return false;
  return epi_ok(ep);
}

long long mx256_split_floats(int M, int N, int K, int out_mode) {
  return out_mode == 0 ? 2LL * split_tail(M, N, K) * 65536 : 0;
}

int mx256_launch(const void* A, const void* SA, long long lda, long long ldsa, long long rpb, long long a_bs,
                 long long s_bs, const void* W, const void* SW, long long ldw, long long ldsw, int M, int N, int K,
                 const Gemm256Epi& ep, int out_mode, void* out_scales, long long ldso, hipStream_t s, float* ws,
                 long long ws_floats) {
  if (!mx256_supported(M, N, K, lda, ldsa, rpb, a_bs, s_bs, ldw, ldsw, A, SA, W, SW, ep, out_mode, out_scales))
    return SBK_ERR_ARG;
  G256 p{reinterpret_cast<const uint8_t*>(A), reinterpret_cast<const uint8_t*>(SA), lda, ldsa, rpb, a_bs, s_bs,
         reinterpret_cast<const uint8_t*>(W), reinterpret_cast<const uint8_t*>(SW), ldw, ldsw, M, N, K, ep,
         out_mode, reinterpret_cast<uint8_t*>(out_scales), ldso};
  switch (out_mode) {
    case 0: return launch_o<true, 0>(p, s, ws, ws_floats);
    case 1: return launch_o<true, 1>(p, s);
    default: return launch_o<true, 2>(p, s);
  }
}

// MXFP8 GEMM on the 256 x 256 multi-phase kernel: the arguments of
// sbk_mx_gemm (mxgemm.hip), N % 256 == 0 and K % 128 == 0; SBK_ERR_ARG
// outside that envelope.  sbk_mx_gemm dispatches here by itself for large M.
SBK_API int sbk_mx_gemm256(const uint8_t* A, const uint8_t* SA, long long lda, long long ldsa, long long rpb,
                           long long a_bs, long long s_bs, const uint8_t* W, const uint8_t* SW, long long ldw,
                           long long ldsw, int M, int N, int K, const float* bias, int act, float alpha,
                           const float* res, long long ldr, void* out, long long ldc, int out_mode,
                           uint8_t* out_scales, long long ldso, void* stream) {
  if (ldr > 0x7fffffffLL || ldc > 0x7fffffffLL) return SBK_ERR_ARG;
  const Gemm256Epi ep{bias, act, 0.f, res, (int)ldr, alpha, nullptr, out, (int)ldc, out_mode == 1};
  return mx256_launch(A, SA, lda, ldsa, rpb, a_bs, s_bs, W, SW, ldw, ldsw, M, N, K, ep, out_mode, out_scales, ldso,
                      (hipStream_t)stream);
}
