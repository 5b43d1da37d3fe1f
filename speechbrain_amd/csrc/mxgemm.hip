// MXFP8 GEMM for the config-5 encoder (wav2vec2 latent extractor convs and
// the 24-layer TransformerEncoder projections), gfx950 block-scaled MFMA.
//
//   C[M, N] = epilogue( sum_k A[m, k] * W[n, k] )
//   A: e4m3 (M, K) with E8M0 scales (M, K/32), W: e4m3 (N, K) + (N, K/32)
//   (nn.Linear [out][in] layout; both operands K-contiguous).
//
// v_mfma_scale_f32_32x32x64_f8f6f4 (layout measured by scripts/mx_probe4.hip):
// lane l feeds row (l & 31); operand bytes 0-15 of BOTH lane halves form the
// first 32-element K block and bytes 16-31 the second; the E8M0 scale of
// block b of row r comes from lane r + 32*b.  So the OCP MX block (32 along
// K) maps onto two 16-B halves and one scale byte per lane, and the hardware
// applies both operands' scales: no dequantisation pass, no per-tensor amax.  It runs at 2x the bf16
// MFMA rate (MI355X_MICROARCH.md, matrix cores).
//
// Tile 128 x 128 x 128 B, 4 waves (2 x 2), wave tile 64 x 64 = 2 x 2 MFMA
// tiles of 32 x 32; operands and scales staged global -> LDS by LDS-DMA
// (global_load_lds, 16 B data / 4 B scale dwords) into two buffers; the
// 16-B chunk index of a 128-B row is XOR-swizzled by (row & 7) on the
// source address so fragment reads spread over the banks.  Block -> tile
// map is XCD-aware (consecutive tiles of one XCD share A rows in its L2).
//
// A-row addressing supports the strided, overlapping rows of a valid
// convolution: row m = (b, t) = (m / rpb, m % rpb) starts at
// A + b*a_bs + t*lda (and the scales at SA + b*s_bs + t*ldsa), so
// Conv1d(k, stride) over (T, C) channels-last input is the GEMM with
// K = k*C, lda = stride*C and the weight permuted to [out][tap][in]
// (wav2vec.py:28-88 conv layers 1..6, CNN.py:309-516 "valid").
//
// Epilogue: bias, GELU / ReLU, alpha * val + fp32 residual, output fp32,
// bf16 or MXFP8 (+ scales, amax over the 32 lanes of a tile row).
#include "mx.h"
#include "gemm256.h"

using namespace sbk;

namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 128;  // BK in bytes = fp8 elements
constexpr int NT = 256;
constexpr int TILE_BYTES = BM * BK;          // 16 KB per operand per stage
constexpr int SC_BYTES = BM * 4;             // 4 scale bytes per row per stage
constexpr int STAGE = 2 * TILE_BYTES + 2 * SC_BYTES;

struct MxArgs {
  const uint8_t* A;
  const uint8_t* SA;
  long long lda, ldsa;       // bytes
  long long rpb, a_bs, s_bs; // rows per batch, batch strides (bytes)
  const uint8_t* W;
  const uint8_t* SW;
  long long ldw, ldsw;
  int M, N, K;
  const float* bias;
  int act;                   // 0 none, 3 relu, 4 gelu
  float alpha;
  const float* res;
  long long ldr;
  void* out;
  long long ldc;
  int out_mode;              // 0 fp32, 1 bf16, 2 mxfp8
  uint8_t* out_scales;
  long long ldso;
};

// LDS-DMA: `g` is this lane's source, `lds_wave` the WAVE-UNIFORM destination
// base; lane l's bytes land at lds_wave + l * size.
__device__ __forceinline__ void glds16(const void* g, void* lds_wave) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* g, void* lds_wave) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave, 4, 0, 0);
}

__device__ __forceinline__ long long a_row(const MxArgs& p, int m) {
  const long long b = m / p.rpb, t = m - b * p.rpb;
  return b * p.a_bs + t * p.lda;
}
__device__ __forceinline__ long long a_srow(const MxArgs& p, int m) {
  const long long b = m / p.rpb, t = m - b * p.rpb;
  return b * p.s_bs + t * p.ldsa;
}

template <int ACT>
__device__ __forceinline__ float act_f(float x) {
  if (ACT == 4) return gelu_erf(x);
  if (ACT == 3) return fmaxf(x, 0.f);
  return x;
}

template <int ACT, int OUT>
__global__ void __launch_bounds__(NT) mx_gemm_kernel(MxArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  // XCD-aware tile order: each XCD (g % 8) walks a contiguous range of the
  // row-major tile list, so tiles sharing A rows meet in one L2
  const int ntn = p.N / BN, ntm = (p.M + BM - 1) / BM, nt = ntm * ntn;
  int g = blockIdx.x;
  if ((nt & 7) == 0) g = (g & 7) * (nt >> 3) + (g >> 3);
  const int tm = g / ntn, tn = g - tm * ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = p.K / BK;

  // staging map: thread tid moves rows (tid >> 3) + 32*i, chunk (tid & 7), i = 0..3
  const int srow = tid >> 3, sch = tid & 7;
  long long aoff[4], woff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = srow + 32 * i;
    const int m = min(m0 + r, p.M - 1);
    aoff[i] = a_row(p, m) + 16 * (sch ^ (r & 7));
    woff[i] = (long long)(n0 + r) * p.ldw + 16 * (sch ^ (r & 7));
  }
  // scales: waves 0-1 stage A rows (64 each), waves 2-3 W rows, one dword per row
  const int sr = (wv & 1) * 64 + lane;
  const long long soff = (wv < 2) ? a_srow(p, min(m0 + sr, p.M - 1)) : (long long)(n0 + sr) * p.ldsw;
  const uint8_t* sbase = (wv < 2) ? p.SA : p.SW;

  auto issue = [&](int kt, int buf) {
    uint8_t* st = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // the wave's 64 lanes cover rows wv*8 + 32*i + (lane >> 3), chunks lane & 7
      glds16(p.A + aoff[i] + kt * BK, st + (wv * 8 + 32 * i) * BK);
      glds16(p.W + woff[i] + kt * BK, st + TILE_BYTES + (wv * 8 + 32 * i) * BK);
    }
    glds4(sbase + soff + kt * 4, st + 2 * TILE_BYTES + (wv >= 2 ? SC_BYTES : 0) + (wv & 1) * 256);
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  const int fr = lane & 31, fh = lane >> 5;
  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) issue(kt + 1, (kt + 1) & 1);
    const uint8_t* st = smem + (kt & 1) * STAGE;
    const uint8_t* As = st;
    const uint8_t* Ws = st + TILE_BYTES;
    const uint32_t* Ss = reinterpret_cast<const uint32_t*>(st + 2 * TILE_BYTES);
    uint32_t sa[2], sw[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      sa[i] = Ss[wm * 64 + i * 32 + fr];
      sw[i] = Ss[BM + wn * 64 + i * 32 + fr];
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      // operand bytes 0-15 of both lane halves form scale block 0 of the
      // 64-deep step, bytes 16-31 block 1 (scripts/mx_probe4.hip): lane half
      // h takes the 16-B chunks 4s + h (block 2s) and 4s + 2 + h (block 2s + 1)
      const int c0 = 4 * s + fh, c1 = 4 * s + 2 + fh;
      i32x8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ra = wm * 64 + i * 32 + fr;
        const int4 x0 = *reinterpret_cast<const int4*>(As + ra * BK + 16 * (c0 ^ (ra & 7)));
        const int4 x1 = *reinterpret_cast<const int4*>(As + ra * BK + 16 * (c1 ^ (ra & 7)));
        af[i] = i32x8{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const int rb = wn * 64 + i * 32 + fr;
        const int4 y0 = *reinterpret_cast<const int4*>(Ws + rb * BK + 16 * (c0 ^ (rb & 7)));
        const int4 y1 = *reinterpret_cast<const int4*>(Ws + rb * BK + 16 * (c1 ^ (rb & 7)));
        bf[i] = i32x8{y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
      }
      const int sh = 8 * (2 * s + fh);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
              af[i], bf[j], acc[i][j], 0, 0, 0, (int)((sa[i] >> sh) & 0xFF), 0, (int)((sw[j] >> sh) & 0xFF));
    }
  }

  // epilogue from the accumulators: C/D of 32x32 tiles,
  // col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
  if (OUT == 2) {
    // MXFP8 output: block amax over the 32 lanes of a tile row (DPP), e4m3
    // bytes and scales staged in LDS, then written as full 16-B vectors
    // (byte-wide global stores of the same tile ran ~2x the main loop)
    constexpr int CS = BN + 16;  // byte row stride of the staged tile
    uint8_t* Ct = smem;
    uint8_t* Sc = smem + BM * CS;
    __syncthreads();  // every wave is done reading the operand stages
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int cl = wn * 64 + j * 32 + fr;
        const float bv = p.bias ? p.bias[n0 + cl] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          float v = act_f<ACT>(acc[i][j][r] + bv) * p.alpha;
          if (p.res && m0 + rl < p.M) v += p.res[(long long)(m0 + rl) * p.ldr + n0 + cl];
          const int sb = mx_scale_byte(group_max<32>(fabsf(v)));
          const float q = clamp_e4m3(v * mx_inv_scale(sb));
          Ct[rl * CS + cl] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(q, q, 0, false) & 0xFF);
          if (fr == 0) Sc[rl * 4 + wn * 2 + j] = (uint8_t)sb;
        }
      }
    }
    __syncthreads();
    uint8_t* out = reinterpret_cast<uint8_t*>(p.out);
#pragma unroll
    for (int c = tid; c < BM * BN / 16; c += NT) {
      const int rl = c >> 3, ch = c & 7;
      if (m0 + rl < p.M)
        *reinterpret_cast<int4*>(out + (long long)(m0 + rl) * p.ldc + n0 + 16 * ch) =
            *reinterpret_cast<const int4*>(Ct + rl * CS + 16 * ch);
    }
    if (tid < BM && m0 + tid < p.M)
      *reinterpret_cast<uint32_t*>(p.out_scales + (long long)(m0 + tid) * p.ldso + (n0 >> 5)) =
          *reinterpret_cast<const uint32_t*>(Sc + tid * 4);
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + j * 32 + fr;
      const float bv = p.bias ? p.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        float v = act_f<ACT>(acc[i][j][r] + bv) * p.alpha;
        if (row < p.M) {
          if (p.res) v += p.res[(long long)row * p.ldr + col];
          if (OUT == 1)
            reinterpret_cast<uint16_t*>(p.out)[(long long)row * p.ldc + col] = f32_to_bf16(v);
          else
            reinterpret_cast<float*>(p.out)[(long long)row * p.ldc + col] = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Large-M form: 256 x 128 tile, 8 waves (4 x 2, wave tile 64 x 64), THREE
// LDS stages with two in flight across each barrier.  The stage fills are
// inline-asm LDS-DMA pieces (the compiler then sees no LDS write in flight
// and places no alias-guard vmcnt(0) before the fragment reads), each wave
// issues exactly 7 per stage (4 A, 2 W, 1 scale dword piece), and the wait
// that retires stage kt is the counted vmcnt(7) that leaves stage kt+1 in
// flight, followed by a raw s_barrier (a __syncthreads() would drain it).
// 2x the W reuse of the 128 x 128 tile; 1 workgroup (8 waves) per CU.
constexpr int BM2 = 256, NT2 = 512;
constexpr int SC2 = (BM2 + BN) * 4 + 512;     // A + W scale dwords (+ dummy piece of waves 6-7)
constexpr int STAGE2 = BM2 * BK + BN * BK + SC2;
constexpr int NSTAGE2 = 3;

__device__ __forceinline__ void dma(const void* src, void* lds_wave, int bytes16) {
  const uint32_t la = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)lds_wave));
  if (bytes16)
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(la) : "memory", "m0");
  else
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(la) : "memory", "m0");
}

template <int ACT, int OUT>
__global__ void __launch_bounds__(NT2) mx_gemm256_kernel(MxArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;  // 4 x 2 waves
  const int ntn = p.N / BN, ntm = (p.M + BM2 - 1) / BM2, nt = ntm * ntn;
  int g = blockIdx.x, tm, tn;
  if ((ntn & 7) == 0) {
    // XCD x (= g % 8, the dispatcher's round robin) owns W column tiles
    // [x*cpx, x*cpx + cpx) for every row tile: its W slice stays resident in
    // that XCD's L2 and only A streams (each A row block is read once per XCD)
    const int cpx = ntn >> 3, q = g >> 3;
    tn = (g & 7) * cpx + q % cpx;
    tm = q / cpx;
  } else {
    if ((nt & 7) == 0) g = (g & 7) * (nt >> 3) + (g >> 3);
    tm = g / ntn;
    tn = g - tm * ntn;
  }
  const int m0 = tm * BM2, n0 = tn * BN;
  const int nk = p.K / BK;

  // staging: wave wv moves A rows wv*8 + 64*i + (lane >> 3) (i < 4) and
  // W rows wv*8 + 64*i + (lane >> 3) (i < 2), chunk lane & 7 (swizzled source)
  const int lr = lane >> 3, lc = lane & 7;
  long long aoff[4], woff[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wv * 8 + 64 * i + lr;
    aoff[i] = a_row(p, min(m0 + r, p.M - 1)) + 16 * (lc ^ (r & 7));
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = wv * 8 + 64 * i + lr;
    woff[i] = (long long)(n0 + r) * p.ldw + 16 * (lc ^ (r & 7));
  }
  // scale pieces: waves 0-3 A rows 64*wv + lane, waves 4-5 W rows 64*(wv-4) + lane,
  // waves 6-7 a dummy copy of W row scales into a spare slot (uniform vmcnt)
  const uint8_t* ssrc;
  int sdst;
  if (wv < 4) {
    ssrc = p.SA + a_srow(p, min(m0 + 64 * wv + lane, p.M - 1));
    sdst = BM2 * BK + BN * BK + 256 * wv;
  } else {
    const int r = 64 * (wv & 1) + lane;
    ssrc = p.SW + (long long)(n0 + r) * p.ldsw;
    sdst = BM2 * BK + BN * BK + (wv < 6 ? BM2 * 4 + 256 * (wv - 4) : (BM2 + BN) * 4 + 256 * (wv & 1));
  }

  auto issue = [&](int kt, int buf) {
    uint8_t* st = smem + buf * STAGE2;
#pragma unroll
    for (int i = 0; i < 4; ++i) dma(p.A + aoff[i] + (long long)kt * BK, st + (wv * 8 + 64 * i) * BK, 1);
#pragma unroll
    for (int i = 0; i < 2; ++i) dma(p.W + woff[i] + (long long)kt * BK, st + BM2 * BK + (wv * 8 + 64 * i) * BK, 1);
    dma(ssrc + kt * 4, st + sdst, 0);
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  const int fr = lane & 31, fh = lane >> 5;
  issue(0, 0);
  if (nk > 1) issue(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    // retire stage kt (this wave's pieces), leave stage kt+1 in flight
    if (kt + 1 < nk)
      asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + 2 < nk) issue(kt + 2, (kt + 2) % NSTAGE2);
    const uint8_t* st = smem + (kt % NSTAGE2) * STAGE2;
    const uint8_t* As = st;
    const uint8_t* Ws = st + BM2 * BK;
    const uint32_t* Ss = reinterpret_cast<const uint32_t*>(st + BM2 * BK + BN * BK);
    uint32_t sa[2], sw[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      sa[i] = Ss[wm * 64 + i * 32 + fr];
      sw[i] = Ss[BM2 + wn * 64 + i * 32 + fr];
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c0 = 4 * s + fh, c1 = 4 * s + 2 + fh;
      i32x8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ra = wm * 64 + i * 32 + fr;
        const int4 x0 = *reinterpret_cast<const int4*>(As + ra * BK + 16 * (c0 ^ (ra & 7)));
        const int4 x1 = *reinterpret_cast<const int4*>(As + ra * BK + 16 * (c1 ^ (ra & 7)));
        af[i] = i32x8{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const int rb = wn * 64 + i * 32 + fr;
        const int4 y0 = *reinterpret_cast<const int4*>(Ws + rb * BK + 16 * (c0 ^ (rb & 7)));
        const int4 y1 = *reinterpret_cast<const int4*>(Ws + rb * BK + 16 * (c1 ^ (rb & 7)));
        bf[i] = i32x8{y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
      }
      const int sh = 8 * (2 * s + fh);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
              af[i], bf[j], acc[i][j], 0, 0, 0, (int)((sa[i] >> sh) & 0xFF), 0, (int)((sw[j] >> sh) & 0xFF));
    }
  }

  if (OUT == 2) {
    constexpr int CS = BN + 16;
    uint8_t* Ct = smem;
    uint8_t* Sc = smem + BM2 * CS;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int cl = wn * 64 + j * 32 + fr;
        const float bv = p.bias ? p.bias[n0 + cl] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          float v = act_f<ACT>(acc[i][j][r] + bv) * p.alpha;
          if (p.res && m0 + rl < p.M) v += p.res[(long long)(m0 + rl) * p.ldr + n0 + cl];
          const int sb = mx_scale_byte(group_max<32>(fabsf(v)));
          const float q = clamp_e4m3(v * mx_inv_scale(sb));
          Ct[rl * CS + cl] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(q, q, 0, false) & 0xFF);
          if (fr == 0) Sc[rl * 4 + wn * 2 + j] = (uint8_t)sb;
        }
      }
    }
    __syncthreads();
    uint8_t* out = reinterpret_cast<uint8_t*>(p.out);
#pragma unroll
    for (int c = tid; c < BM2 * BN / 16; c += NT2) {
      const int rl = c >> 3, ch = c & 7;
      if (m0 + rl < p.M)
        *reinterpret_cast<int4*>(out + (long long)(m0 + rl) * p.ldc + n0 + 16 * ch) =
            *reinterpret_cast<const int4*>(Ct + rl * CS + 16 * ch);
    }
    if (tid < BM2 && m0 + tid < p.M)
      *reinterpret_cast<uint32_t*>(p.out_scales + (long long)(m0 + tid) * p.ldso + (n0 >> 5)) =
          *reinterpret_cast<const uint32_t*>(Sc + tid * 4);
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + j * 32 + fr;
      const float bv = p.bias ? p.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        float v = act_f<ACT>(acc[i][j][r] + bv) * p.alpha;
        if (row < p.M) {
          if (p.res) v += p.res[(long long)row * p.ldr + col];
          if (OUT == 1)
            reinterpret_cast<uint16_t*>(p.out)[(long long)row * p.ldc + col] = f32_to_bf16(v);
          else
            reinterpret_cast<float*>(p.out)[(long long)row * p.ldc + col] = v;
        }
      }
    }
  }
}

template <int ACT>
int launch_act(const MxArgs& p, hipStream_t s) {
  if (p.M >= 16 * BM2) {  // enough 256-row tiles to fill the chip
    const long long nt2 = (long long)((p.M + BM2 - 1) / BM2) * (p.N / BN);
    const size_t lds2 = NSTAGE2 * STAGE2;
    switch (p.out_mode) {
      case 0: hipLaunchKernelGGL((mx_gemm256_kernel<ACT, 0>), dim3((unsigned)nt2), dim3(NT2), lds2, s, p); break;
      case 1: hipLaunchKernelGGL((mx_gemm256_kernel<ACT, 1>), dim3((unsigned)nt2), dim3(NT2), lds2, s, p); break;
      default: hipLaunchKernelGGL((mx_gemm256_kernel<ACT, 2>), dim3((unsigned)nt2), dim3(NT2), lds2, s, p); break;
    }
    SBK_CHECK_LAUNCH();
    return 0;
  }
  const long long nt = (long long)((p.M + BM - 1) / BM) * (p.N / BN);
  const size_t lds = 2 * STAGE;
  switch (p.out_mode) {
    case 0: hipLaunchKernelGGL((mx_gemm_kernel<ACT, 0>), dim3((unsigned)nt), dim3(NT), lds, s, p); break;
    case 1: hipLaunchKernelGGL((mx_gemm_kernel<ACT, 1>), dim3((unsigned)nt), dim3(NT), lds, s, p); break;
    default: hipLaunchKernelGGL((mx_gemm_kernel<ACT, 2>), dim3((unsigned)nt), dim3(NT), lds, s, p); break;
  }
  SBK_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// C = epi(A · Wᵀ), MXFP8 operands (see header).  Requirements: K % 128 == 0,
// N % 128 == 0, 16-B aligned A/W rows (lda, a_bs, ldw % 16 == 0) and 4-B
// aligned scale rows (ldsa, s_bs, ldsw % 4 == 0).  rpb = rows per batch for
// the conv addressing (rpb >= M for a plain GEMM).  Row m < M only: rows of
// the last tile beyond M are loaded from row M-1 and not stored.
static int mx_gemm_impl(const uint8_t* A, const uint8_t* SA, long long lda, long long ldsa, long long rpb,
                        long long a_bs, long long s_bs, const uint8_t* W, const uint8_t* SW, long long ldw,
                        long long ldsw, int M, int N, int K, const float* bias, int act, float alpha, const float* res,
                        long long ldr, void* out, long long ldc, int out_mode, uint8_t* out_scales, long long ldso,
                        float* ws, long long ws_floats, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (K % BK) || (N % BN) || rpb <= 0) return SBK_ERR_ARG;
  if ((lda | a_bs | ldw) & 15) return SBK_ERR_ARG;
  if ((ldsa | s_bs | ldsw) & 3) return SBK_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(W)) & 15) return SBK_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(SA) | reinterpret_cast<uintptr_t>(SW)) & 3) return SBK_ERR_ARG;
  if (out_mode == 2 && (!out_scales || (ldc & 15) || (ldso & 3) ||
                        ((reinterpret_cast<uintptr_t>(out) & 15) | (reinterpret_cast<uintptr_t>(out_scales) & 3))))
    return SBK_ERR_ARG;
  if (act != 0 && act != 3 && act != 4) return SBK_ERR_ARG;
  MxArgs p{A, SA, lda, ldsa, rpb, a_bs, s_bs, W, SW, ldw, ldsw, M, N, K, bias, act, alpha, res, ldr,
           out, ldc, out_mode, out_scales, ldso};
  hipStream_t s = (hipStream_t)stream;
  // the 256 x 256 multi-phase kernel (gemm256.hip) when it fills the chip:
  // 1.1-1.5x these kernels on config 5's shapes (profiles/r05c_mx256.log)
  if (ldr <= 0x7fffffffLL && ldc <= 0x7fffffffLL && (long long)((M + 255) / 256) * (N / 256) >= 180) {
    const Gemm256Epi ep{bias, act, 0.f, res, (int)ldr, alpha, nullptr, out, (int)ldc, out_mode == 1};
    if (mx256_supported(M, N, K, lda, ldsa, rpb, a_bs, s_bs, ldw, ldsw, A, SA, W, SW, ep, out_mode, out_scales))
      return mx256_launch(A, SA, lda, ldsa, rpb, a_bs, s_bs, W, SW, ldw, ldsw, M, N, K, ep, out_mode, out_scales, ldso,
                          s, ws, ws_floats);
  }
  if (act == 4) return launch_act<4>(p, s);
  if (act == 3) return launch_act<3>(p, s);
  return launch_act<0>(p, s);
}

SBK_API int sbk_mx_gemm(const uint8_t* A, const uint8_t* SA, long long lda, long long ldsa, long long rpb,
                        long long a_bs, long long s_bs, const uint8_t* W, const uint8_t* SW, long long ldw,
                        long long ldsw, int M, int N, int K, const float* bias, int act, float alpha, const float* res,
                        long long ldr, void* out, long long ldc, int out_mode, uint8_t* out_scales, long long ldso,
                        void* stream) {
  return mx_gemm_impl(A, SA, lda, ldsa, rpb, a_bs, s_bs, W, SW, ldw, ldsw, M, N, K, bias, act, alpha, res, ldr, out,
                      ldc, out_mode, out_scales, ldso, nullptr, 0, stream);
}

// sbk_mx_gemm with an fp32 workspace for the 256-tile kernel's split-K tail
// (gemm256.hip split_tail): ws_floats >= sbk_mx_gemm_ws_floats(M, N, K,
// out_mode) enables it, a smaller or null ws runs whole tiles
SBK_API long long sbk_mx_gemm_ws_floats(int M, int N, int K, int out_mode) {
  if ((long long)((M + 255) / 256) * (N / 256) < 180) return 0;  // sbk_mx_gemm's 256-tile threshold
  return mx256_split_floats(M, N, K, out_mode);
}

SBK_API int sbk_mx_gemm_ws(const uint8_t* A, const uint8_t* SA, long long lda, long long ldsa, long long rpb,
                           long long a_bs, long long s_bs, const uint8_t* W, const uint8_t* SW, long long ldw,
                           long long ldsw, int M, int N, int K, const float* bias, int act, float alpha,
                           const float* res, long long ldr, void* out, long long ldc, int out_mode,
                           uint8_t* out_scales, long long ldso, float* ws, long long ws_floats, void* stream) {
  if (ws_floats < 0 || (ws_floats > 0 && (!ws || (reinterpret_cast<uintptr_t>(ws) & 15)))) return SBK_ERR_ARG;
  return mx_gemm_impl(A, SA, lda, ldsa, rpb, a_bs, s_bs, W, SW, ldw, ldsw, M, N, K, bias, act, alpha, res, ldr, out,
                      ldc, out_mode, out_scales, ldso, ws, ws_floats, stream);
}

// MXFP8 quantisation of a row-major fp32 / bf16 matrix (M, K), K % 32 == 0:
// q (M, ldq bytes) e4m3 and scales (M, ldsq bytes), one per 32 columns.
// Used for weights (once, cached by the modules) and any operand that has
// no fused producer.
namespace {
__global__ void __launch_bounds__(256) mx_quant_kernel(const void* __restrict__ x, int in_bf16, long long ldx, int M,
                                                       int K, uint8_t* __restrict__ q, long long ldq,
                                                       uint8_t* __restrict__ sc, long long ldsq) {
  // one 32-element block per lane: 8 blocks per 256-thread row segment
  const long long nb = (long long)M * (K / 32);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (long long)gridDim.x * blockDim.x) {
    const int row = (int)(i / (K / 32)), blk = (int)(i % (K / 32));
    float v[32];
    if (in_bf16) {
      const uint16_t* xr = reinterpret_cast<const uint16_t*>(x) + (long long)row * ldx + blk * 32;
#pragma unroll
      for (int j = 0; j < 32; ++j) v[j] = bf16_to_f32(xr[j]);
    } else {
      const float* xr = reinterpret_cast<const float*>(x) + (long long)row * ldx + blk * 32;
#pragma unroll
      for (int j = 0; j < 32; ++j) v[j] = xr[j];
    }
    float am = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) am = fmaxf(am, fabsf(v[j]));
    const int sb = mx_scale_byte(am);
    const float inv = mx_inv_scale(sb);
    uint32_t* qr = reinterpret_cast<uint32_t*>(q + (long long)row * ldq + blk * 32);
#pragma unroll
    for (int j = 0; j < 32; j += 4) qr[j / 4] = pack4_e4m3(v[j] * inv, v[j + 1] * inv, v[j + 2] * inv, v[j + 3] * inv);
    sc[(long long)row * ldsq + blk] = (uint8_t)sb;
  }
}

__global__ void mx_dequant_kernel(const uint8_t* __restrict__ q, long long ldq, const uint8_t* __restrict__ sc,
                                  long long ldsq, int M, int K, float* __restrict__ out) {
  const long long n = (long long)M * K;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int row = (int)(i / K), c = (int)(i % K);
    out[i] = e4m3_to_f32(q[(long long)row * ldq + c]) * ldexpf(1.f, (int)sc[(long long)row * ldsq + c / 32] - 127);
  }
}
}  // namespace

SBK_API int sbk_mx_quant(const void* x, int in_bf16, long long ldx, int M, int K, uint8_t* q, long long ldq,
                         uint8_t* scales, long long ldsq, void* stream) {
  if (M <= 0 || K <= 0 || (K % 32)) return SBK_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(q) & 3) || (ldq & 3)) return SBK_ERR_ARG;
  const long long nb = (long long)M * (K / 32);
  long long g = (nb + 255) / 256;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(mx_quant_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, x, in_bf16, ldx, M, K, q,
                     ldq, scales, ldsq);
  SBK_CHECK_LAUNCH();
  return 0;
}

// fp32 value of an MXFP8 matrix (tests / reference checks only)
SBK_API int sbk_mx_dequant(const uint8_t* q, long long ldq, const uint8_t* scales, long long ldsq, int M, int K,
                           float* out, void* stream) {
  if (M <= 0 || K <= 0 || (K % 32)) return SBK_ERR_ARG;
  long long g = ((long long)M * K + 255) / 256;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(mx_dequant_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, q, ldq, scales, ldsq, M,
                     K, out);
  SBK_CHECK_LAUNCH();
  return 0;
}
