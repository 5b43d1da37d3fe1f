// Fused transducer head: joint ("sum" + nonlinearity) -> output projection
// (Linear J -> V, no bias) -> log-softmax -> RNN-T log-prob gather, and the
// backward of the same chain, without the (B, T, U1, V) logits or their fp32
// gradient ever existing in HBM.
//
// Reference chain (the LibriSpeech transducer recipe):
//   speechbrain/nnet/transducer/transducer_joint.py:57-95  z = act(tn + pn)
//   speechbrain/nnet/linear.py (transducer_lin, bias=False)  logits = z W^T
//   speechbrain/nnet/losses.py:27-85 (log_softmax) and
//   speechbrain/nnet/loss/transducer_loss.py:31-236 (gather, α/β, gradients).
//
// Kernels (rows r = (b, t, u) of the lattice, M = B*T*U1; Vp = V rounded up
// to 128, columns >= V masked):
//   thead_kernel<0>  per 64-row tile: z rows generated once into LDS (bf16,
//                    the autocast operand), W streamed by LDS-DMA in 64x64
//                    tiles through a 3-slot ring, S = z W^T on MFMA in fp32,
//                    online max / sum-exp over the V chunks -> lse, and the
//                    logits at blank / label -> log-probs for the lattice.
//   thead_kernel<1>  the same recompute with lse known -> dS = ∂L/∂logits
//                    = g·softmax - onehots (the dense_grad of rnnt.hip) in
//                    bf16 (M, Vp): the only (rows x V) tensor, half the size
//                    of the fp32 logits it replaces, consumed by
//                      dZ = dS W      (sbk_gemm, then sbk_joint_bwd)
//   thead_wgrad      dW = dS^T Z: one workgroup per (128 v x 128 j) tile of
//                    one utterance, z regenerated (pn rows of the utterance
//                    resident in LDS), both operands read k-transposed
//                    (ds_read_b64_tr_b16), fp32 atomics into dW.
#include "mfma.h"

using namespace sbk;

namespace {

// 96 KB of W ring: 6 slots of 128 vocabulary rows x 64 k (16 KB)
constexpr int TH_BM = 128, TH_BN = 128, TH_BK = 64, TH_NT = 512, TH_NB = 12 * 64 / TH_BN;

struct TheadArgs {
  const float* tn;    // (B, T, J) fp32
  const float* pn;    // (B, U1, J) fp32
  const bf16_t* w;    // (Vp, J) bf16, rows >= V zero
  const int* labels;  // (B, U1 - 1)
  int B, T, U1, J, V, Vp, blank, act;
  float slope;
  int M;
  float *lse, *lpb, *lpl;          // forward outputs (M)
  const float *lse_in, *gb, *gl;   // dlogits inputs (M)
  const float* scale;
  int scale_per_b;
  bf16_t* ds;  // (M, Vp)
};

// The joint nonlinearities of the fused head are all one branch-free form,
// v >= 0 ? v : v * slope, with slope 1 (identity), 0 (ReLU) or the
// LeakyReLU slope: the host maps the act code (tanh stays on the
// materialised path).
// act(t + p) of 8 values packed to bf16 (round to nearest even): packed fp32
// adds / multiplies, leaky as max(v, slope v) (host: slope <= 1), and
// v_cvt_pk_bf16_f32 — ~3 VALU per value instead of ~10 with the scalar
// select and the software rounding of f32_to_bf16.
__device__ __forceinline__ uint4 zpack8(float4 t0, float4 t1, float4 p0, float4 p1, float slope) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  const f2 v[4] = {f2{t0.x, t0.y} + f2{p0.x, p0.y}, f2{t0.z, t0.w} + f2{p0.z, p0.w},
                   f2{t1.x, t1.y} + f2{p1.x, p1.y}, f2{t1.z, t1.w} + f2{p1.z, p1.w}};
  uint32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f2 s = v[i] * slope;
    q[i] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{fmaxf(v[i][0], s[0]), fmaxf(v[i][1], s[1])}, b2));
  }
  return uint4{q[0], q[1], q[2], q[3]};
}

__device__ __forceinline__ bf16x8 ld8(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// max / sum over the 16 lanes of a DPP row (one column group of a 16x16 tile)
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f32<0x140>(v));
  v = fmaxf(v, dpp_f32<0x141>(v));
  v = fmaxf(v, dpp_f32<0x4E>(v));
  return fmaxf(v, dpp_f32<0xB1>(v));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f32<0x140>(v);
  v += dpp_f32<0x141>(v);
  v += dpp_f32<0x4E>(v);
  return v + dpp_f32<0xB1>(v);
}

// 8 z values of row r, columns j .. j+7, packed bf16 (the GEMM operand)
__device__ __forceinline__ uint4 z8(const float* tp, const float* pp, int act, float slope) {
  const float4 t0 = *reinterpret_cast<const float4*>(tp), t1 = *reinterpret_cast<const float4*>(tp + 4);
  const float4 p0 = *reinterpret_cast<const float4*>(pp), p1 = *reinterpret_cast<const float4*>(pp + 4);
  return zpack8(t0, t1, p0, p1, slope);
}

// vmcnt(n) for a run-time n (the number of younger vector-memory operations
// a wait may leave outstanding); immediates only exist per value
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
#define SBK_VM(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    SBK_VM(0) SBK_VM(1) SBK_VM(2) SBK_VM(3) SBK_VM(4) SBK_VM(5) SBK_VM(6) SBK_VM(7) SBK_VM(8) SBK_VM(9) SBK_VM(10)
    SBK_VM(11) SBK_VM(12) SBK_VM(13) SBK_VM(14) SBK_VM(15) SBK_VM(16) SBK_VM(17) SBK_VM(18) SBK_VM(19) SBK_VM(20)
    SBK_VM(21) SBK_VM(22) SBK_VM(23) SBK_VM(24) SBK_VM(25) SBK_VM(26) SBK_VM(27) SBK_VM(28)
#undef SBK_VM
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// 8 waves x 16 rows = 128 rows per workgroup.  Wave w holds the z fragments
// of its 16 rows for the whole K = J in VGPRs (J / 32 x 4 registers,
// generated once from tn / pn), so LDS holds only the W stream: 128 x 64
// tiles (16 KB) through a 6-slot ring, 5 tiles (80 KB) in flight, one
// barrier per step.  MODE 0: a lane holds S[w*16 + 4g + r][t*16 + fr] for
// the 8 column tiles t of the 128-column V chunk, so a row's reductions are
// in-lane over t plus one 16-lane DPP reduction, and no cross-wave merge is
// needed.  MODE 1 swaps the MFMA operands (D[v][m]): a lane holds 4
// consecutive v of one row and stores them as one 8-B bf16 quad.
// Measured at config 4 (M = 782080, J = 1024, V = 1000): fwd 2.61 ms
// (614 TF/s), dlogits 2.66 ms; 64-column chunks (12 x 8 KB ring) 3.00 /
// 4.42 ms; the first version (64-row tiles, z in LDS, 3-slot ring) 8.97 /
// 7.26 ms.
template <int MODE, int JK>
__global__ void __launch_bounds__(TH_NT) thead_kernel(TheadArgs a) {
  constexpr int J = JK * 32, BN = TH_BN, BK = TH_BK, NB = TH_NB, DEPTH = NB - 1, NTL = BN / 16;
  constexpr int KS = J / BK;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);           // NB x BN x BK, chunk c of row r at c ^ ((r >> 1) & 7)

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * TH_BM;
  const int NS = KS * (a.Vp / BN);
  const int Um = a.U1 - 1;

  // ---- W tile s (V chunk s / KS, k step s % KS) -> slot s % NB: BN / 8
  // pieces of 8 rows x 128 B; wave w issues pieces w, w + 8, ...
  constexpr int PPW = BN / 64;  // pieces per wave per tile
  static_assert(PPW * 64 == BN, "whole pieces per wave");
  // (w has Vp rows, the padding zero: no clamp, so the per-lane source is one
  // base pointer plus a wave-uniform offset)
  const bf16_t* wlane = a.w + (long long)(w * 8 + (lane >> 3)) * J + (((lane & 7) ^ (((w * 8 + (lane >> 3)) >> 1) & 7)) << 3);
  auto issue = [&](int s) __attribute__((always_inline)) {
    const int vc = s / KS, ks = s - vc * KS;
    bf16_t* dst = ring + (s % NB) * BN * BK;
#pragma unroll
    for (int i = 0; i < PPW; ++i)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(wlane + ((long long)(vc * BN + 64 * i) * J + ks * BK)),
          (__attribute__((address_space(3))) void*)(dst + (w * 8 + 64 * i) * BK), 16, 0, 0);
  };
#pragma unroll
  for (int s = 0; s < DEPTH; ++s)
    if (s < NS) issue(s);

  // ---- z fragments of row w*16 + fr, k = 32 kk + 8 g .. +7 (rows past M clamp)
  bf16x8 za[JK];
  {
    const int row = min(m0 + w * 16 + fr, a.M - 1);
    const int u = row % a.U1, bt = row / a.U1, b = bt / a.T;
    const float* tp = a.tn + (long long)bt * J + 8 * g;
    const float* pp = a.pn + ((long long)b * a.U1 + u) * J + 8 * g;
#pragma unroll
    for (int kk = 0; kk < JK; ++kk) {
      const uint4 q = z8(tp + 32 * kk, pp + 32 * kk, a.act, a.slope);
      za[kk] = *reinterpret_cast<const bf16x8*>(&q);
      // bound the loads hoisted ahead of their conversions (register
      // pressure: za alone is 4*JK VGPRs): fragment kk is final here
      if (kk % 2 == 1) asm volatile("" : "+v"(za[kk]), "+v"(za[kk - 1])::"memory");
    }
  }
  // this lane's 4 rows w*16 + 4g + r: labels, running (max, sum) / dS coefficients
  int yl[4];
  float mx[4], sm[4], capb[4], capl[4], lsev[4], cbv[4], clv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = min(m0 + w * 16 + 4 * g + r, a.M - 1);
    const int u = row % a.U1, b = row / (a.T * a.U1);
    yl[r] = u < Um ? a.labels[b * Um + u] : -1;
    mx[r] = -INFINITY;
    sm[r] = 0.f;
    capb[r] = capl[r] = -INFINITY;
  }
  // MODE 1 computes D[v][m] (operands swapped): the lane's one row is w*16 + fr
  int y1 = -1;
  if (MODE == 1) {
    const int row = min(m0 + w * 16 + fr, a.M - 1);
    const int u = row % a.U1, b = row / (a.T * a.U1);
    const float sc = a.scale[a.scale_per_b ? b : 0];
    y1 = u < Um ? a.labels[b * Um + u] : -1;
    lsev[0] = a.lse_in[row];
    cbv[0] = a.gb[row] * sc;
    clv[0] = a.gl[row] * sc;
  }
  const bool full = m0 + TH_BM <= a.M;  // MODE 1: every dS store of the workgroup is issued (NTL per chunk)

  f32x4 acc[NTL];
#pragma unroll
  for (int t = 0; t < NTL; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int vc = 0; vc < NS / KS; ++vc) {
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int s = vc * KS + ks;
    // this wave's pieces of tile s landed: younger are the tiles issued
    // after it and (MODE 1) the 4 dS stores of every chunk end since then
    {
      int younger = PPW * min(DEPTH - 1, NS - 1 - s);
      if (MODE == 1 && full)
        for (int e = max(0, s - DEPTH); e < s; ++e) younger += (e % KS == KS - 1) ? NTL : 0;
      wait_vm(younger);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + DEPTH < NS) issue(s + DEPTH);  // into the slot read at step s-1
    const bf16_t* tile = ring + (s % NB) * BN * BK;
#pragma unroll
    for (int h = 0; h < BK / 32; ++h) {
      bf16x8 fb[NTL];
#pragma unroll
      for (int t = 0; t < NTL; ++t) {
        const int br = t * 16 + fr;
        fb[t] = ld8(tile + br * BK + (((h * 4 + g) ^ ((br >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int t = 0; t < NTL; ++t)
        acc[t] = MODE == 0 ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(za[ks * 2 + h], fb[t], acc[t], 0, 0, 0)
                           : __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[t], za[ks * 2 + h], acc[t], 0, 0, 0);
    }
  }
    // ---- V chunk vc complete: lane holds S[rows 4g + r][v = vc*BN + t*16 + fr]
    if (MODE == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float cm = -INFINITY;
#pragma unroll
        for (int t = 0; t < NTL; ++t) {
          const int v = vc * BN + t * 16 + fr;
          if (v < a.V) cm = fmaxf(cm, acc[t][r]);
          if (v == a.blank) capb[r] = acc[t][r];
          if (v < a.V && v == yl[r]) capl[r] = acc[t][r];
        }
        const float nm = fmaxf(mx[r], row16_max(cm));
        if (nm != -INFINITY) {
          float e = 0.f;
#pragma unroll
          for (int t = 0; t < NTL; ++t) {
            const int v = vc * BN + t * 16 + fr;
            e += v < a.V ? __expf(acc[t][r] - nm) : 0.f;
          }
          sm[r] = sm[r] * __expf(mx[r] - nm) + row16_sum(e);
          mx[r] = nm;
        }
      }
    } else {
      // lane holds dS rows v = vc*BN + t*16 + 4g .. +3 of row m = w*16 + fr:
      // one 8-B store of 4 bf16 per tile (a row's 64 columns from 16 lanes)
      const int row = m0 + w * 16 + fr;
#pragma unroll
      for (int t = 0; t < NTL; ++t) {
        const int v0 = vc * BN + t * 16 + 4 * g;
        float d[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int v = v0 + r;
          d[r] = 0.f;
          if (v < a.V) {
            const float p = __expf(acc[t][r] - lsev[0]);
            d[r] = (v == a.blank ? cbv[0] : 0.f) + (v == y1 ? clv[0] : 0.f) - p * (cbv[0] + clv[0]);
          }
        }
        uint2 pk;
        pk.x = pack_bf16x2(d[0], d[1]);
        pk.y = pack_bf16x2(d[2], d[3]);
        if (row < a.M) *reinterpret_cast<uint2*>(a.ds + (long long)row * a.Vp + v0) = pk;
      }
    }
#pragma unroll
    for (int t = 0; t < NTL; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (MODE == 1) return;
  // ---- lse and the two log-probs of this lane's rows (one lane per row writes)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float cb = row16_max(capb[r]), cl = row16_max(capl[r]);
    const int row = m0 + w * 16 + 4 * g + r;
    if (fr == 0 && row < a.M) {
      const float l = mx[r] + logf(sm[r]);
      const int u = row % a.U1;
      a.lse[row] = l;
      a.lpb[row] = cb - l;
      // label outside [0, V): NaN (never captured), as gather_kernel
      a.lpl[row] = u < Um ? (cl == -INFINITY ? __builtin_nanf("") : cl - l) : 0.f;
    }
  }
}

// dW[v][j] += sum over the rows r of utterance b: dS[r][v] * z[r][j].
// grid (Vp / 128, J / 128, B); 4 waves as 2 (v) x 2 (j), 64 x 64 each.  Per
// 64-row step: the dS tile [r][v] and the z tile [r][j] (regenerated from tn
// and the utterance's pn rows, kept in LDS) are register-prefetched one step
// ahead, stored row-major ([r][128 + 16]: conflict-free transposed reads)
// and read k-transposed (ds_read_b64_tr_b16) for both MFMA operands.
constexpr int WG_BV = 128, WG_BJ = 128, WG_BK = 64, WG_LD = 144;

__device__ __forceinline__ bf16x8 frag_tr(const bf16_t* X, int k0, int dbase, int lane) {
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const bf16_t* a0 = X + (k0 + 4 * g + q) * WG_LD + dbase + 4 * p;
  const bf16_t* a1 = a0 + 16 * WG_LD;
  const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4_t*)(a0));
  const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4_t*)(a1));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__global__ void __launch_bounds__(256) thead_wgrad_kernel(const bf16_t* __restrict__ ds, int ldds,
                                                          const float* __restrict__ tn, const float* __restrict__ pn,
                                                          const int* __restrict__ Tl, int T, int U1, int J, int V,
                                                          int act, float slope, float* __restrict__ dw) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* Sd = reinterpret_cast<bf16_t*>(smem);  // WG_BK x WG_LD   dS tile [r][v]
  bf16_t* Zt = Sd + WG_BK * WG_LD;               // WG_BK x WG_LD   z tile [r][j]
  float* pnl = reinterpret_cast<float*>(Zt + WG_BK * WG_LD);  // U1 x 128 pn[b, u, j-tile]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int v0 = blockIdx.x * WG_BV, j0 = blockIdx.y * WG_BJ, b = blockIdx.z;
  const int Tb = min(max(Tl[b], 0), T);
  const long long rbase = (long long)b * T * U1;
  const int nrow = Tb * U1;  // rows t >= Tb carry dS = 0
  for (int i = tid; i < U1 * (WG_BJ / 4); i += 256) {
    const int u = i / (WG_BJ / 4), c4 = i - u * (WG_BJ / 4);
    *reinterpret_cast<float4*>(pnl + u * WG_BJ + 4 * c4) =
        *reinterpret_cast<const float4*>(pn + ((long long)b * U1 + u) * J + j0 + 4 * c4);
  }
  // per thread per step: 4 chunks of 8 of each tile; chunk c -> row c >> 4, cols 8 (c & 15)
  const float u1inv = 1.0f / (float)U1;
  uint4 sv[4];
  float4 tv[4][2];
  auto gload = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + i * 256, rr = k0 + (c >> 4), cc = (c & 15) * 8;
      const int rc = min(rr, nrow - 1);
      sv[i] = rr < nrow ? *reinterpret_cast<const uint4*>(ds + (rbase + rc) * ldds + v0 + cc) : uint4{0u, 0u, 0u, 0u};
      int t = (int)((float)rc * u1inv);
      t -= (t * U1 > rc);
      t += ((t + 1) * U1 <= rc);
      const float* tp = tn + (((long long)b * T + t) * J + j0 + cc);
      tv[i][0] = *reinterpret_cast<const float4*>(tp);
      tv[i][1] = *reinterpret_cast<const float4*>(tp + 4);
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (nrow + WG_BK - 1) / WG_BK;
  if (nk > 0) gload(0);
  __syncthreads();  // pnl
  for (int kt = 0; kt < nk; ++kt) {
    const int k0 = kt * WG_BK;
    // stage step kt (registers -> LDS), then prefetch step kt + 1
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + i * 256, r = c >> 4, cc = (c & 15) * 8;
      const int rc = min(k0 + r, nrow - 1);
      int t = (int)((float)rc * u1inv);
      t -= (t * U1 > rc);
      t += ((t + 1) * U1 <= rc);
      const int u = rc - t * U1;
      const float* pp = pnl + u * WG_BJ + cc;
      const float4 p0 = *reinterpret_cast<const float4*>(pp), p1 = *reinterpret_cast<const float4*>(pp + 4);
      *reinterpret_cast<uint4*>(Zt + r * WG_LD + cc) = zpack8(tv[i][0], tv[i][1], p0, p1, slope);
      *reinterpret_cast<uint4*>(Sd + r * WG_LD + cc) = sv[i];
    }
    __syncthreads();
    if (kt + 1 < nk) gload(k0 + WG_BK);
#pragma unroll
    for (int kk = 0; kk < WG_BK / 32; ++kk) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag_tr(Sd, kk * 32, wm * 64 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag_tr(Zt, kk * 32, wn * 64 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // D[v][j]: lane holds rows v = 4g + r, column j = lane & 15 of each tile
  const int g = lane >> 4, fr = lane & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int v = v0 + wm * 64 + i * 16 + 4 * g + r;
      if (v >= V) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) atomicAdd(dw + (long long)v * J + j0 + wn * 64 + j * 16 + fr, acc[i][j][r]);
    }
}

size_t thead_lds(int mode) {
  (void)mode;
  return (size_t)TH_NB * TH_BN * TH_BK * 2;
}

template <int MODE, int JK>
int launch_thead_j(const TheadArgs& a, hipStream_t s) {
  const size_t lds = thead_lds(MODE);
  if (hipError_t e = sbk::lds_optin(reinterpret_cast<const void*>(&thead_kernel<MODE, JK>), lds)) return (int)e;
  hipLaunchKernelGGL((thead_kernel<MODE, JK>), dim3((a.M + TH_BM - 1) / TH_BM), dim3(TH_NT), lds, s, a);
  SBK_CHECK_LAUNCH();
  return 0;
}

template <int MODE>
int launch_thead(const TheadArgs& a, hipStream_t s) {
  switch (a.J) {
    case 128: return launch_thead_j<MODE, 4>(a, s);
    case 256: return launch_thead_j<MODE, 8>(a, s);
    case 512: return launch_thead_j<MODE, 16>(a, s);
    case 1024: return launch_thead_j<MODE, 32>(a, s);
    default: return SBK_ERR_ARG;
  }
}

int thead_check(const float* tn, const float* pn, const void* w, const int* labels, int B, int T, int U1, int J,
                int V, int blank, int act) {
  if (!tn || !pn || !w || !labels || B <= 0 || T <= 0 || U1 <= 0 || V <= 0 || blank < 0 || blank >= V)
    return SBK_ERR_ARG;
  if (J != 128 && J != 256 && J != 512 && J != 1024) return SBK_ERR_ARG;
  if (act != 0 && act != 3 && act != 6) return SBK_ERR_ARG;
  if ((long long)B * T * U1 > 0x7fffffffLL / 2) return SBK_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(tn) | reinterpret_cast<uintptr_t>(pn) | reinterpret_cast<uintptr_t>(w)) & 15)
    return SBK_ERR_ARG;
  return 0;
}

}  // namespace

namespace {
// leaky slope of the joint activation (identity 1, ReLU 0); the kernels use
// max(v, slope v), exact for slopes <= 1 (entry points reject larger ones)
float act_slope(int act, float slope) { return act == 0 ? 1.f : (act == 6 ? 0.f : slope); }
}  // namespace

SBK_API int sbk_thead_vpad(int V) { return (V + 127) / 128 * 128; }

SBK_API int sbk_thead_fwd(const float* tn, const float* pn, const void* w, const int* labels, int B, int T, int U1,
                          int J, int V, int blank, int act, float slope, float* lse, float* lpb, float* lpl,
                          void* stream) {
  if (int rc = thead_check(tn, pn, w, labels, B, T, U1, J, V, blank, act)) return rc;
  if (!lse || !lpb || !lpl) return SBK_ERR_ARG;
  TheadArgs a{};
  a.tn = tn; a.pn = pn; a.w = reinterpret_cast<const bf16_t*>(w); a.labels = labels;
  a.B = B; a.T = T; a.U1 = U1; a.J = J; a.V = V; a.Vp = sbk_thead_vpad(V); a.blank = blank; a.act = act;
  if (act_slope(act, slope) > 1.f) return SBK_ERR_ARG;
  a.slope = act_slope(act, slope); a.M = B * T * U1;
  a.lse = lse; a.lpb = lpb; a.lpl = lpl;
  return launch_thead<0>(a, (hipStream_t)stream);
}

SBK_API int sbk_thead_dlogits(const float* tn, const float* pn, const void* w, const int* labels, int B, int T, int U1,
                              int J, int V, int blank, int act, float slope, const float* lse, const float* gb,
                              const float* gl, const float* scale, int scale_per_b, void* ds, void* stream) {
  if (int rc = thead_check(tn, pn, w, labels, B, T, U1, J, V, blank, act)) return rc;
  if (!lse || !gb || !gl || !scale || !ds || (reinterpret_cast<uintptr_t>(ds) & 15)) return SBK_ERR_ARG;
  TheadArgs a{};
  a.tn = tn; a.pn = pn; a.w = reinterpret_cast<const bf16_t*>(w); a.labels = labels;
  a.B = B; a.T = T; a.U1 = U1; a.J = J; a.V = V; a.Vp = sbk_thead_vpad(V); a.blank = blank; a.act = act;
  if (act_slope(act, slope) > 1.f) return SBK_ERR_ARG;
  a.slope = act_slope(act, slope); a.M = B * T * U1;
  a.lse_in = lse; a.gb = gb; a.gl = gl; a.scale = scale; a.scale_per_b = scale_per_b;
  a.ds = reinterpret_cast<bf16_t*>(ds);
  return launch_thead<1>(a, (hipStream_t)stream);
}

SBK_API int sbk_thead_wgrad(const void* ds, const float* tn, const float* pn, const int* Tl, int B, int T, int U1,
                            int J, int V, int act, float slope, float* dw, void* stream) {
  if (act_slope(act, slope) > 1.f) return SBK_ERR_ARG;
  if (!ds || !tn || !pn || !Tl || !dw || B <= 0 || T <= 0 || U1 <= 0 || V <= 0) return SBK_ERR_ARG;
  if (act != 0 && act != 3 && act != 6) return SBK_ERR_ARG;
  if (J <= 0 || J % 128 || (long long)T * U1 > (1 << 24)) return SBK_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(ds) | reinterpret_cast<uintptr_t>(tn) | reinterpret_cast<uintptr_t>(pn)) & 15)
    return SBK_ERR_ARG;
  const size_t lds = (size_t)2 * WG_BK * WG_LD * 2 + (size_t)U1 * WG_BJ * 4;
  if (lds > 160 * 1024) return SBK_ERR_ARG;
  if (hipError_t e = sbk::lds_optin(reinterpret_cast<const void*>(&thead_wgrad_kernel), lds)) return (int)e;
  const int Vp = sbk_thead_vpad(V);
  hipLaunchKernelGGL(thead_wgrad_kernel, dim3(Vp / WG_BV, J / WG_BJ, B), dim3(256), lds, (hipStream_t)stream,
                     reinterpret_cast<const bf16_t*>(ds), Vp, tn, pn, Tl, T, U1, J, V, act, act_slope(act, slope), dw);
  SBK_CHECK_LAUNCH();
  return 0;
}
