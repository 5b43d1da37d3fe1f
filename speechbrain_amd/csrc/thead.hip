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

constexpr int TH_BM = 64, TH_BN = 64, TH_BK = 64, TH_NT = 256, TH_NB = 3;

struct TheadArgs {
  const float* tn;    // (B, T, J) fp32
  const float* pn;    // (B, U1, J) fp32
  const bf16_t* w;    // (V, J) bf16
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

__device__ __forceinline__ float th_act(int act, float v, float slope) {
  if (act == 3) return v >= 0.f ? v : v * slope;
  if (act == 5) return tanhf(v);
  if (act == 6) return v > 0.f ? v : 0.f;
  return v;
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
  uint4 q;
  q.x = (uint32_t)f32_to_bf16(th_act(act, t0.x + p0.x, slope)) | ((uint32_t)f32_to_bf16(th_act(act, t0.y + p0.y, slope)) << 16);
  q.y = (uint32_t)f32_to_bf16(th_act(act, t0.z + p0.z, slope)) | ((uint32_t)f32_to_bf16(th_act(act, t0.w + p0.w, slope)) << 16);
  q.z = (uint32_t)f32_to_bf16(th_act(act, t1.x + p1.x, slope)) | ((uint32_t)f32_to_bf16(th_act(act, t1.y + p1.y, slope)) << 16);
  q.w = (uint32_t)f32_to_bf16(th_act(act, t1.z + p1.z, slope)) | ((uint32_t)f32_to_bf16(th_act(act, t1.w + p1.w, slope)) << 16);
  return q;
}

// 4 waves; wave w owns columns w*16 .. +15 of each 64-column V chunk and all
// 64 rows (4 m-tiles): a lane holds S[4g + r + 16 mt][v = fr] (16 rows of one
// column), so a row's reductions over the chunk are 16-lane DPP reductions
// and the 4 waves' partial (max, sum) merge once, after the last chunk.
template <int MODE>
__global__ void __launch_bounds__(TH_NT) thead_kernel(TheadArgs a) {
  constexpr int BM = TH_BM, BN = TH_BN, BK = TH_BK, NB = TH_NB, MTL = BM / 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int J = a.J;
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);  // BM x J, 16-B chunk c of row r at c ^ (r & 15)
  bf16_t* ring = As + BM * J;                    // NB x BN x BK, chunk c of row r at c ^ ((r >> 1) & 7)
  float* capb = reinterpret_cast<float*>(ring + NB * BN * BK);  // MODE 0: blank / label logits, (max, sum) x 4 waves
  float* capl = capb + BM;
  float* redm = capl + BM;
  float* reds = redm + 4 * BM;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * BM;
  const int KS = J / BK, NVC = a.Vp / BN, NS = KS * NVC;
  const int Um = a.U1 - 1;

  // ---- W tile s (V chunk s / KS, k step s % KS) -> ring slot s % NB:
  // 8 KB = 8 pieces of 8 rows; wave w issues pieces w and w + 4
  const int lrow = lane >> 3, lchk = lane & 7;
  auto issue = [&](int s) __attribute__((always_inline)) {
    const int vc = s / KS, ks = s - vc * KS;
    bf16_t* dst = ring + (s % NB) * BN * BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = i * 4 + w, r = p * 8 + lrow;
      const int v = min(vc * BN + r, a.V - 1);
      const bf16_t* src = a.w + (long long)v * J + ks * BK + ((lchk ^ ((r >> 1) & 7)) << 3);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(dst + p * 8 * BK), 16, 0, 0);
    }
  };
  issue(0);
  issue(1);  // NS = (J / 64) * (Vp / 64) >= 4

  // ---- z rows of the tile -> LDS (rows past M clamp; never stored)
  {
    const int CPR = J / 8;
#pragma unroll 4
    for (int c = tid; c < BM * CPR; c += TH_NT) {
      const int r = c / CPR, ch = c - r * CPR;
      const int row = min(m0 + r, a.M - 1);
      const int u = row % a.U1, bt = row / a.U1, b = bt / a.T;
      const uint4 q = z8(a.tn + (long long)bt * J + ch * 8, a.pn + ((long long)b * a.U1 + u) * J + ch * 8, a.act,
                         a.slope);
      *reinterpret_cast<uint4*>(As + r * J + ((ch ^ (r & 15)) << 3)) = q;
    }
  }
  // this lane's rows: labels (and the dlogits coefficients)
  int yl[MTL][4];
  float lsev[MTL][4], cbv[MTL][4], clv[MTL][4], mx[MTL][4], sm[MTL][4];
#pragma unroll
  for (int mt = 0; mt < MTL; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = min(m0 + mt * 16 + 4 * g + r, a.M - 1);
      const int u = row % a.U1, b = row / (a.T * a.U1);
      yl[mt][r] = u < Um ? a.labels[b * Um + u] : -1;
      mx[mt][r] = -INFINITY;
      sm[mt][r] = 0.f;
      if (MODE == 1) {
        const float sc = a.scale[a.scale_per_b ? b : 0];
        lsev[mt][r] = a.lse_in[row];
        cbv[mt][r] = a.gb[row] * sc;
        clv[mt][r] = a.gl[row] * sc;
      }
    }
  if (MODE == 0 && tid < BM) {
    capb[tid] = __builtin_nanf("");
    capl[tid] = __builtin_nanf("");
  }
  __syncthreads();

  f32x4 acc[MTL];
#pragma unroll
  for (int mt = 0; mt < MTL; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  bool stored = false;  // MODE 1: the previous step issued this thread's two dS stores
  for (int s = 0; s < NS; ++s) {
    // this wave's pieces of tile s landed (tile s+1 in flight; after a chunk
    // end in MODE 1 also the two dS stores issued behind it)
    if (s + 1 >= NS)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (MODE == 1 && stored)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    stored = false;
    if (s + 2 < NS) issue(s + 2);  // into the slot read at step s-1
    const int vc = s / KS, ks = s - vc * KS;
    const bf16_t* tile = ring + (s % NB) * BN * BK;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int br = w * 16 + fr;
      const bf16x8 fb = ld8(tile + br * BK + (((kk * 4 + g) ^ ((br >> 1) & 7)) << 3));
      const int ch = ks * 8 + kk * 4 + g;
#pragma unroll
      for (int mt = 0; mt < MTL; ++mt) {
        const bf16x8 fa = ld8(As + (mt * 16 + fr) * J + ((ch ^ fr) << 3));
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[mt], 0, 0, 0);
      }
    }
    if (ks != KS - 1) continue;
    // ---- V chunk vc complete: S[rows][v], v = vc*BN + w*16 + fr
    const int v = vc * BN + w * 16 + fr;
    const bool valid = v < a.V;
    if (MODE == 0) {
#pragma unroll
      for (int mt = 0; mt < MTL; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = valid ? acc[mt][r] : -INFINITY;
          const float nm = fmaxf(mx[mt][r], row16_max(x));
          if (nm != -INFINITY) {
            const float e = valid ? __expf(x - nm) : 0.f;
            sm[mt][r] = sm[mt][r] * __expf(mx[mt][r] - nm) + row16_sum(e);
            mx[mt][r] = nm;
          }
          const int lr = mt * 16 + 4 * g + r;
          if (v == a.blank) {
            const uint32_t la = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) float*)(capb + lr));
            asm volatile("ds_write_b32 %0, %1" ::"v"(la), "v"(acc[mt][r]) : "memory");
          }
          if (valid && v == yl[mt][r]) {
            const uint32_t la = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) float*)(capl + lr));
            asm volatile("ds_write_b32 %0, %1" ::"v"(la), "v"(acc[mt][r]) : "memory");
          }
        }
    } else {
      // dS in bf16 -> the slot just read (free once every wave is past its
      // fragment reads) -> 16-B row stores; the slot is refilled only after
      // the next step's barrier, behind these reads
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      bf16_t* scr = ring + (s % NB) * BN * BK;  // BM x BN, linear
#pragma unroll
      for (int mt = 0; mt < MTL; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float d = 0.f;
          if (valid) {
            const float p = __expf(acc[mt][r] - lsev[mt][r]);
            d = (v == a.blank ? cbv[mt][r] : 0.f) + (v == yl[mt][r] ? clv[mt][r] : 0.f) -
                p * (cbv[mt][r] + clv[mt][r]);
          }
          const int lr = mt * 16 + 4 * g + r;
          const uint32_t la =
              (uint32_t)(uintptr_t)((__attribute__((address_space(3))) bf16_t*)(scr + lr * BN + w * 16 + fr));
          const uint32_t hv = f32_to_bf16(d);
          asm volatile("ds_write_b16 %0, %1" ::"v"(la), "v"(hv) : "memory");
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const bool full = m0 + BM <= a.M;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = tid + i * TH_NT, lr = c >> 3, chk = c & 7;
        const uint32_t la = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) bf16_t*)(scr + lr * BN + chk * 8));
        uint4 q;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(q) : "v"(la) : "memory");
        if (m0 + lr < a.M)
          *reinterpret_cast<uint4*>(a.ds + (long long)(m0 + lr) * a.Vp + vc * BN + chk * 8) = q;
      }
      stored = full && s + 1 < NS;
    }
#pragma unroll
    for (int mt = 0; mt < MTL; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (MODE == 1) return;
  // ---- merge the 4 waves' (max, sum) per row; lse and the two log-probs
  if (fr == 0) {
#pragma unroll
    for (int mt = 0; mt < MTL; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        redm[w * BM + mt * 16 + 4 * g + r] = mx[mt][r];
        reds[w * BM + mt * 16 + 4 * g + r] = sm[mt][r];
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < BM && m0 + tid < a.M) {
    const int row = m0 + tid;
    float M = -INFINITY;
#pragma unroll
    for (int k = 0; k < 4; ++k) M = fmaxf(M, redm[k * BM + tid]);
    float S = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) S += reds[k * BM + tid] * __expf(redm[k * BM + tid] - M);
    const float l = M + logf(S);
    const int u = row % a.U1;
    a.lse[row] = l;
    a.lpb[row] = capb[tid] - l;
    // label outside [0, V): NaN (the capture never happened), as gather_kernel
    a.lpl[row] = u < Um ? capl[tid] - l : 0.f;
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
      const float4 t0 = tv[i][0], t1 = tv[i][1];
      uint4 q;
      q.x = (uint32_t)f32_to_bf16(th_act(act, t0.x + p0.x, slope)) | ((uint32_t)f32_to_bf16(th_act(act, t0.y + p0.y, slope)) << 16);
      q.y = (uint32_t)f32_to_bf16(th_act(act, t0.z + p0.z, slope)) | ((uint32_t)f32_to_bf16(th_act(act, t0.w + p0.w, slope)) << 16);
      q.z = (uint32_t)f32_to_bf16(th_act(act, t1.x + p1.x, slope)) | ((uint32_t)f32_to_bf16(th_act(act, t1.y + p1.y, slope)) << 16);
      q.w = (uint32_t)f32_to_bf16(th_act(act, t1.z + p1.z, slope)) | ((uint32_t)f32_to_bf16(th_act(act, t1.w + p1.w, slope)) << 16);
      *reinterpret_cast<uint4*>(Zt + r * WG_LD + cc) = q;
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

size_t thead_lds(int J, int mode) {
  return (size_t)TH_BM * J * 2 + (size_t)TH_NB * TH_BN * TH_BK * 2 + (mode == 0 ? (size_t)10 * TH_BM * 4 : 0);
}

template <int MODE>
int launch_thead(const TheadArgs& a, hipStream_t s) {
  const size_t lds = thead_lds(a.J, MODE);
  if (lds > 160 * 1024) return SBK_ERR_ARG;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&thead_kernel<MODE>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL((thead_kernel<MODE>), dim3((a.M + TH_BM - 1) / TH_BM), dim3(TH_NT), lds, s, a);
  SBK_CHECK_LAUNCH();
  return 0;
}

int thead_check(const float* tn, const float* pn, const void* w, const int* labels, int B, int T, int U1, int J,
                int V, int blank, int act) {
  if (!tn || !pn || !w || !labels || B <= 0 || T <= 0 || U1 <= 0 || V <= 0 || blank < 0 || blank >= V)
    return SBK_ERR_ARG;
  if (J <= 0 || J % 128 || J > 1024) return SBK_ERR_ARG;
  if (act != 0 && act != 3 && act != 5 && act != 6) return SBK_ERR_ARG;
  if ((long long)B * T * U1 > 0x7fffffffLL / 2) return SBK_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(tn) | reinterpret_cast<uintptr_t>(pn) | reinterpret_cast<uintptr_t>(w)) & 15)
    return SBK_ERR_ARG;
  return 0;
}

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
  a.slope = slope; a.M = B * T * U1;
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
  a.slope = slope; a.M = B * T * U1;
  a.lse_in = lse; a.gb = gb; a.gl = gl; a.scale = scale; a.scale_per_b = scale_per_b;
  a.ds = reinterpret_cast<bf16_t*>(ds);
  return launch_thead<1>(a, (hipStream_t)stream);
}

SBK_API int sbk_thead_wgrad(const void* ds, const float* tn, const float* pn, const int* Tl, int B, int T, int U1,
                            int J, int V, int act, float slope, float* dw, void* stream) {
  if (!ds || !tn || !pn || !Tl || !dw || B <= 0 || T <= 0 || U1 <= 0 || V <= 0) return SBK_ERR_ARG;
  if (J <= 0 || J % 128 || (long long)T * U1 > (1 << 24)) return SBK_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(ds) | reinterpret_cast<uintptr_t>(tn) | reinterpret_cast<uintptr_t>(pn)) & 15)
    return SBK_ERR_ARG;
  const size_t lds = (size_t)2 * WG_BK * WG_LD * 2 + (size_t)U1 * WG_BJ * 4;
  if (lds > 160 * 1024) return SBK_ERR_ARG;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&thead_wgrad_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  const int Vp = sbk_thead_vpad(V);
  hipLaunchKernelGGL(thead_wgrad_kernel, dim3(Vp / WG_BV, J / WG_BJ, B), dim3(256), lds, (hipStream_t)stream,
                     reinterpret_cast<const bf16_t*>(ds), Vp, tn, pn, Tl, T, U1, J, V, act, slope, dw);
  SBK_CHECK_LAUNCH();
  return 0;
}
