// Fused Transformer-XL relative-position self-attention (RelPosMHAXL).
//
// Reference: speechbrain/nnet/attention.py:485-639 (RelPosMHAXL.forward),
// rel_shift :468-483.  For query i, key j (T queries = T keys):
//   score[i,j] = ( (q_i + u)·k_j  +  (q_i + v)·p_{T-1-i+j} ) / sqrt(d_model)
//   masked (key padding) -> -inf, softmax over j, out_i = Σ_j P[i,j] v_j
// where p = linear_pos(RelPosEncXL) and rel_shift is applied in closed form
// (out[i,j] = bd[i, T-1-i+j]) — the (B,H,T,2T-1) bd tensor the reference
// materialises (145 MB at B=32, T=376) never exists here.
//
// One workgroup = (batch b, head h, BQ=32 query rows); 4 waves.
//  phase 1: per 64-key chunk, MFMA tiles of (q+u)Kᵀ straight into an fp32
//           LDS score block S[32][T], and of G = (q+v) P_bandᵀ for the
//           KC+BQ-1 positional rows the chunk needs; S += G[ii][jj+BQ-1-ii].
//  phase 2: exact (two-pass) softmax per row in fp32 from LDS; optional fp32
//           probability output (the reference's returned attention map).
//  phase 3: O = P·V on MFMA with V staged transposed per chunk.
// bf16 inputs use v_mfma_f32_16x16x32_bf16, fp32 inputs exact f32 MFMA
// (see mfma.h); softmax and accumulation are fp32 in both.
#include "mfma.h"

using namespace sbk;

namespace {

constexpr int BQ = 32;
constexpr int KC = 64;

template <typename T, int DHP>
struct AttnLds {
  static constexpr int PAD = MT<T>::PAD;
  static constexpr int QR = DHP + PAD;      // row stride of Qu/Qv/Kc/Pc (elements)
  static constexpr int GR = KC + BQ + 4;    // fp32 G row stride
  static constexpr int VR = KC + PAD;       // Vt row stride
  static size_t bytes(int Tp) {
    const size_t q = (size_t)2 * BQ * QR * sizeof(T);
    const size_t s = (size_t)BQ * (Tp + 4) * 4;
    const size_t p1 = (size_t)KC * QR * sizeof(T) + (size_t)(KC + BQ) * QR * sizeof(T) + (size_t)BQ * GR * 4;
    const size_t p3 = (size_t)BQ * (Tp + PAD) * sizeof(T) + (size_t)DHP * VR * sizeof(T);
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    return al(q) + al(s) + al(p1 > p3 ? p1 : p3);
  }
};

template <typename T, int DHP>
__global__ void __launch_bounds__(256) relpos_attn_kernel(const T* __restrict__ qkv, const T* __restrict__ pk,
                                                          const float* __restrict__ pbu, const float* __restrict__ pbv,
                                                          const uint8_t* __restrict__ kpm, int B, int Tn, int H,
                                                          int dh, float scale, T* __restrict__ out,
                                                          float* __restrict__ probs) {
  using Tr = MT<T>;
  using L = AttnLds<T, DHP>;
  constexpr int QR = L::QR, GR = L::GR, VR = L::VR, PAD = L::PAD;
  const int Tp = (Tn + KC - 1) / KC * KC;
  const int SR = Tp + 4;
  const int PR = Tp + PAD;
  const int d_model = H * dh;
  const int qrow3 = 3 * d_model;  // qkv row length

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  T* Qu = reinterpret_cast<T*>(smem);
  T* Qv = Qu + BQ * QR;
  float* S = reinterpret_cast<float*>(smem + al((size_t)2 * BQ * QR * sizeof(T)));
  unsigned char* r1 = reinterpret_cast<unsigned char*>(S) + al((size_t)BQ * SR * 4);
  T* Kc = reinterpret_cast<T*>(r1);
  T* Pc = Kc + KC * QR;
  float* G = reinterpret_cast<float*>(r1 + (size_t)KC * QR * sizeof(T) + (size_t)(KC + BQ) * QR * sizeof(T));
  T* Pb = reinterpret_cast<T*>(r1);
  T* Vt = Pb + BQ * PR;

  const int nqt = (Tn + BQ - 1) / BQ;
  const int qt = blockIdx.x % nqt;
  const int bh = blockIdx.x / nqt;
  const int h = bh % H, b = bh / H;
  const int i0 = qt * BQ;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  const T* qkv_b = qkv + (long long)b * Tn * qrow3 + h * 3 * dh;

  // ---- Q + u, Q + v into LDS (zero padded rows/dims) ----
  for (int e = tid; e < BQ * DHP; e += 256) {
    const int ii = e / DHP, d = e - ii * DHP;
    const int i = i0 + ii;
    float q = 0.f, u = 0.f, v = 0.f;
    if (i < Tn && d < dh) {
      q = Tr::to_f32(qkv_b[(long long)i * qrow3 + d]);
      u = pbu[h * dh + d];
      v = pbv[h * dh + d];
    }
    Qu[ii * QR + d] = Tr::from_f32(i < Tn && d < dh ? q + u : 0.f);
    Qv[ii * QR + d] = Tr::from_f32(i < Tn && d < dh ? q + v : 0.f);
  }

  // ---- phase 1: scores ----
  const int ntiles_s = (BQ / 16) * (KC / 16);            // 8
  const int ntiles_g = (BQ / 16) * ((KC + BQ) / 16);     // 12
  for (int j0 = 0; j0 < Tp; j0 += KC) {
    __syncthreads();  // previous chunk's readers of Kc/Pc/G are done (and Q staged)
    for (int e = tid; e < KC * DHP; e += 256) {
      const int jj = e / DHP, d = e - jj * DHP;
      const int j = j0 + jj;
      Kc[jj * QR + d] = (j < Tn && d < dh) ? qkv_b[(long long)j * qrow3 + dh + d] : Tr::from_f32(0.f);
    }
    const int rbase = Tn - BQ - i0 + j0;
    for (int e = tid; e < (KC + BQ) * DHP; e += 256) {
      const int rr = e / DHP, d = e - rr * DHP;
      const int r = rbase + rr;
      Pc[rr * QR + d] = (rr < KC + BQ - 1 && r >= 0 && r <= 2 * Tn - 2 && d < dh)
                            ? pk[(long long)r * d_model + h * dh + d]
                            : Tr::from_f32(0.f);
    }
    __syncthreads();
    for (int t = wid; t < ntiles_s + ntiles_g; t += 4) {
      const bool isg = t >= ntiles_s;
      const int tt = isg ? t - ntiles_s : t;
      const int ncol = isg ? (KC + BQ) / 16 : KC / 16;
      const int tm = tt / ncol, tn = tt - tm * ncol;
      const T* a = (isg ? Qv : Qu) + (tm * 16 + fr) * QR + fk;
      const T* bm = (isg ? Pc : Kc) + (tn * 16 + fr) * QR + fk;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < DHP / 32; ++ks) Tr::mma(acc, Tr::load(a + ks * 32), Tr::load(bm + ks * 32));
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ii = tm * 16 + 4 * (lane >> 4) + r;
        const int jj = tn * 16 + fr;
        if (isg)
          G[ii * GR + jj] = acc[r];
        else
          S[ii * SR + j0 + jj] = acc[r];
      }
    }
    __syncthreads();
    for (int e = tid; e < BQ * KC; e += 256) {
      const int ii = e / KC, jj = e - ii * KC;
      const int j = j0 + jj;
      float s = (S[ii * SR + j] + G[ii * GR + jj + BQ - 1 - ii]) * scale;
      if (j >= Tn || (kpm && kpm[(long long)b * Tn + j])) s = -INFINITY;
      S[ii * SR + j] = s;
    }
  }
  __syncthreads();

  // ---- phase 2: softmax rows (wave per row) ----
  for (int ii = wid; ii < BQ; ii += 4) {
    const int i = i0 + ii;
    float* srow = S + ii * SR;
    float m = -INFINITY;
    for (int j = lane; j < Tn; j += 64) m = fmaxf(m, srow[j]);
    m = wave_max(m);
    float sum = 0.f;
    for (int j = lane; j < Tn; j += 64) {
      const float e = expf(srow[j] - m);
      srow[j] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    const float inv = 1.0f / sum;
    float* prow = (probs && i < Tn) ? probs + (((long long)b * H + h) * Tn + i) * Tn : nullptr;
    for (int j = lane; j < Tp; j += 64) {
      float p = 0.f;
      if (j < Tn && i < Tn) {
        p = srow[j] * inv;
        if (prow) prow[j] = p;
      }
      Pb[ii * PR + j] = Tr::from_f32(p);
    }
  }

  // ---- phase 3: O = P V ----
  constexpr int NT3 = (BQ / 16) * (DHP / 16) / 4;  // output tiles per wave
  f32x4 acc[NT3];
#pragma unroll
  for (int q = 0; q < NT3; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < Tp; j0 += KC) {
    __syncthreads();  // Pb complete / previous Vt consumers done
    for (int e = tid; e < KC * DHP; e += 256) {
      const int jj = e / DHP, d = e - jj * DHP;
      const int j = j0 + jj;
      Vt[d * VR + jj] = (j < Tn && d < dh) ? qkv_b[(long long)j * qrow3 + 2 * dh + d] : Tr::from_f32(0.f);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NT3; ++q) {
      const int t = wid + 4 * q;
      const int tm = t / (DHP / 16), tn = t - tm * (DHP / 16);
      const T* a = Pb + (tm * 16 + fr) * PR + j0 + fk;
      const T* bm = Vt + (tn * 16 + fr) * VR + fk;
#pragma unroll
      for (int ks = 0; ks < KC / 32; ++ks) Tr::mma(acc[q], Tr::load(a + ks * 32), Tr::load(bm + ks * 32));
    }
  }
#pragma unroll
  for (int q = 0; q < NT3; ++q) {
    const int t = wid + 4 * q;
    const int tm = t / (DHP / 16), tn = t - tm * (DHP / 16);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + tm * 16 + 4 * (lane >> 4) + r;
      const int d = tn * 16 + fr;
      if (i < Tn && d < dh) out[((long long)b * Tn + i) * d_model + h * dh + d] = Tr::from_f32(acc[q][r]);
    }
  }
}

template <typename T, int DHP>
int launch(const void* qkv, const void* pk, const float* pbu, const float* pbv, const uint8_t* kpm, int B, int Tn,
           int H, int dh, float scale, void* out, float* probs, hipStream_t s) {
  const int Tp = (Tn + KC - 1) / KC * KC;
  const size_t lds = AttnLds<T, DHP>::bytes(Tp);
  if (lds > 160 * 1024) return SBK_ERR_ARG;
  const int grid = B * H * ((Tn + BQ - 1) / BQ);
  hipLaunchKernelGGL((relpos_attn_kernel<T, DHP>), dim3(grid), dim3(256), lds, s, reinterpret_cast<const T*>(qkv),
                     reinterpret_cast<const T*>(pk), pbu, pbv, kpm, B, Tn, H, dh, scale, reinterpret_cast<T*>(out),
                     probs);
  SBK_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// qkv: (B, T, 3*d) head-interleaved in_proj output [h][q|k|v][dh];
// pk: (2T-1, d) linear_pos output; pbu/pbv: (H*dh) fp32; kpm: (B, T) uint8 or null;
// out: (B, T, d); probs: (B, H, T, T) fp32 or null.
SBK_API int sbk_relpos_attention(int dtype_bf16, const void* qkv, const void* pk, const float* pbu, const float* pbv,
                                 const uint8_t* kpm, int B, int Tn, int H, int dh, float scale, void* out, float* probs,
                                 void* stream) {
  if (B <= 0 || Tn <= 0 || H <= 0 || dh <= 0 || dh > 128) return SBK_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (dtype_bf16)
    return dh <= 64 ? launch<bf16_t, 64>(qkv, pk, pbu, pbv, kpm, B, Tn, H, dh, scale, out, probs, s)
                    : launch<bf16_t, 128>(qkv, pk, pbu, pbv, kpm, B, Tn, H, dh, scale, out, probs, s);
  return dh <= 64 ? launch<float, 64>(qkv, pk, pbu, pbv, kpm, B, Tn, H, dh, scale, out, probs, s)
                  : launch<float, 128>(qkv, pk, pbu, pbv, kpm, B, Tn, H, dh, scale, out, probs, s);
}

SBK_API long long sbk_relpos_attention_lds(int dtype_bf16, int Tn, int dh) {
  const int Tp = (Tn + KC - 1) / KC * KC;
  if (dtype_bf16) return dh <= 64 ? (long long)AttnLds<bf16_t, 64>::bytes(Tp) : (long long)AttnLds<bf16_t, 128>::bytes(Tp);
  return dh <= 64 ? (long long)AttnLds<float, 64>::bytes(Tp) : (long long)AttnLds<float, 128>::bytes(Tp);
}
