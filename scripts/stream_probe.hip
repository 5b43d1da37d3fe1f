// Microbenchmark (never the product): the per-CU L2 -> LDS weight stream of
// the layer-chain FFN kernel (ffn.hip) in isolation.  One 8-wave workgroup
// per CU streams the same STEPS x (8 x GL KB) weight image (L2 / MALL
// resident, as the layer's weights are) through an NS-slot LDS-DMA ring, the
// way ffn_kernel does: wait for tile s (counted vmcnt), read the wave's own
// fragments (ds_read_b128), issue tile s + NS into the freed slot, MFMAs.
// Variants switch the reads / extra reads (phase-2 hidden operand) / MFMAs
// off and on, and vary the ring depth and tile size, to find what bounds a
// step: the DMA rate per CU, LDS bandwidth, or latency x bytes in flight.
// build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC -o gpurun_probe_stream.so scripts/stream_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

// MODE bits: 1 = fragment reads, 2 = extra hidden-operand reads (6 x b128), 4 = MFMAs.
// LDB = 0: every step's tile is one contiguous 8*GL KB block; LDB > 0: the
// tile is 64 k (128 B) of 8*GL*8 rows of a row-major matrix with LDB-byte rows,
// the chain's weight layout (W1 / Wp rows 512 B, W2 rows 2 KB), with its
// XOR-swizzled 16-B chunk order.
template <int NS, int GL, int MODE, int LDB>
__global__ void __launch_bounds__(512) stream_k(const uint16_t* __restrict__ w, int steps, float* out,
                                                unsigned long long* clk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int TILE = 8 * GL * 1024;  // bytes per step per CU
  unsigned char* ring = smem;
  unsigned char* hs = smem + NS * TILE;  // 6 KB per wave of "hidden" operand
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int fr = lane & 15, g = lane >> 4;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  auto issue = [&](int s, int slot) __attribute__((always_inline)) {
    const unsigned char* src = reinterpret_cast<const unsigned char*>(w) + (long long)(s % steps) * TILE;
    if (LDB) {
      constexpr int CPM = LDB / 128;  // 128-B column blocks (steps) per matrix
      const int sm = s % steps;
      src = reinterpret_cast<const unsigned char*>(w) + (long long)(sm / CPM) * (GL * 64) * LDB + (sm % CPM) * 128;
    }
#pragma unroll
    for (int i = 0; i < GL; ++i) {
      const int piece = wv * GL + i;
      const int row = piece * 8 + (lane >> 3);
      const int off = LDB ? row * LDB + (((lane & 7) ^ ((row >> 1) & 7)) << 4) : piece * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + off),
                                       (__attribute__((address_space(3))) void*)(ring + slot * TILE + piece * 1024), 16,
                                       0, 0);
    }
  };
#pragma unroll
  for (int s = 0; s < NS; ++s) issue(s, s);
  f32x4 acc[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 xa[2][3];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int m = 0; m < 3; ++m)
      for (int j = 0; j < 8; ++j) xa[k][m][j] = (__bf16)(0.001f * (lane + j + k + m));
  for (int s = 0; s < steps; ++s) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL * (NS - 1)) : "memory");
    const int slot = s % NS;
    bf16x8 fw[2][2], fh[2][3];
    if (MODE & 1) {
      // the wave's GL KB: 8*GL rows of 128 B; 16-row fragments, XOR-swizzled chunks
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int row = (wv * GL * 8 + t * 16 + fr) % (GL * 64);
          const uint32_t la = lds_addr(ring + slot * TILE + row * 128 + ((((ks * 4 + g) ^ ((row >> 1) & 7))) << 4));
          asm volatile("ds_read_b128 %0, %1" : "=v"(fw[ks][t]) : "v"(la) : "memory");
        }
    }
    if (MODE & 2) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int m = 0; m < 3; ++m) {
          const uint32_t la = lds_addr(hs + ((m * 16 + fr) * 272 + ((s & 3) * 64) + ks * 32 + 8 * g) * 2);
          asm volatile("ds_read_b128 %0, %1" : "=v"(fh[ks][m]) : "v"(la) : "memory");
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // tie every asm-read fragment to a wait: the compiler takes an asm
    // output as written at the asm statement, so without this it hoists the
    // MFMAs above the wait and reuses registers the reads land in later
    // (the first two probe versions faulted that way)
    if (MODE & 1) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int t = 0; t < 2; ++t) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fw[ks][t]));
    }
    if (MODE & 2) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int m = 0; m < 3; ++m) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fh[ks][m]));
    }
    if (s + NS < steps + NS) issue(s + NS, slot);
    if (MODE & 4) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int m = 0; m < 3; ++m)
            acc[t * 3 + m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                (MODE & 1) ? fw[ks][t] : xa[ks][t], (MODE & 2) ? fh[ks][m] : xa[ks][m], acc[t * 3 + m], 0, 0, 0);
    } else if (MODE & 3) {
      // consume every dword of every fragment: an asm output with dead parts
      // lets the compiler reuse those registers before the read returns
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      unsigned v = 0;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
          if (MODE & 1) {
            const u32x4 q = __builtin_bit_cast(u32x4, fw[ks][t]);
            v ^= q[0] ^ q[1] ^ q[2] ^ q[3];
          }
#pragma unroll
        for (int m = 0; m < 3; ++m)
          if (MODE & 2) {
            const u32x4 q = __builtin_bit_cast(u32x4, fh[ks][m]);
            v ^= q[0] ^ q[1] ^ q[2] ^ q[3];
          }
      }
      acc[0][0] += (float)(v & 1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < 6; ++i) v += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 512 + tid] = v;
  if (tid == 0) {
    clk[blockIdx.x * 2] = t1 - t0;
    clk[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

template <int NS, int GL, int MODE, int LDB>
int launch(const void* w, int steps, float* out, unsigned long long* clk, int grid, void* stream) {
  const int lds = 160 * 1024;  // one workgroup per CU
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&stream_k<NS, GL, MODE, LDB>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
      return 1;
    attr = true;
  }
  hipLaunchKernelGGL((stream_k<NS, GL, MODE, LDB>), dim3(grid), dim3(512), lds, (hipStream_t)stream,
                     reinterpret_cast<const uint16_t*>(w), steps, out, clk);
  return (int)hipGetLastError();
}

#define V(NS, GL, MODE, LDB) \
  if (ns == NS && gl == GL && mode == MODE && ldb == LDB) return launch<NS, GL, MODE, LDB>(w, steps, out, clk, grid, stream);

extern "C" __attribute__((visibility("default"))) int stream_probe(int ns, int gl, int mode, int ldb, const void* w, int steps,
                                                                    float* out, unsigned long long* clk, int grid,
                                                                    void* stream) {
#define MODES(NS, GL) V(NS, GL, 0, 0) V(NS, GL, 1, 0) V(NS, GL, 3, 0) V(NS, GL, 5, 0) V(NS, GL, 7, 0)
  MODES(2, 4)
  MODES(4, 4)
  MODES(2, 8)
  V(2, 4, 0, 512) V(2, 4, 7, 512) V(2, 4, 0, 2048) V(2, 4, 7, 2048)
  V(4, 4, 0, 512) V(4, 4, 7, 512) V(4, 4, 0, 2048) V(4, 4, 7, 2048)
  return 2;
}
