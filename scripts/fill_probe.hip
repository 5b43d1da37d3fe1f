// Weight-stream fill-rate probe for the layer chain (VERDICT r5
// item 3): does feeding half of each 32-KB weight tile through VGPR loads +
// ds_write_b128, beside LDS-DMA for the other half, raise the per-CU
// L2 -> LDS rate above the all-LDS-DMA stream the chain uses?
//
// One 8-wave workgroup per CU (LDS request forces one per CU), 256
// workgroups, every workgroup streams the same 2.4-MB image (76 tiles of
// 256 rows x 64 k bf16 = 32 KB, L2-resident like the chain's weights) through
// a 2-slot ring: tile t+1 is issued, tile t waited for (counted vmcnt), its
// wave-private 4 KB read back by ds_read_b128 and, optionally, MFMAs issued
// per step to stand in for the chain's 12 per wave.
//   mode 0: 4 LDS-DMA pieces (1 KB per wave each) per wave and tile (the chain)
//   mode 1: 2 LDS-DMA pieces + 2 global_load_dwordx4 -> ds_write_b128
//   mode 2: 4 global_load_dwordx4 -> ds_write_b128
// Build: hipcc --offload-arch=gfx950 -O3 -o fill_probe scripts/fill_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned short bf16_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int NT = 512, TILES = 76, TILE_EL = 256 * 64, WAVE_EL = TILE_EL / 8;

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}
__device__ __forceinline__ f32x4 gld4(const bf16_t* p) {
  f32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void lds_st4(void* p, f32x4 v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ f32x4 lds_f4(const void* p) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}

template <int MODE, int NMFMA>
__global__ void __launch_bounds__(NT) fill_kernel(const bf16_t* __restrict__ img, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int NDMA = MODE == 0 ? 4 : MODE == 1 ? 2 : 0;
  constexpr int NV = 4 - NDMA;
  // VGPR-staged pieces of the two tiles in flight; slots are compile-time
  // (a run-time slot index made the compiler copy the asm load destinations
  // while the loads were in flight: the first version faulted)
  f32x4 st0[4], st1[4];
  auto issue = [&](int t, f32x4(&stage)[4]) __attribute__((always_inline)) {
    const bf16_t* src = img + (size_t)t * TILE_EL + w * WAVE_EL + lane * 8;
    bf16_t* dst = ring + (t & 1) * TILE_EL + w * WAVE_EL;
    const auto ls = (__attribute__((address_space(3))) void*)dst;
    const auto gs = (const __attribute__((address_space(1))) void*)src;
    if constexpr (NDMA >= 1) __builtin_amdgcn_global_load_lds(gs, ls, 16, 0, 0);
    if constexpr (NDMA >= 2) __builtin_amdgcn_global_load_lds(gs, ls, 16, 1024, 0);
    if constexpr (NDMA >= 3) __builtin_amdgcn_global_load_lds(gs, ls, 16, 2048, 0);
    if constexpr (NDMA >= 4) __builtin_amdgcn_global_load_lds(gs, ls, 16, 3072, 0);
#pragma unroll
    for (int i = 0; i < NV; ++i) stage[i] = gld4(src + (NDMA + i) * 512);
  };
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  f32x4 macc[4] = {};
  auto step = [&](int t, f32x4(&cur)[4], f32x4(&nxt)[4]) __attribute__((always_inline)) {
    if (t + 1 < TILES) {
      issue(t + 1, nxt);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile t landed; tile t+1's 4 ops in flight
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bf16_t* slot = ring + (t & 1) * TILE_EL + w * WAVE_EL;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      asm volatile("" : "+v"(cur[i]));
      lds_st4(slot + (NDMA + i) * 512 + lane * 8, cur[i]);
    }
    f32x4 r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = lds_f4(slot + i * 512 + lane * 8);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3])::"memory");
#pragma unroll
    for (int i = 0; i < 4; ++i) acc += r[i];
    const bf16x8 fa = *reinterpret_cast<bf16x8*>(&r[0]);
    const bf16x8 fb = *reinterpret_cast<bf16x8*>(&r[1]);
#pragma unroll
    for (int m = 0; m < NMFMA; ++m) macc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, macc[m & 3], 0, 0, 0);
  };
  issue(0, st0);
  for (int t = 0; t < TILES; t += 2) {
    step(t, st0, st1);
    step(t + 1, st1, st0);
  }
  const f32x4 s = acc + macc[0] + macc[1] + macc[2] + macc[3];
  out[blockIdx.x * NT + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

template <int MODE, int NMFMA>
static void run(const bf16_t* img, float* out, int grid, size_t lds, int reps) {
  auto k = fill_kernel<MODE, NMFMA>;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, dim3(grid), dim3(NT), lds, 0, img, out);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(NT), lds, 0, img, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / reps;
  if (hipGetLastError() != hipSuccess) {
    printf("launch failed\n");
    exit(1);
  }
  std::vector<float> h((size_t)grid * NT);
  hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost);
  double cs = 0.0;
  for (float v : h) cs += v;
  const double bytes_cu = (double)TILES * TILE_EL * 2;
  printf("mode %d (%d LDS-DMA + %d VGPR pieces per wave-tile), %2d MFMA/step: %7.2f us per launch, "
         "%6.1f GB/s per CU, %5.1f B/clk at 2.4 GHz, %.2f TB/s chip (L2->LDS), checksum %.6e\n",
         MODE, MODE == 0 ? 4 : MODE == 1 ? 2 : 0, MODE == 0 ? 0 : MODE == 1 ? 2 : 4, NMFMA, us,
         bytes_cu / us * 1e-3, bytes_cu / (us * 2400.0), bytes_cu * grid / us * 1e-6, cs);
}

int main() {
  const size_t n = (size_t)TILES * TILE_EL;
  std::vector<bf16_t> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (bf16_t)(0x3c00 + (i * 2654435761u >> 20) % 256);
  bf16_t* img;
  float* out;
  const int grid = 256;
  hipMalloc(&img, n * 2);
  hipMalloc(&out, (size_t)grid * NT * 4);
  hipMemcpy(img, h.data(), n * 2, hipMemcpyHostToDevice);
  const size_t lds = 96 * 1024;  // > 80 KB: one workgroup per CU
  for (int rep = 0; rep < 2; ++rep) {
    run<0, 0>(img, out, grid, lds, 50);
    run<1, 0>(img, out, grid, lds, 50);
    run<2, 0>(img, out, grid, lds, 50);
    run<0, 12>(img, out, grid, lds, 50);
    run<1, 12>(img, out, grid, lds, 50);
    run<2, 12>(img, out, grid, lds, 50);
  }
  hipFree(img);
  hipFree(out);
  return 0;
}
