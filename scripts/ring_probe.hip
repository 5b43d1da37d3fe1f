// Weight-ring depth probe for the layer chain: the chain streams
// 32-KB weight tiles through a 2-slot LDS ring, one tile in flight behind the
// one being multiplied.  Does a deeper ring at the same LDS (4 x 16 KB, three
// tiles in flight) or more LDS (3 x 32 KB) raise the per-CU L2 -> LDS rate?
// Same harness as scripts/fill_probe.hip: one 8-wave workgroup per CU, 256
// workgroups, each streaming the same 2.36-MB image by LDS-DMA (wave-private
// 1-KB pieces), reading its share back with ds_read_b128 and issuing MFMAs in
// proportion to the bytes (12 per 32 KB, the chain's per-step count).
// Build: hipcc --offload-arch=gfx950 -O3 -o ring_probe scripts/ring_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short bf16_t;

constexpr int NT = 512;
constexpr size_t IMG_BYTES = 72 * 32768;  // 2.36 MB: 72 x 32 KB = 144 x 16 KB

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}
__device__ __forceinline__ f32x4 lds_f4(const void* p) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// XR: extra ds_read_b128 per wave and 32-KB step from a shared 6-KB region
// (the chain's phase-2 A fragments: every wave reads the same hidden chunk):
// XR > 0 after the weight reads' wait (a second LDS round trip), XR < 0
// issued with the weight reads under one wait, as the chain's step does
template <int TKB, int NB, int NMFMA, int XR = 0>
__global__ void __launch_bounds__(NT) ring_kernel(const bf16_t* __restrict__ img, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int TB = TKB * 1024, WB = TB / 8, PPT = WB / 1024;  // tile, wave share, 1-KB pieces per wave
  constexpr int TILES = (int)(IMG_BYTES / TB);
  static_assert(TILES % NB == 0 && PPT >= 1 && PPT <= 4, "shape");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const char* base = reinterpret_cast<const char*>(img) + w * WB + lane * 16;
  auto issue = [&](int t) __attribute__((always_inline)) {
    const auto gs = (const __attribute__((address_space(1))) void*)(base + (size_t)t * TB);
    const auto ls = (__attribute__((address_space(3))) void*)(smem + (t % NB) * TB + w * WB);
    __builtin_amdgcn_global_load_lds(gs, ls, 16, 0, 0);
    if constexpr (PPT >= 2) __builtin_amdgcn_global_load_lds(gs, ls, 16, 1024, 0);
    if constexpr (PPT >= 3) __builtin_amdgcn_global_load_lds(gs, ls, 16, 2048, 0);
    if constexpr (PPT >= 4) __builtin_amdgcn_global_load_lds(gs, ls, 16, 3072, 0);
  };
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  f32x4 macc[4] = {};
#pragma unroll
  for (int s = 0; s < NB - 1; ++s) issue(s);
  for (int t = 0; t < TILES; ++t) {
    if (t + NB - 1 < TILES) {
      issue(t + NB - 1);
      vm_wait<(NB - 1) * PPT>();  // tile t landed; the next NB - 1 tiles stay in flight
    } else {
      vm_wait<0>();
    }
    const unsigned char* slot = smem + (t % NB) * TB + w * WB + lane * 16;
    f32x4 r[4];
#pragma unroll
    for (int i = 0; i < PPT; ++i) r[i] = lds_f4(slot + i * 1024);
    // XR2: the extra reads issued with the weight reads, one wait for all
    constexpr int XR2 = XR < 0 ? -XR : 0;
    f32x4 h2[XR2 > 0 ? XR2 : 1];
    if constexpr (XR2 > 0) {
      const unsigned char* hs = smem + NB * TB + (lane & 15) * 16 + (w & 1) * 256;
#pragma unroll
      for (int i = 0; i < XR2; ++i) h2[i] = lds_f4(hs + i * 1024);
    }
    if constexpr (PPT == 4)
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3])::"memory");
    else if constexpr (PPT == 2)
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1])::"memory");
    else
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0])::"memory");
#pragma unroll
    for (int i = 0; i < PPT; ++i) acc += r[i];
    if constexpr (XR2 > 0) {  // landed with the weight reads (the wait above is lgkmcnt(0))
#pragma unroll
      for (int i = 0; i < XR2; ++i) {
        asm volatile("" : "+v"(h2[i]));
        acc += h2[i];
      }
    }
    if constexpr (XR > 0) {  // the shared region sits past the ring (NB * TB <= 96 KB - 6 KB)
      const unsigned char* hs = smem + NB * TB + (lane & 15) * 16 + (w & 1) * 256;
      f32x4 h[XR];
#pragma unroll
      for (int i = 0; i < XR; ++i) h[i] = lds_f4(hs + i * 1024);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < XR; ++i) {
        asm volatile("" : "+v"(h[i]));
        acc += h[i];
      }
    }
    const bf16x8 fa = *reinterpret_cast<bf16x8*>(&r[0]);
    const bf16x8 fb = *reinterpret_cast<bf16x8*>(&r[PPT - 1]);
#pragma unroll
    for (int m = 0; m < NMFMA * PPT / 4; ++m)
      macc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, macc[m & 3], 0, 0, 0);
  }
  const f32x4 s = acc + macc[0] + macc[1] + macc[2] + macc[3];
  out[blockIdx.x * NT + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

template <int TKB, int NB, int NMFMA, int XR = 0>
static void run(const bf16_t* img, float* out, int grid, int reps) {
  auto k = ring_kernel<TKB, NB, NMFMA, XR>;
  const size_t lds = 96 * 1024;  // >= every ring here; > 80 KB: one workgroup per CU
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
  (void)hipEventElapsedTime(&ms, e0, e1);
  if (hipGetLastError() != hipSuccess) {
    printf("launch failed\n");
    exit(1);
  }
  std::vector<float> h((size_t)grid * NT);
  (void)hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost);
  double cs = 0.0;
  for (float v : h) cs += v;
  const double us = ms * 1e3 / reps;
  printf("tile %2d KB x %d slots (%d in flight, %3d KB ring), %2d MFMA + %d extra b128 reads per 32 KB: %7.2f us, "
         "%6.1f GB/s per CU, %5.1f B/clk at 2.4 GHz, checksum %.6e\n",
         TKB, NB, NB - 1, TKB * NB, NMFMA, XR, us, IMG_BYTES / us * 1e-3, IMG_BYTES / (us * 2400.0), cs);
}

int main() {
  const size_t n = IMG_BYTES / 2;
  std::vector<bf16_t> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (bf16_t)(0x3c00 + (i * 2654435761u >> 20) % 256);
  bf16_t* img;
  float* out;
  const int grid = 256;
  (void)hipMalloc(&img, IMG_BYTES);
  (void)hipMalloc(&out, (size_t)grid * NT * 4);
  (void)hipMemcpy(img, h.data(), IMG_BYTES, hipMemcpyHostToDevice);
  if (getenv("RING_PROBE_XR")) {  // the chain's phase-2 LDS reads beside the stream
    for (int rep = 0; rep < 2; ++rep) {
      run<32, 2, 12, 0>(img, out, grid, 50);
      run<32, 2, 12, 6>(img, out, grid, 50);
      run<32, 2, 12, -6>(img, out, grid, 50);
      run<32, 2, 12, -12>(img, out, grid, 50);
    }
    (void)hipFree(img);
    (void)hipFree(out);
    return 0;
  }
  for (int rep = 0; rep < 2; ++rep) {
    run<32, 2, 0>(img, out, grid, 50);
    run<32, 3, 0>(img, out, grid, 50);
    run<16, 2, 0>(img, out, grid, 50);
    run<16, 3, 0>(img, out, grid, 50);
    run<16, 4, 0>(img, out, grid, 50);
    run<32, 2, 12>(img, out, grid, 50);
    run<32, 3, 12>(img, out, grid, 50);
    run<16, 4, 12>(img, out, grid, 50);
    run<32, 2, 24>(img, out, grid, 50);
    run<32, 3, 24>(img, out, grid, 50);
    run<16, 4, 24>(img, out, grid, 50);
  }
  (void)hipFree(img);
  (void)hipFree(out);
  return 0;
}
