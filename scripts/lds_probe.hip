// LDS bank-conflict model probe for ds_read_b128 on gfx950 (never the
// product).  Does a 16-B LDS read conflict when two lanes of the same
// 8-lane group hit one bank set (the "8 lanes per cycle" model), or
// already when lanes i and i + 8 do (a "16 lanes per cycle" model)?  The
// product kernels' swizzles assume the 8-lane model; this times both shapes.
//   pattern 0: lane i -> 16 i B (contiguous; conflict-free in any model)
//   pattern 1: lane i -> 32 (i % 8) + 512 (i / 8) B (8 lanes cover the 64
//              banks; lanes i and i + 8 share a bank set)
//   pattern 2: lane i -> 16 (i % 16) + 1024 (i / 16) B (16 lanes cover the
//              64 banks; lanes i and i + 16 share a bank set)
//   pattern 3: lane i -> 256 i B (every lane the same bank set: worst case)
// usage: hipcc --offload-arch=gfx950 -O3 -o scripts/lds_probe scripts/lds_probe.hip && scripts/lds_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void __launch_bounds__(512) lds_pat(int pat, int iters, float* out) {
  __shared__ __attribute__((aligned(16))) float lds[16384];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 16384; i += blockDim.x) lds[i] = (float)(i & 255);
  __syncthreads();
  int off;  // floats
  if (pat == 0)
    off = lane * 4;
  else if (pat == 1)
    off = (lane & 7) * 8 + (lane >> 3) * 128;
  else if (pat == 2)
    off = (lane & 15) * 4 + (lane >> 4) * 256;
  else
    off = lane * 64;
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const int wofs = (tid >> 6) * 32;  // waves read different (same-shaped) rows
  for (int it = 0; it < iters; ++it) {
    const f4 v = *reinterpret_cast<const f4*>(lds + ((off + wofs + (it & 7) * 2048) & 16383));
    acc += v;
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == -1.f) out[tid] = acc[0];  // keep the reads
}

int main() {
  float* out;
  hipMalloc(&out, 4096 * sizeof(float));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 4096, waves = 8;
  for (int pat = 0; pat < 4; ++pat) {
    hipLaunchKernelGGL(lds_pat, dim3(256), dim3(64 * waves), 0, 0, pat, iters, out);  // warm
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(lds_pat, dim3(256), dim3(64 * waves), 0, 0, pat, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    const double per = ms / 5 * 1e-3 * 2.1e9 / ((double)iters * waves);  // cycles per wave read per CU (2.1 GHz)
    printf("pattern %d: %.3f ms per launch, ~%.2f cycles per ds_read_b128 per CU\n", pat, ms / 5, per);
  }
  hipFree(out);
  return 0;
}
