// Which lane's E8M0 scale applies to A block (row r, k-block b) of
// v_mfma_scale_f32_32x32x64_f8f6f4 (test tool)?  Packing: lane (r, h) holds
// k = 32h + j.  A row r = 1.0 on block b only, B = 1.0 everywhere, lane l's
// A scale = 120 + (l % 16) (distinct within each half), B scale 127.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void k(int blk, int opsel, float* d) {
  int l = threadIdx.x, h = l >> 5;
  i32x8 av, bv;
  int one = 0x38383838;  // e4m3 1.0 = 0x38
  for (int i = 0; i < 8; ++i) { av[i] = (h == blk) ? one : 0; bv[i] = one; }
  int sa = 100 + l;
  f32x16 acc = {};
  if (opsel == 0)
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 0, 0, 0, sa, 0, 127);
  else
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 0, 0, 0, sa << 8, 0, 127);
  for (int r = 0; r < 16; ++r) d[l * 16 + r] = acc[r];
}
int main() {
  float* dd; float hd[1024];
  (void)hipMalloc(&dd, 4096);
  for (int blk = 0; blk < 2; ++blk) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, blk, 0, dd);
    (void)hipMemcpy(hd, dd, 4096, hipMemcpyDeviceToHost);
    printf("block %d:", blk);
    for (int row = 0; row < 32; ++row) {
      // find value at (row, col 0): lane with col 0 and its register
      int l = (row & 4) ? 32 : 0; int rg = (row & 3) + 4 * (row >> 3);
      float v = hd[l * 16 + rg];
      int e = (int)lrintf(log2f(v / 32.f)) + 127;
      printf(" r%d:s%d", row, e);
    }
    printf("\n");
  }
  return 0;
}
