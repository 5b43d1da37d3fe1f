// For each operand byte (lane half h, byte j) of row 0: which lane's A scale
// multiplies it?  A row 0 = 1.0 at (h, j) only, B = 1.0; all A scales 127
// except lane `hot` (128); D[0][0] is 2 when lane `hot`'s scale applies,
// 1 when another lane's does, 0 when the byte is not in row 0 (test tool).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void k(int hh, int jj, int hot, float* d) {
  int l = threadIdx.x, h = l >> 5, r = l & 31;
  i32x8 av, bv;
  for (int i = 0; i < 8; ++i) {
    unsigned v = 0;
    for (int b = 0; b < 4; ++b) if (r == 0 && h == hh && 4 * i + b == jj) v |= 0x38u << (8 * b);
    av[i] = (int)v;
    bv[i] = 0x38383838;
  }
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = d[64 + l * 16 + r];  // zeros from memory: keeps C/D off the A/B registers
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 0, 0, 0, l == hot ? 128 : 127, 0, 127);
  if (l == 0) d[0] = acc[0];
}
int main() {
  float* dd; float v;
  (void)hipMalloc(&dd, 8192);
  (void)hipMemset(dd, 0, 8192);
  for (int h = 0; h < 2; ++h) {
    printf("h=%d:", h);
    for (int j = 0; j < 32; ++j) {
      int found = -1; float base = -1;
      for (int hot = 0; hot < 64; ++hot) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, h, j, hot, dd);
        hipError_t e1 = hipGetLastError(), e2 = hipDeviceSynchronize();
        if (e1 != hipSuccess || e2 != hipSuccess) { printf("launch error %s %s\n", hipGetErrorString(e1), hipGetErrorString(e2)); return 1; }
        (void)hipMemcpy(&v, dd, 4, hipMemcpyDeviceToHost);
        if (v == 2.f) found = hot;
        if (hot == 63) base = v;
      }
      printf(" %d(%g)", found, base);
    }
    printf("\n");
  }
  return 0;
}
