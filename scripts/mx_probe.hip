// Probe of the v_mfma_scale_f32_32x32x64_f8f6f4 operand layout (test tool):
// random small-integer e4m3 A (32x64), B (64x32); lane/byte packing under
// several hypotheses; the one whose MFMA result equals the CPU product wins.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k(const unsigned char* a, const unsigned char* b, int sa, int sb, float* d) {
  int l = threadIdx.x;
  i32x8 av, bv;
  const int* ap = (const int*)(a + l * 32);
  const int* bp = (const int*)(b + l * 32);
  for (int i = 0; i < 8; ++i) { av[i] = ap[i]; bv[i] = bp[i]; }
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 0, 0, 0, sa, 0, sb);
  for (int r = 0; r < 16; ++r) d[l * 16 + r] = acc[r];
}

static unsigned char enc(int v) {  // small integer -> e4m3 (exact for |v| <= 8)
  if (v == 0) return 0;
  unsigned s = v < 0 ? 0x80 : 0; int a = abs(v);
  int e = 0; while ((1 << (e + 1)) <= a) ++e;
  int m = (int)((a / (float)(1 << e) - 1.f) * 8.f + 0.5f);
  return (unsigned char)(s | ((e + 7) << 3) | m);
}

int main() {
  int A[32][64], B[64][32];
  srand(1);
  for (int i = 0; i < 32; ++i) for (int k = 0; k < 64; ++k) A[i][k] = rand() % 9 - 4;
  for (int k = 0; k < 64; ++k) for (int j = 0; j < 32; ++j) B[k][j] = rand() % 9 - 4;
  float ref[32][32];
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) { float s = 0; for (int k = 0; k < 64; ++k) s += A[i][k] * B[k][j]; ref[i][j] = s; }
  unsigned char *da, *db; float* dd;
  hipMalloc(&da, 2048); hipMalloc(&db, 2048); hipMalloc(&dd, 4096);
  unsigned char ha[2048], hb[2048]; float hd[1024];
  const char* names[] = {"k=32h+j", "k=16(j/8)+8h+j%8", "k=8(j/4)... h*4", "k=2j+h"};
  for (int hyp = 0; hyp < 4; ++hyp) {
    for (int l = 0; l < 64; ++l) for (int j = 0; j < 32; ++j) {
      int r = l & 31, h = l >> 5, kk;
      if (hyp == 0) kk = 32 * h + j;
      else if (hyp == 1) kk = 16 * (j / 8) + 8 * h + (j % 8);
      else if (hyp == 2) kk = 8 * (j / 4) + 4 * h + (j % 4);
      else kk = 2 * j + h;
      ha[l * 32 + j] = enc(A[r][kk]);
      hb[l * 32 + j] = enc(B[kk][r]);
    }
    hipMemcpy(da, ha, 2048, hipMemcpyHostToDevice); hipMemcpy(db, hb, 2048, hipMemcpyHostToDevice);
    for (int sc = 0; sc < 2; ++sc) {
      int sa = sc ? 128 : 127, sb = 127;
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, sa, sb, dd);
      hipMemcpy(hd, dd, 4096, hipMemcpyDeviceToHost);
      int bad = 0; double ratio = 0;
      for (int l = 0; l < 64; ++l) for (int rg = 0; rg < 16; ++rg) {
        int row = (rg & 3) + 8 * (rg >> 2) + 4 * (l >> 5), col = l & 31;
        float want = ref[row][col] * (sc ? 2.f : 1.f);
        if (fabsf(hd[l * 16 + rg] - want) > 1e-3f) ++bad;
      }
      printf("hyp %d (%s) scale_a=%d: mismatches %d / 1024\n", hyp, names[hyp], sa, bad);
    }
  }
  // scale operand 0 (unscaled select) check
  return 0;
}
