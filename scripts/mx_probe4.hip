// v_mfma_scale_f32_32x32x64_f8f6f4 with per-lane E8M0 scales (test tool):
// random small-integer A (32x64) / B (64x32), packed under packing P, scales
// per lane; count mismatches against the CPU product under scale rules
//   R0: element (r, k) uses the scale of the lane that holds it
//   R1: element (r, k) uses the scale of lane r + 32 * (k / 32)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void k(const unsigned char* a, const unsigned char* b, const int* sa, const int* sb, float* d) {
  int l = threadIdx.x;
  i32x8 av, bv;
  const int* ap = (const int*)(a + l * 32);
  const int* bp = (const int*)(b + l * 32);
  for (int i = 0; i < 8; ++i) { av[i] = ap[i]; bv[i] = bp[i]; }
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 0, 0, 0, sa[l], 0, sb[l]);
  for (int r = 0; r < 16; ++r) d[l * 16 + r] = acc[r];
}
static unsigned char enc(int v) {
  if (v == 0) return 0;
  unsigned s = v < 0 ? 0x80 : 0; int a = abs(v);
  int e = 0; while ((1 << (e + 1)) <= a) ++e;
  int m = (int)((a / (float)(1 << e) - 1.f) * 8.f + 0.5f);
  return (unsigned char)(s | ((e + 7) << 3) | m);
}
static int kmap(int P, int h, int j) {
  if (P == 0) return 32 * h + j;
  if (P == 1) return 16 * (j / 8) + 8 * h + (j % 8);
  if (P == 2) return 8 * (j / 4) + 4 * h + (j % 4);
  return 2 * j + h;
}
int main() {
  int A[32][64], B[64][32];
  srand(7);
  for (int i = 0; i < 32; ++i) for (int q = 0; q < 64; ++q) A[i][q] = rand() % 9 - 4;
  for (int q = 0; q < 64; ++q) for (int j = 0; j < 32; ++j) B[q][j] = rand() % 9 - 4;
  int hsa[64], hsb[64];
  for (int l = 0; l < 64; ++l) { hsa[l] = 124 + (l * 7) % 7; hsb[l] = 124 + (l * 5 + 3) % 6; }
  unsigned char *da, *db; int *dsa, *dsb; float* dd;
  (void)hipMalloc(&da, 2048); (void)hipMalloc(&db, 2048); (void)hipMalloc(&dsa, 256); (void)hipMalloc(&dsb, 256);
  (void)hipMalloc(&dd, 4096);
  (void)hipMemcpy(dsa, hsa, 256, hipMemcpyHostToDevice); (void)hipMemcpy(dsb, hsb, 256, hipMemcpyHostToDevice);
  unsigned char ha[2048], hb[2048]; float hd[1024];
  for (int P = 0; P < 4; ++P) {
    int lane_of[64];  // k -> lane half holding it (for row r: lane r + 32*h)
    for (int l = 0; l < 64; ++l) for (int j = 0; j < 32; ++j) {
      int r = l & 31, h = l >> 5, q = kmap(P, h, j);
      ha[l * 32 + j] = enc(A[r][q]);
      hb[l * 32 + j] = enc(B[q][r]);
      if (r == 0) lane_of[q] = h;
    }
    (void)hipMemcpy(da, ha, 2048, hipMemcpyHostToDevice); (void)hipMemcpy(db, hb, 2048, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
    (void)hipMemcpy(hd, dd, 4096, hipMemcpyDeviceToHost);
    for (int R = 0; R < 2; ++R) {
      int bad = 0;
      for (int l = 0; l < 64; ++l) for (int rg = 0; rg < 16; ++rg) {
        int row = (rg & 3) + 8 * (rg >> 2) + 4 * (l >> 5), col = l & 31;
        double s = 0;
        for (int q = 0; q < 64; ++q) {
          int la = R == 0 ? row + 32 * lane_of[q] : row + 32 * (q / 32);
          int lb = R == 0 ? col + 32 * lane_of[q] : col + 32 * (q / 32);
          s += A[row][q] * B[q][col] * ldexp(1.0, hsa[la] - 127) * ldexp(1.0, hsb[lb] - 127);
        }
        if (fabs(hd[l * 16 + rg] - s) > 1e-3 * (1 + fabs(s))) ++bad;
      }
      printf("packing %d rule R%d: mismatches %d / 1024\n", P, R, bad);
    }
  }
  return 0;
}
