// Probe (not product): operand/result lane maps of v_mfma_f64_4x4x4f64 (4 blocks) on
// gfx950. For every lane x: d = mfma(e_x, 1) and d = mfma(1, e_x) (one-hot operands),
// and d = mfma(a, b) for one-hot pairs; prints the nonzero output lanes.
// Result (profiles/r01/mfma4_probe.txt), block b = trajectory slot:
//   A[m][k] of block b at lane 16k + 4b + m,  B[k][n] at lane 16k + 4b + n,
//   D[m][n] at lane 16m + 4b + n.
// So D feeds the B operand unchanged and the A operand as its transpose.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double* da, double* db, double* dab) {
  const int l = threadIdx.x;
  for (int x = 0; x < 64; ++x) {
    da[x * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(l == x ? 1.0 : 0.0, 1.0, 0.0, 0, 0, 0);
    db[x * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, l == x ? 1.0 : 0.0, 0.0, 0, 0, 0);
  }
  // A one-hot at lane x, B one-hot at lane y: nonzero output iff the pair meets in some k
  for (int x = 0; x < 16; ++x)
    for (int y = 0; y < 16; ++y)
      dab[(x * 16 + y) * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(l == x ? 1.0 : 0.0, l == y ? 1.0 : 0.0, 0.0, 0, 0, 0);
}
int main() {
  double *da, *db, *dab;
  hipMalloc(&da, 64 * 64 * 8); hipMalloc(&db, 64 * 64 * 8); hipMalloc(&dab, 256 * 64 * 8);
  k<<<1, 64>>>(da, db, dab);
  static double ha[64 * 64], hb[64 * 64], hab[256 * 64];
  hipMemcpy(ha, da, sizeof ha, hipMemcpyDeviceToHost);
  hipMemcpy(hb, db, sizeof hb, hipMemcpyDeviceToHost);
  hipMemcpy(hab, dab, sizeof hab, hipMemcpyDeviceToHost);
  for (int x = 0; x < 64; ++x) {
    printf("A%02d:", x); for (int l = 0; l < 64; ++l) if (ha[x * 64 + l] != 0) printf(" %d", l); printf("\n");
  }
  for (int x = 0; x < 64; ++x) {
    printf("B%02d:", x); for (int l = 0; l < 64; ++l) if (hb[x * 64 + l] != 0) printf(" %d", l); printf("\n");
  }
  for (int x = 0; x < 16; ++x)
    for (int y = 0; y < 16; ++y) {
      int n = 0; for (int l = 0; l < 64; ++l) n += hab[(x * 16 + y) * 64 + l] != 0;
      if (n) { printf("AB %d %d:", x, y); for (int l = 0; l < 64; ++l) if (hab[(x * 16 + y) * 64 + l] != 0) printf(" %d", l); printf("\n"); }
    }
  return 0;
}
