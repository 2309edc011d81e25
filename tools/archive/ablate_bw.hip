// (Round 3: the ABL bits / -DILQR_* switches this probe uses exist only in the tree
// tools/archive/ablation/restore_tree.sh restores; build it there.)
// Ablation harness for the backward kernel (not part of the product): times
// lq_backward_wave<12,4,ABL> for several ABL bit sets at B=4096, T=100 so the
// share of MFMA / factor+solve / LDS hand-off / stores / gradient can be read off.
#include "../ilqr.jl_amd/csrc/ilqr_lq.hip"
#include <cstdio>
#include <vector>
#include <random>
#include <cmath>
using namespace ilqr;
template <int ABL>
__global__ __launch_bounds__(256, 4) void abl_kernel(LQParams P, int B, int T, const double* x, const double* u,
                                                  double* d, double* K, int* flag) {
  __shared__ __attribute__((aligned(16))) double lds[WAVES_PER_WG * BW_LDS];
  const int w = threadIdx.x >> 6;
  const int b = blockIdx.x * WAVES_PER_WG + w;
  if (b >= B) return;
  // phase-offset experiment (harness only): stagger the 4 waves of a SIMD
  // (WGs sharing a SIMD are ~256 block indices apart: one wave per SIMD per WG)
  const int gen = (blockIdx.x >> 8) & 3;
  if constexpr ((ABL & (1 << 14)) != 0) { for (int i = 0; i < gen; ++i) __builtin_amdgcn_s_sleep(8); }
  bool nan = lq_backward_wave<12, 4, (ABL & ((1 << 14) - 1))>(P, b, T, x, u, d, K, 0.01, lds + w * BW_LDS);
  if (nan && (threadIdx.x & 63) == 0) atomicAdd(flag, 1);
}
#define CK(x) do { hipError_t e=(x); if(e!=hipSuccess){printf("err %s line %d\n",hipGetErrorString(e),__LINE__); return 1;} } while(0)
template <int ABL>
int run(const char* name, LQParams P, int B, int T, double* x, double* u, double* d, double* K, int* flag) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int grid = (B + 3) / 4;
  for (int i = 0; i < 150; ++i) abl_kernel<ABL><<<grid, 256>>>(P, B, T, x, u, d, K, flag);  // clock run-in
  CK(hipDeviceSynchronize());
  const int R = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < R; ++i) abl_kernel<ABL><<<grid, 256>>>(P, B, T, x, u, d, K, flag);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-40s %8.1f us\n", name, 1000.0 * ms / R);
  return 0;
}
int main() {
  const int B = 4096, T = 100, n = 12, m = 4;
  std::mt19937_64 g(1); std::uniform_real_distribution<double> U(-1, 1);
  auto mk = [&](size_t N, double sc, bool eye, int dim) { std::vector<double> v(N); for (auto& e : v) e = sc * U(g);
    if (eye) for (size_t b = 0; b < N / (dim * dim); ++b) for (int i = 0; i < dim; ++i) v[b * dim * dim + i * dim + i] += 1.0; return v; };
  auto A = mk((size_t)B * n * n, 0.02, true, n), Bm = mk((size_t)B * n * m, 0.1, false, 1);
  auto Q = mk((size_t)B * n * n, 0.0, true, n), R = mk((size_t)B * m * m, 0.0, true, m), Qf = Q;
  auto x = mk((size_t)B * (T + 1) * n, 1.0, false, 1), u = mk((size_t)B * T * m, 0.1, false, 1);
  auto up = [&](std::vector<double>& v) { double* p; hipMalloc(&p, v.size() * 8); hipMemcpy(p, v.data(), v.size() * 8, hipMemcpyHostToDevice); return p; };
  LQParams P{up(A), up(Bm), up(Q), up(R), up(Qf)};
  double *xd = up(x), *ud = up(u), *d, *K; int* flag;
  CK(hipMalloc(&d, (size_t)B * T * m * 8)); CK(hipMalloc(&K, (size_t)B * T * m * n * 8)); CK(hipMalloc(&flag, 4));
  std::vector<double> Kref((size_t)B * T * m * n), Kv(Kref.size());
  auto diff = [&](const char* name) {
    CK(hipMemcpy(Kv.data(), K, Kv.size() * 8, hipMemcpyDeviceToHost));
    double mx = 0, ref = 0;
    for (size_t i = 0; i < Kv.size(); ++i) { mx = fmax(mx, fabs(Kv[i] - Kref[i])); ref = fmax(ref, fabs(Kref[i])); }
    printf("%-40s rel diff vs full %.3e\n", name, mx / ref);
    return 0;
  };
  run<0>("product", P, B, T, xd, ud, d, K, flag);
  CK(hipMemcpy(Kref.data(), K, Kref.size() * 8, hipMemcpyDeviceToHost));
  run<4096>("Y on VALU (dpp), Z on MFMA", P, B, T, xd, ud, d, K, flag); diff("Y on VALU, Z on MFMA");
  for (int rep = 0; rep < 2; ++rep) {
    run<0>("product", P, B, T, xd, ud, d, K, flag);
    run<4096>("Y on VALU (dpp), Z on MFMA", P, B, T, xd, ud, d, K, flag);
  }
  run<2048>("cofactor solve + refinement", P, B, T, xd, ud, d, K, flag); diff("cofactor + refinement");
  run<2048 + 8192>("cofactor solve, no refinement", P, B, T, xd, ud, d, K, flag); diff("cofactor, no refinement");
  run<128>("Schur4 solve", P, B, T, xd, ud, d, K, flag); diff("Schur4 solve");
  for (int rep = 0; rep < 2; ++rep) {
    printf("-- cofactor, round %d\n", rep);
    run<0>("product (LDLT solve)", P, B, T, xd, ud, d, K, flag);
    run<2048>("cofactor solve + refinement", P, B, T, xd, ud, d, K, flag);
    run<2048 + 8192>("cofactor solve, no refinement", P, B, T, xd, ud, d, K, flag);
  }
  run<1024>("VALU Y/Z (dpp)", P, B, T, xd, ud, d, K, flag); diff("VALU Y/Z (dpp)");
  for (int rep = 0; rep < 2; ++rep) {
    printf("-- VALU products, round %d\n", rep);
    run<0>("product (MFMA Y/Z)", P, B, T, xd, ud, d, K, flag);
    run<1024>("VALU Y/Z (dpp)", P, B, T, xd, ud, d, K, flag);
    run<1024 + 1>("VALU Y/Z, no factor/solve", P, B, T, xd, ud, d, K, flag);
    run<1024 + 8>("VALU Y/Z, no K/d stores", P, B, T, xd, ud, d, K, flag);
    run<1024 + 31>("VALU Y/Z chain + selects only", P, B, T, xd, ud, d, K, flag);
  }
  for (int rep = 0; rep < 1; ++rep) {
    printf("-- round %d\n", rep);
    run<0>("product", P, B, T, xd, ud, d, K, flag);
    run<256>("round-1 gradient", P, B, T, xd, ud, d, K, flag);
    run<512>("round-1 stores", P, B, T, xd, ud, d, K, flag);
    run<768>("round-1 gradient + stores", P, B, T, xd, ud, d, K, flag);
    run<768 + 96>("round-1 v4 (2 Newton, sym 4)", P, B, T, xd, ud, d, K, flag);
    run<1>("no factor/solve", P, B, T, xd, ud, d, K, flag);
    run<2>("no symmetrisation", P, B, T, xd, ud, d, K, flag);
    run<4>("no LDS hand-off", P, B, T, xd, ud, d, K, flag);
    run<8>("no K/d stores", P, B, T, xd, ud, d, K, flag);
    run<16>("no gradient reduction", P, B, T, xd, ud, d, K, flag);
    run<31>("MFMA chain + selects only", P, B, T, xd, ud, d, K, flag);
  }
  return 0;
}
