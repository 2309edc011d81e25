// (Round 3: the ABL bits / -DILQR_* switches this probe uses exist only in the tree
// tools/archive/ablation/restore_tree.sh restores; build it there.)
// Probe for the four-trajectories-per-wave backward (not part of the product):
// times lq_backward4_kernel against the one-trajectory-per-wave lq_backward_kernel
// at B=4096, T=100 (random stable LQ problems, as tools/archive/ablate_bw.hip) and reports
// the max relative difference of K and d between the two.
#include "../ilqr.jl_amd/csrc/ilqr_lq.hip"
#include "../ilqr.jl_amd/csrc/ilqr_bw4.hip"
#include <cstdio>
#include <vector>
#include <random>
#include <cmath>
#include <string>
using namespace ilqr;
#define CK(x) do { hipError_t e=(x); if(e!=hipSuccess){printf("err %s line %d\n",hipGetErrorString(e),__LINE__); return 1;} } while(0)
int main(int argc, char** argv) {
  // argv[1]: batch size (random stable LQ problems), or "quad": the headline quadrotor
  // batch of tools/quad256.bin (tools/dump_quad.py) against the symmetrised C oracle
  const bool quad = argc > 1 && std::string(argv[1]) == "quad";
  const int B = quad ? 256 : (argc > 1 ? atoi(argv[1]) : 4096), T = 100, n = 12, m = 4;
  std::mt19937_64 g(1); std::uniform_real_distribution<double> U(-1, 1);
  auto mk = [&](size_t N, double sc, bool eye, int dim) { std::vector<double> v(N); for (auto& e : v) e = sc * U(g);
    if (eye) for (size_t b = 0; b < N / (dim * dim); ++b) for (int i = 0; i < dim; ++i) v[b * dim * dim + i * dim + i] += 1.0; return v; };
  auto A = mk((size_t)B * n * n, 0.02, true, n), Bm = mk((size_t)B * n * m, 0.1, false, 1);
  auto Q = mk((size_t)B * n * n, 0.01, true, n), R = mk((size_t)B * m * m, 0.01, true, m), Qf = mk((size_t)B * n * n, 0.01, true, n);
  auto x = mk((size_t)B * (T + 1) * n, 1.0, false, 1), u = mk((size_t)B * T * m, 0.1, false, 1);
  std::vector<double> Kor((size_t)B * T * m * n), dor((size_t)B * T * m);
  if (quad) {
    FILE* f = fopen("tools/quad256.bin", "rb");
    if (!f) { printf("tools/quad256.bin missing (python tools/dump_quad.py)\n"); return 1; }
    for (auto* v : {&A, &Bm, &Q, &R, &Qf, &x, &u, &Kor, &dor})
      if (fread(v->data(), 8, v->size(), f) != v->size()) { printf("short read\n"); return 1; }
    fclose(f);
  }
  auto up = [&](std::vector<double>& v) { double* p; hipMalloc(&p, v.size() * 8); hipMemcpy(p, v.data(), v.size() * 8, hipMemcpyHostToDevice); return p; };
  LQParams P{up(A), up(Bm), up(Q), up(R), up(Qf)};
  double *xd = up(x), *ud = up(u), *d, *K; int32_t* st;
  CK(hipMalloc(&d, (size_t)B * T * m * 8)); CK(hipMalloc(&K, (size_t)B * T * m * n * 8)); CK(hipMalloc(&st, B * 4));
  std::vector<double> Kref((size_t)B * T * m * n), dref((size_t)B * T * m), Kv(Kref.size()), dv(dref.size());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto time = [&](const char* name, auto launch) -> int {
    for (int i = 0; i < 150; ++i) launch();
    CK(hipDeviceSynchronize());
    const int R = 30;
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-36s B=%d %8.1f us\n", name, B, 1000.0 * ms / R);
    return 0;
  };
  auto prod = [&] { (void)launch_lq_backward_v6(12, 4, P, B, T, xd, ud, d, K, st, 0.01, 0); };
  auto bw4 = [&] { (void)launch_lq_backward4(P, B, T, xd, ud, d, K, st, 0.01, 0); };
  auto rel = [](const std::vector<double>& a, const std::vector<double>& r, const char* nm) {
    double mx = 0, ref = 0; size_t bad = 0, at = 0;
    for (size_t i = 0; i < a.size(); ++i) {
      if (!(fabs(a[i] - r[i]) <= mx)) { if (a[i] != a[i]) { ++bad; continue; } mx = fabs(a[i] - r[i]); at = i; }
      ref = fmax(ref, fabs(r[i]));
    }
    printf("%s: max |diff| %.3e (at %zu: %.17g vs %.17g), max |ref| %.3e, rel %.3e, NaN %zu\n", nm, mx, at, a[at], r[at], ref, mx / ref, bad);
  };
  if (time("product (1 trajectory / wave)", prod)) return 1;
  CK(hipMemcpy(Kref.data(), K, Kref.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(dref.data(), d, dref.size() * 8, hipMemcpyDeviceToHost));
  if (quad) {  // errors against the oracle; the v6 kernel's first
    printf("reference: symmetrised C oracle\n");
    Kv = Kref; dv = dref; Kref = Kor; dref = dor;
    rel(Kv, Kref, "v6 K"); rel(dv, dref, "v6 d");
  }
  CK(hipMemset(K, 0xff, Kref.size() * 8)); CK(hipMemset(d, 0xff, dref.size() * 8));
  bw4(); CK(hipDeviceSynchronize());
  CK(hipMemcpy(Kv.data(), K, Kv.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(dv.data(), d, dv.size() * 8, hipMemcpyDeviceToHost));
  rel(Kv, Kref, "K"); rel(dv, dref, "d");
  auto diff = [&](const char* name) -> int {
    CK(hipMemset(K, 0xff, Kref.size() * 8)); CK(hipMemset(d, 0xff, dref.size() * 8));
    CK(hipDeviceSynchronize());
    return 0;
  };
  (void)diff;
#define VAR(ABLV, NAME) do { \
    auto f = [&] { lq_backward4_kernel<ABLV><<<bw4_grid(B), 256, 0, 0>>>(P, B, T, xd, ud, d, K, st, 0.01); }; \
    if (time(NAME, f)) return 1; \
    if (((ABLV) & 79) == 0) { \
      CK(hipMemcpy(Kv.data(), K, Kv.size() * 8, hipMemcpyDeviceToHost)); \
      CK(hipMemcpy(dv.data(), d, dv.size() * 8, hipMemcpyDeviceToHost)); \
      rel(Kv, Kref, "  K"); rel(dv, dref, "  d"); } } while (0)
  if (argc > 2) {  // scan mode: default variant only
    for (int rep = 0; rep < 2; ++rep) { if (time("product (1 trajectory / wave)", prod)) return 1; VAR(0, "bw4"); }
    return 0;
  }
  for (int rep = 0; rep < 2; ++rep) {
    if (time("product (1 trajectory / wave)", prod)) return 1;
    VAR(0, "bw4 (sweeps, Lz4)");
    VAR(512, "bw4 stores aux=1");
    VAR(1024, "bw4 stores aux=2");
    VAR(1536, "bw4 stores aux=3");
    VAR(8, "bw4 -stores");
  }
  return 0;
}
