// Probe for backward-kernel schedules (not part of the product): times the v7
// four-trajectories-per-wave kernel (lq_backward4_kernel) against the v8 schedule
// variants (lq_backward4_v8_kernel) at B=4096, T=100 on random stable LQ problems,
// checks the variants return v7's bits, and (argv[1] = "quad") their error against the
// symmetrised C oracle on tools/quad256.bin (tools/dump_quad.py).
#include "../ilqr.jl_amd/csrc/ilqr_lq.hip"
#include "../ilqr.jl_amd/csrc/ilqr_bw4.hip"
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>
using namespace ilqr;
#define CK(x) do { hipError_t e=(x); if(e!=hipSuccess){printf("err %s line %d\n",hipGetErrorString(e),__LINE__); return 1;} } while(0)

int main(int argc, char** argv) {
  const bool quad = argc > 1 && std::string(argv[1]) == "quad";
  const int B = quad ? 256 : (argc > 1 ? atoi(argv[1]) : 4096), T = 100, n = 12, m = 4;
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> U(-1, 1);
  auto mk = [&](size_t N, double sc, bool eye, int dim) {
    std::vector<double> v(N);
    for (auto& e : v) e = sc * U(g);
    if (eye) for (size_t b = 0; b < N / (dim * dim); ++b) for (int i = 0; i < dim; ++i) v[b * dim * dim + i * dim + i] += 1.0;
    return v;
  };
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
  double *xd = up(x), *ud = up(u), *d, *K;
  int32_t* st;
  CK(hipMalloc(&d, (size_t)B * T * m * 8)); CK(hipMalloc(&K, (size_t)B * T * m * n * 8)); CK(hipMalloc(&st, B * 4));
  std::vector<double> K7((size_t)B * T * m * n), d7((size_t)B * T * m), Kv(K7.size()), dv(d7.size());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto time = [&](const char* name, auto launch) -> int {
    for (int i = 0; i < 200; ++i) launch();
    CK(hipDeviceSynchronize());
    const int R = 50;
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-40s B=%d %8.2f us\n", name, B, 1000.0 * ms / R);
    return 0;
  };
  auto rel = [](const std::vector<double>& a, const std::vector<double>& r, const char* nm) {
    double mx = 0, ref = 0; size_t bad = 0;
    for (size_t i = 0; i < a.size(); ++i) {
      if (a[i] != a[i]) { ++bad; continue; }
      mx = fmax(mx, fabs(a[i] - r[i])); ref = fmax(ref, fabs(r[i]));
    }
    printf("  %s: rel %.3e NaN %zu\n", nm, mx / ref, bad);
  };
  auto v7 = [&] { lq_backward4_kernel<0><<<bw4_grid(B), 256, 0, 0>>>(P, B, T, xd, ud, d, K, st, 0.01); };
  if (time("v7 lq_backward4_kernel", v7)) return 1;
  CK(hipMemcpy(K7.data(), K, K7.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(d7.data(), d, d7.size() * 8, hipMemcpyDeviceToHost));
  if (quad) { rel(K7, Kor, "v7 K vs oracle"); rel(d7, dor, "v7 d vs oracle"); }
  auto check = [&](const char* nm) -> int {
    CK(hipMemcpy(Kv.data(), K, Kv.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(dv.data(), d, dv.size() * 8, hipMemcpyDeviceToHost));
    const bool same = !memcmp(Kv.data(), K7.data(), Kv.size() * 8) && !memcmp(dv.data(), d7.data(), dv.size() * 8);
    printf("  %s: bits %s v7\n", nm, same ? "==" : "!=");
    if (!same) { rel(Kv, K7, "K vs v7"); rel(dv, d7, "d vs v7"); }
    if (quad) { rel(Kv, Kor, "K vs oracle"); rel(dv, dor, "d vs oracle"); }
    return 0;
  };
#define VAR8(SGV, NAME) do { \
    CK(hipMemset(K, 0xff, K7.size() * 8)); CK(hipMemset(d, 0xff, d7.size() * 8)); \
    auto f = [&] { lq_backward4_v8_kernel<SGV><<<bw4_grid(B), 256, 0, 0>>>(P, B, T, xd, ud, d, K, st, 0.01); }; \
    if (time(NAME, f)) return 1; \
    if (check(NAME)) return 1; } while (0)
  for (int rep = 0; rep < 2; ++rep) {
    if (time("v7 lq_backward4_kernel", v7)) return 1;
    VAR8(0, "v8 reordered");
  }
  // cycles per step and the clock, from the waves' own counters
  {
    unsigned long long* clk;
    const int nw = (B + 3) / 4;
    CK(hipMalloc(&clk, 16 * nw));
    for (int i = 0; i < 100; ++i) v7();
    lq_backward4_v8_kernel<2><<<bw4_grid(B), 256, 0, 0>>>(P, B, T, xd, ud, d, K, st, 0.01, clk);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> c(2 * nw);
    CK(hipMemcpy(c.data(), clk, 16 * nw, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0, cmax = 0;
    for (int w = 0; w < nw; ++w) { cyc += c[2 * w]; rt += c[2 * w + 1]; cmax = fmax(cmax, (double)c[2 * w]); }
    cyc /= nw; rt /= nw;
    printf("v8 loop: %.0f shader cycles (max %.0f) = %.1f cycles/step, %.2f us at 100 MHz real time -> %.3f GHz\n",
           cyc, cmax, cyc / T, rt / 100.0, cyc / (rt / 100.0) / 1000.0);
  }
  return 0;
}
