// (Round 3: the ABL bits / -DILQR_* switches this probe uses exist only in the tree
// tools/archive/ablation/restore_tree.sh restores; build it there.)
// Probe: the 2-link forward kernel (ilqr_twolink.hip) at BASELINE config 2's size,
// B = 1024, T = 50 (argv: B T), for the build variants of the rollout
// (-DILQR_TL_RK4_SHIFT=0/1, -DILQR_FW_GROUP_PF), the line-search lanes per trajectory L and
// the waves per workgroup W, with one accepted trial (prev_cost = +Inf) and with a
// four-trial search (prev_cost = −Inf, max_trials = 4: exhausted after trial 4). Prints
// one JSON line per NU. Build: tools/archive/tl_fw_probe.sh.
#include "../ilqr.jl_amd/csrc/ilqr_twolink.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(e) do { hipError_t _e = (e); if (_e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(_e), __LINE__); exit(1); } } while (0)

namespace ilqr {
namespace {

template <int NU, int L, int W>
double time_fw(const TwoLinkParams& P, int B, int T, const double* x, const double* u, const double* d,
               const double* K, const double* pc, double* xn, double* un, double* nc, int32_t* tr,
               int32_t* st, LSParams ls, int reps) {
  const int grid = (L * B + 64 * W - 1) / (64 * W);
  for (int i = 0; i < 20; ++i)
    tl_forward_kernel<NU, L, W><<<grid, 64 * W>>>(P, B, T, x, u, nullptr, d, K, pc, xn, un, nc, tr, st, ls);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i)
    tl_forward_kernel<NU, L, W><<<grid, 64 * W>>>(P, B, T, x, u, nullptr, d, K, pc, xn, un, nc, tr, st, ls);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return 1000.0 * ms / reps;
}

template <int NU>
void run(int B, int T) {
  const TwoLinkParams P = two_link_params();
  std::vector<double> hx((size_t)B * (T + 1) * 4), hu((size_t)B * T * NU), hd((size_t)B * T * NU),
      hK((size_t)B * T * NU * 4);
  srand(7);
  auto rnd = [] { return rand() / (double)RAND_MAX; };
  for (auto& v : hx) v = rnd();
  for (auto& v : hu) v = 0.2 * (rnd() - 0.5);
  for (auto& v : hd) v = 0.1 * (rnd() - 0.5);
  for (auto& v : hK) v = 0.1 * (rnd() - 0.5);
  double *x, *u, *d, *K, *pinf, *pneg, *xn, *un, *nc;
  int32_t *tr, *st;
  CK(hipMalloc(&x, hx.size() * 8)); CK(hipMalloc(&u, hu.size() * 8)); CK(hipMalloc(&d, hd.size() * 8));
  CK(hipMalloc(&K, hK.size() * 8)); CK(hipMalloc(&xn, hx.size() * 8)); CK(hipMalloc(&un, hu.size() * 8));
  CK(hipMalloc(&pinf, B * 8)); CK(hipMalloc(&pneg, B * 8)); CK(hipMalloc(&nc, B * 8));
  CK(hipMalloc(&tr, B * 4)); CK(hipMalloc(&st, B * 4));
  CK(hipMemcpy(x, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(u, hu.data(), hu.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d, hd.data(), hd.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(K, hK.data(), hK.size() * 8, hipMemcpyHostToDevice));
  std::vector<double> inf(B, INFINITY), neg(B, -INFINITY);
  CK(hipMemcpy(pinf, inf.data(), B * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(pneg, neg.data(), B * 8, hipMemcpyHostToDevice));
  LSParams ls{0.0, 1.0, 0.5, 1e-6, 4};
  const int reps = 200;
  printf("{\"nu\": %d, \"B\": %d, \"T\": %d, \"rk4_shift\": %d, \"pf\": %d", NU, B, T,
         ILQR_TL_RK4_SHIFT, ILQR_FW_GROUP_PF);
  auto both = [&](const char* tag, auto f) {
    printf(", \"us_%s_trial1\": %.2f, \"us_%s_trials4\": %.2f", tag, f(pinf), tag, f(pneg));
  };
  both("L4W1", [&](double* pc) { return time_fw<NU, 4, 1>(P, B, T, x, u, d, K, pc, xn, un, nc, tr, st, ls, reps); });
  both("L4W4", [&](double* pc) { return time_fw<NU, 4, 4>(P, B, T, x, u, d, K, pc, xn, un, nc, tr, st, ls, reps); });
  both("L1W1", [&](double* pc) { return time_fw<NU, 1, 1>(P, B, T, x, u, d, K, pc, xn, un, nc, tr, st, ls, reps); });
  both("L1W4", [&](double* pc) { return time_fw<NU, 1, 4>(P, B, T, x, u, d, K, pc, xn, un, nc, tr, st, ls, reps); });
  printf("}\n");
  CK(hipFree(x)); CK(hipFree(u)); CK(hipFree(d)); CK(hipFree(K)); CK(hipFree(xn)); CK(hipFree(un));
  CK(hipFree(pinf)); CK(hipFree(pneg)); CK(hipFree(nc)); CK(hipFree(tr)); CK(hipFree(st));
}

}  // namespace
}  // namespace ilqr

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024;
  const int T = argc > 2 ? atoi(argv[2]) : 50;
  ilqr::run<1>(B, T);
  ilqr::run<2>(B, T);
  return 0;
}
