// Probe (round 4): is the 2-link forward's per-step time set by the latency of one
// rollout's dependent RK4 chain or by the wave's instruction issue? The verdict's two
// candidate cuts differ exactly there: interleaving C independent rollouts per lane only
// pays when the chain leaves issue slots idle (latency-bound); splitting one rollout over
// lanes only pays when it does not.
//
// Kernel: every lane runs T steps of the product's rk4_roll<NU> (ilqr_twolink.hip, the
// forward's branch-free RK4 with the carried sin/cos) on C independent states, the steps
// of the C chains interleaved in program order (the compiler schedules them together: one
// basic block per step). Grid: `waves` one-wave workgroups (64 = BASELINE config 2's
// forward at B = 1024 with four candidate lanes; 1024 = one wave per SIMD). Prints ns per
// step for C = 1, 2, 4 — if C = 2 costs ≈ C = 1, the chain is latency-bound and two
// rollouts per lane are nearly free; if ≈ 2×, the wave is issue-bound and ILP buys
// nothing. Also times the product forward kernel (tl_forward_kernel<1, 4, 1>) at B = 1024,
// T = 50 for the per-step figure of the real pass. Build: tools/archive/tl_ilp_probe.sh.
#include "../ilqr.jl_amd/csrc/ilqr_twolink.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(e) do { hipError_t _e = (e); if (_e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(_e), __LINE__); exit(1); } } while (0)

namespace ilqr {
namespace {

template <int NU, int C>
__global__ __launch_bounds__(64) void rk4_chain_kernel(TwoLinkParams P, int T, double* out) {
  const TLRoll R = tl_roll_consts(P);
  const int g = blockIdx.x * 64 + threadIdx.x;
  double x[C][4];
  double u[C][NU];
  TLCarry cy[C];
  bool bad = false;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    x[c][0] = 0.1 + 1e-6 * g;
    x[c][1] = -0.1 + 1e-3 * c;
    x[c][2] = 0.01 * c;
    x[c][3] = 0.0;
#pragma unroll
    for (int a = 0; a < NU; ++a) u[c][a] = 0.05 * (a + 1) + 0.01 * c;
    sincos_reduced(x[c][1], cy[c].s, cy[c].c);
  }
  for (int t = 0; t < T; ++t) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      double xn[4];
      rk4_roll<NU>(R, x[c], u[c], xn, bad, cy[c]);
#pragma unroll
      for (int i = 0; i < 4; ++i) x[c][i] = xn[i];
    }
  }
  double s = bad ? 1.0 : 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) s += x[c][0] + x[c][1] + x[c][2] + x[c][3];
  out[g] = s;
}

template <int NU, int C>
double time_chain(const TwoLinkParams& P, int waves, int T, double* out, int reps) {
  for (int i = 0; i < 5; ++i) rk4_chain_kernel<NU, C><<<waves, 64>>>(P, T, out);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) rk4_chain_kernel<NU, C><<<waves, 64>>>(P, T, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return 1e6 * ms / reps / T;  // ns per step
}

double time_forward(const TwoLinkParams& P, int B, int T, int reps) {
  constexpr int NU = 1;
  std::vector<double> hx((size_t)B * (T + 1) * 4), hu((size_t)B * T * NU), hd((size_t)B * T * NU),
      hK((size_t)B * T * NU * 4);
  srand(7);
  auto rnd = [] { return rand() / (double)RAND_MAX; };
  for (auto& v : hx) v = rnd();
  for (auto& v : hu) v = 0.2 * (rnd() - 0.5);
  for (auto& v : hd) v = 0.1 * (rnd() - 0.5);
  for (auto& v : hK) v = 0.1 * (rnd() - 0.5);
  double *x, *u, *d, *K, *xn, *un, *nc;
  int32_t *tr, *st;
  CK(hipMalloc(&x, hx.size() * 8));
  CK(hipMalloc(&u, hu.size() * 8));
  CK(hipMalloc(&d, hd.size() * 8));
  CK(hipMalloc(&K, hK.size() * 8));
  CK(hipMalloc(&xn, hx.size() * 8));
  CK(hipMalloc(&un, hu.size() * 8));
  CK(hipMalloc(&nc, B * 8));
  CK(hipMalloc(&tr, B * 4));
  CK(hipMalloc(&st, B * 4));
  CK(hipMemcpy(x, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(u, hu.data(), hu.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d, hd.data(), hd.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(K, hK.data(), hK.size() * 8, hipMemcpyHostToDevice));
  const LSParams ls{0.01, 1.0, 0.5, -1.0, 64};
  const int grid = (4 * B + 63) / 64;
  for (int i = 0; i < 20; ++i)
    tl_forward_kernel<NU, 4, 1><<<grid, 64>>>(P, B, T, x, u, nullptr, d, K, nullptr, xn, un, nc, tr, st, ls);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i)
    tl_forward_kernel<NU, 4, 1><<<grid, 64>>>(P, B, T, x, u, nullptr, d, K, nullptr, xn, un, nc, tr, st, ls);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  for (double* p : {x, u, d, K, xn, un, nc}) CK(hipFree(p));
  CK(hipFree(tr));
  CK(hipFree(st));
  return 1e6 * ms / reps / T;
}

}  // namespace
}  // namespace ilqr

int main() {
  using namespace ilqr;
  const TwoLinkParams P = two_link_params();
  const int T = 400, reps = 50;
  double* out;
  CK(hipMalloc(&out, 1024 * 64 * 8));
  printf("{\"probe\": \"tl_ilp\", \"forward_kernel_ns_per_step_B1024_T50_nu1\": %.1f", time_forward(P, 1024, 50, 200));
  for (int waves : {64, 1024}) {
    printf(", \"waves%d\": {\"nu1_C1\": %.1f, \"nu1_C2\": %.1f, \"nu1_C4\": %.1f, \"nu2_C1\": %.1f, \"nu2_C2\": %.1f}",
           waves, time_chain<1, 1>(P, waves, T, out, reps), time_chain<1, 2>(P, waves, T, out, reps),
           time_chain<1, 4>(P, waves, T, out, reps), time_chain<2, 1>(P, waves, T, out, reps),
           time_chain<2, 2>(P, waves, T, out, reps));
  }
  printf(", \"unit\": \"ns per RK4 step (all C chains of a lane)\"}\n");
  CK(hipFree(out));
  return 0;
}
