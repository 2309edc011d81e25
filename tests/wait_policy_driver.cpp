// Drives ilqr.jl_amd/csrc/ilqr_wait.h (the host's end-of-fit wait) with simulated
// completions: done() turns true at a chosen time after the wait starts. Prints one
// line per scenario: "<name> <median latency µs> <max latency µs>", the latency being
// how long after the simulated completion the wait returned (tests/test_wait_policy.py).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "ilqr_wait.h"

using clk = std::chrono::steady_clock;

// one wait of `units` iterations whose work completes `done_us` after the wait starts;
// → the return latency past the completion, µs
static double one_wait(ilqr::HostWait* hw, int units, int64_t done_us) {
  const auto t0 = clk::now();
  const auto tdone = t0 + std::chrono::microseconds(done_us);
  auto done = [&] { return clk::now() >= tdone; };
  auto idle = [&] { return done() ? 0 : 1; };  // 0 = ok, 1 = not ready
  const int e = ilqr::nap_spin_wait(hw, units, 0, 1, done, idle);
  const auto t1 = clk::now();
  if (e != 0) return 1e9;
  return std::chrono::duration<double, std::micro>(t1 - tdone).count();
}

static void report(const char* name, std::vector<double> v) {
  std::sort(v.begin(), v.end());
  std::printf("%s %.2f %.2f\n", name, v[v.size() / 2], v.back());
}

int main() {
  const int reps = 15;
  // the driver's --steps 20 region: 3-iteration fits (≈450 µs), then a 2-iteration fit
  // (≈300 µs) — completion earlier than the previous wait
  {
    std::vector<double> lat;
    for (int r = 0; r < reps; ++r) {
      ilqr::HostWait hw;
      for (int k = 0; k < 3; ++k) one_wait(&hw, 3, 450);
      lat.push_back(one_wait(&hw, 2, 300));
    }
    report("short_tail_fit", lat);
  }
  // a 1-iteration warmup fit, then a 3-iteration fit (completion later than the previous wait)
  {
    std::vector<double> lat;
    for (int r = 0; r < reps; ++r) {
      ilqr::HostWait hw;
      one_wait(&hw, 1, 150);
      lat.push_back(one_wait(&hw, 3, 450));
    }
    report("after_short_fit", lat);
  }
  // same units, completion at 60 % of the previous wait (a faster fit)
  {
    std::vector<double> lat;
    for (int r = 0; r < reps; ++r) {
      ilqr::HostWait hw;
      one_wait(&hw, 3, 450);
      lat.push_back(one_wait(&hw, 3, 270));
    }
    report("faster_same_units", lat);
  }
  // a long wait (5 ms per iteration): the nap ends before the expected end, the spin sees it
  {
    std::vector<double> lat;
    for (int r = 0; r < 5; ++r) {
      ilqr::HostWait hw;
      one_wait(&hw, 1, 5000);
      lat.push_back(one_wait(&hw, 1, 4950));
    }
    report("long_near_estimate", lat);
  }
  // a long wait that completes far earlier than expected (tol-converged): at most one nap late
  {
    std::vector<double> lat;
    for (int r = 0; r < 5; ++r) {
      ilqr::HostWait hw;
      one_wait(&hw, 1, 5000);
      lat.push_back(one_wait(&hw, 1, 2000));
    }
    report("long_early", lat);
  }
  // no estimate yet, work longer than the 1 ms spin budget: the nap-between-queries phase
  {
    std::vector<double> lat;
    for (int r = 0; r < 5; ++r) {
      ilqr::HostWait hw;
      lat.push_back(one_wait(&hw, 3, 3000));
    }
    report("cold_long", lat);
  }
  // the estimate is per iteration: 3 × 150 µs waits → 150 µs per unit
  {
    ilqr::HostWait hw;
    one_wait(&hw, 3, 450);
    std::printf("us_per_unit %lld\n", (long long)hw.us_per_unit);
  }
  return 0;
}
