// Timeline probe for the pipelined iteration (not part of the product): runs the
// pipe kernel's two roles at steady state (cur = prev = one cold-start iterate, as in
// the middle launches of a pipelined fit) at B=4096, T=100, recording s_memtime per
// workgroup at start / after phase 1 / after the barrier / at the end, plus the CU
// it ran on, then prints per-role phase durations and the launch span.
#include "../ilqr.jl_amd/csrc/ilqr_lq.hip"
#include <algorithm>
#include <cstdio>
#include <map>
#include <random>
#include <vector>
using namespace ilqr;

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memtime(); }

template <int MODE>  // 0: roles as in the product; 1: every WG role B (no overlap)
__global__ __launch_bounds__(256, 4) void probe_kernel(LQParams P, int B, int T, IterArgs a, LSParams ls,
                                                       unsigned long long* ts, unsigned* hw) {
  __shared__ __attribute__((aligned(16))) double lds[PIPE_LDS];
  const int w = threadIdx.x >> 6;
  const int b0 = blockIdx.x * WAVES_PER_WG;
  const bool role_a = MODE == 0 && pipe_role_a(blockIdx.x);
  unsigned long long t0 = now(), t1, t2;
  auto fw = [&]() { if (w == 0) iter_forward_wave<12, 4>(P, b0, B, T, a, ls, lds); };
  auto bw = [&]() {
    const int b = b0 + w;
    if (b < B) (void)lq_backward_wave<12, 4>(P, b, T, a.x, a.u, a.d, a.K, ls.mu, lds + w * BW_LDS);
  };
  if (role_a) fw(); else bw();
  t1 = now();
  __syncthreads();
  t2 = now();
  if (role_a) bw(); else fw();
  __syncthreads();
  if (threadIdx.x == 0) {
    ts[blockIdx.x * 4 + 0] = t0;
    ts[blockIdx.x * 4 + 1] = t1;
    ts[blockIdx.x * 4 + 2] = t2;
    ts[blockIdx.x * 4 + 3] = now();
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    // HW_ID: cu_id [11:8], sh_id [12], se_id [14:13]; XCC_ID [3:0]
    hw[blockIdx.x] = ((id >> 8) & 0x7f) | ((xcc & 0xf) << 8);
  }
}

#define CK(x) do { hipError_t e=(x); if(e!=hipSuccess){printf("err %s line %d\n",hipGetErrorString(e),__LINE__); return 1;} } while(0)

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
  double *xd = up(x), *ud = up(u), *d, *K, *xn, *un, *cost;
  int32_t *st, *tr;
  CK(hipMalloc(&d, (size_t)B * T * m * 8)); CK(hipMalloc(&K, (size_t)B * T * m * n * 8));
  CK(hipMalloc(&xn, x.size() * 8)); CK(hipMalloc(&un, u.size() * 8)); CK(hipMalloc(&cost, B * 8));
  CK(hipMalloc(&st, B * 4)); CK(hipMalloc(&tr, B * 4));
  CK(hipMemset(st, 0, B * 4)); CK(hipMemset(d, 0, (size_t)B * T * m * 8)); CK(hipMemset(K, 0, (size_t)B * T * m * n * 8));
  IterArgs a{};
  a.x = xd; a.u = ud; a.xtraj = nullptr; a.xnew = xn; a.unew = un; a.K = K; a.d = d;
  a.prev_cost = nullptr; a.new_cost = cost; a.trials = tr; a.status = st;
  LSParams ls{0.01, 1.0, 0.5, -1.0, 64};
  const int grid = B / 4;
  unsigned long long* ts; unsigned* hw;
  CK(hipMalloc(&ts, grid * 4 * 8)); CK(hipMalloc(&hw, grid * 4));
  std::vector<unsigned long long> h(grid * 4); std::vector<unsigned> hh(grid);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto report = [&](const char* name, auto kern) -> int {
    for (int i = 0; i < 300; ++i) kern<<<grid, 256>>>(P, B, T, a, ls, ts, hw);  // clock warm-up
    CK(hipDeviceSynchronize());
    const int reps = 50;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) kern<<<grid, 256>>>(P, B, T, a, ls, ts, hw);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(h.data(), ts, h.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hh.data(), hw, hh.size() * 4, hipMemcpyDeviceToHost));
    unsigned long long lo = ~0ull, hi = 0;
    for (int b = 0; b < grid; ++b) { lo = std::min(lo, h[b * 4]); hi = std::max(hi, h[b * 4 + 3]); }
    // s_memtime counts shader-clock ticks
    double sum[2][3] = {}, cnt[2] = {}, start_max = 0;
    std::map<unsigned, int> per_cu_a, per_cu;
    for (int b = 0; b < grid; ++b) {
      const int r = pipe_role_a(b) ? 1 : 0;
      sum[r][0] += h[b * 4 + 1] - h[b * 4 + 0];
      sum[r][1] += h[b * 4 + 2] - h[b * 4 + 1];
      sum[r][2] += h[b * 4 + 3] - h[b * 4 + 2];
      cnt[r] += 1;
      start_max = std::max(start_max, (double)(h[b * 4] - lo));
      per_cu[hh[b]]++;
      per_cu_a[hh[b]] += r;
    }
    int mixed = 0, cus = (int)per_cu.size();
    std::map<int, int> hist;  // number of A workgroups on a CU → CUs
    for (auto& kv : per_cu) { mixed += (per_cu_a[kv.first] * 2 == kv.second); hist[per_cu_a[kv.first] * 10 + kv.second]++; }
    printf("    CU histogram (A WGs, WGs per CU) -> CUs:");
    for (auto& kv : hist) printf("  (%d,%d)->%d", kv.first / 10, kv.first % 10, kv.second);
    printf("\n");
    printf("%-28s %8.1f us/launch  span %7.0f ticks  last WG start %6.0f ticks  CUs %d (half-A %d)\n", name,
           1000.0 * ms / reps, (double)(hi - lo), start_max, cus, mixed);
    for (int r = 0; r < 2; ++r)
      if (cnt[r] > 0)
        printf("    role %c: phase1 %7.0f  barrier wait %7.0f  phase2 %7.0f ticks (mean over %d WGs)\n", r ? 'A' : 'B',
               sum[r][0] / cnt[r], sum[r][1] / cnt[r], sum[r][2] / cnt[r], (int)cnt[r]);
    return 0;
  };
  if (report("pipe (roles A/B)", probe_kernel<0>)) return 1;
  if (report("all role B (bw then fw)", probe_kernel<1>)) return 1;
  return 0;
}
