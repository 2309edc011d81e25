// Host sanitizer driver for the C ABI runtime (ilqr_abi.cpp, ilqr_multi.cpp and the
// host halves of the HIP sources), built with -fsanitize=address,undefined or
// -fsanitize=thread on the HOST side only (-Xarch_host; device code is not
// instrumented) by `make -C ilqr.jl_amd/csrc san SAN=address|thread`, and run by
// tools/san/run_cpu.sh (no GPU: argument validation and every error path) and
// tools/san/run_gpu.sh (a GPU: small fits through every entry point, the multi-device
// calls' host threads included). SURVEY §5. Exit 0 on success.
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/ilqr.h"

static int fails = 0;
#define CHECK(c, ...)                                   \
  do {                                                  \
    if (!(c)) {                                         \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                \
      std::fputc('\n', stderr);                         \
      ++fails;                                          \
    }                                                   \
  } while (0)

extern "C" int hipGetDeviceCount(int*);
extern "C" int hipSetDevice(int);
extern "C" int hipFree(void*);
extern "C" int hipDeviceSynchronize(void);
extern "C" int hipMemGetInfo(size_t*, size_t*);

// the reference's RBD script model (2Dof_arm.urdf floating, zero gravity, its costs)
static ilqr_floating floating_model() {
  ilqr_floating m{};
  m.n_joints = 2;
  m.dt = 0.01;
  m.base_mass = 30.0;
  for (int k = 0; k < 3; ++k) {
    m.base_inertia[4 * k] = 50.0;
    for (int j = 0; j < 2; ++j) {
      m.joint_rot[j][4 * k] = 1.0;
      m.inertia[j][4 * k] = 0.5;
    }
  }
  m.mass[0] = m.mass[1] = 3.0;
  m.joint_pos[0][0] = m.joint_pos[0][1] = 0.5;
  m.joint_pos[1][0] = 1.0;
  m.axis[0][2] = 1.0;
  m.axis[1][1] = 1.0;
  const double tgt[8] = {0, 0, 0, 5, 1, 2, 1, .3}, qw[8] = {100, 100, 100, 1, 1, 1, 10, 10},
               rw[8] = {1, 1, 1, 100, 100, 100, 10, 10}, qfw[8] = {100, 100, 100, 1000, 1000, 1000, 10, 10};
  for (int i = 0; i < 8; ++i) {
    m.target[i] = tgt[i];
    m.q_weight[i] = qw[i];
    m.r_weight[i] = rw[i];
    m.qf_weight[i] = qfw[i];
  }
  m.q_scale = 10.0;
  m.r_scale = 1.0;
  m.qf_scale = 100000.0;
  return m;
}

static void no_gpu_paths() {
  CHECK(ilqr_abi_version() > 0, "abi version");
  for (int s = 0; s <= 7; ++s) CHECK(std::strlen(ilqr_status_string((ilqr_status)s)) > 0, "status string %d", s);
  CHECK(ilqr_last_error() != nullptr, "last error");
  ilqr_options o;
  ilqr_default_options(&o);
  ilqr_default_options(nullptr);
  CHECK(o.max_iter == 100 && o.max_trials == 64 && o.mu == 0.01, "default options");
  CHECK(ilqr_supported(ILQR_PROBLEM_LQ, 12, 4) == 1 && ilqr_supported(ILQR_PROBLEM_LQ, 13, 4) == 0, "supported");
  CHECK(ilqr_supported(ILQR_PROBLEM_TWO_LINK, 4, 2) == 1 && ilqr_supported(99, 1, 1) == 0, "supported kinds");
  ilqr_handle* h = nullptr;
  CHECK(ilqr_create(nullptr, 0, 12, 4, 10, 8) == ILQR_ERR_BAD_ARG, "create null out");
  CHECK(ilqr_create(&h, 0, 0, 4, 10, 8) == ILQR_ERR_BAD_DIMS && !h, "create bad nx");
  CHECK(ilqr_create(&h, 0, 12, 4, -1, 8) == ILQR_ERR_BAD_DIMS && !h, "create bad T");
  CHECK(ilqr_create(&h, 0, 12, 4, 10, 0) == ILQR_ERR_BAD_DIMS && !h, "create bad batch");
  CHECK(ilqr_destroy(nullptr) == ILQR_OK, "destroy null");
  CHECK(ilqr_set_stream(nullptr, nullptr) == ILQR_ERR_BAD_ARG, "set_stream null");
  CHECK(ilqr_set_schedule(nullptr, 0) == ILQR_ERR_BAD_ARG, "set_schedule null");
  CHECK(ilqr_sync(nullptr) == ILQR_ERR_BAD_ARG, "sync null");
  ilqr_problem p{ILQR_PROBLEM_LQ, 0, nullptr, nullptr, nullptr, nullptr, nullptr};
  double buf[64] = {0};
  int32_t ibuf[8] = {0};
  CHECK(ilqr_backward(nullptr, &p, nullptr, buf, buf, buf, buf, ibuf) == ILQR_ERR_BAD_ARG, "backward null");
  CHECK(ilqr_forward(nullptr, &p, nullptr, buf, buf, nullptr, buf, buf, buf, buf, buf, buf, ibuf, ibuf) ==
            ILQR_ERR_BAD_ARG, "forward null");
  CHECK(ilqr_iterate(nullptr, &p, nullptr, buf, buf, nullptr, buf, buf, buf, buf, buf, ibuf, ibuf) ==
            ILQR_ERR_BAD_ARG, "iterate null");
  CHECK(ilqr_fit(nullptr, &p, nullptr, buf, buf, nullptr, buf, buf, buf, ibuf, ibuf) == ILQR_ERR_BAD_ARG, "fit null");
  ilqr_history hist{buf, ibuf, nullptr, nullptr};
  CHECK(ilqr_fit_ex(nullptr, &p, nullptr, buf, buf, nullptr, buf, buf, buf, ibuf, ibuf, &hist) == ILQR_ERR_BAD_ARG,
        "fit_ex null");
  CHECK(ilqr_backward_tiles(nullptr, nullptr, nullptr, buf, buf, ibuf) == ILQR_ERR_BAD_ARG, "tiles null");
  ilqr_multi* m = nullptr;
  int devs[2] = {0, 0};
  CHECK(ilqr_multi_create(&m, devs, 0, 12, 4, 10, 8) == ILQR_ERR_BAD_ARG && !m, "multi no devices");
  CHECK(ilqr_multi_create(&m, nullptr, 2, 12, 4, 10, 8) == ILQR_ERR_BAD_ARG, "multi null devices");
  CHECK(ilqr_multi_create(&m, devs, 2, 12, 0, 10, 8) == ILQR_ERR_BAD_DIMS && !m, "multi bad dims");
  CHECK(ilqr_multi_destroy(nullptr) == ILQR_OK, "multi destroy null");
  CHECK(ilqr_multi_set_schedule(nullptr, 0) == ILQR_ERR_BAD_ARG, "multi schedule null");
  CHECK(ilqr_multi_devices(nullptr) == 0, "multi devices null");
  CHECK(ilqr_multi_set_problem(nullptr, &p) == ILQR_ERR_BAD_ARG, "multi set_problem null");
  CHECK(ilqr_multi_load(nullptr, buf, buf, nullptr) == ILQR_ERR_BAD_ARG, "multi load null");
  CHECK(ilqr_multi_fit_resident(nullptr, nullptr, 0, nullptr) == ILQR_ERR_BAD_ARG, "multi fit_resident null");
  CHECK(ilqr_multi_gather(nullptr, buf, buf, buf, ibuf, ibuf) == ILQR_ERR_BAD_ARG, "multi gather null");
  CHECK(ilqr_multi_fit(nullptr, &p, nullptr, buf, buf, nullptr, buf, buf, buf, ibuf, ibuf) == ILQR_ERR_BAD_ARG,
        "multi fit null");
  CHECK(ilqr_host_alloc(16, nullptr) == ILQR_ERR_BAD_ARG && ilqr_host_free(nullptr) == ILQR_OK, "host alloc args");
  ilqr_chain c{};
  ilqr_chain_handle* ch = nullptr;
  CHECK(ilqr_chain_create(nullptr, 0, &c, 10, 8, ILQR_F64, ILQR_LINEARIZE_DUAL) == ILQR_ERR_BAD_ARG, "chain null");
  CHECK(ilqr_chain_create(&ch, 0, &c, 10, 8, ILQR_F64, ILQR_LINEARIZE_DUAL) == ILQR_ERR_BAD_DIMS, "chain no joints");
  c.n_joints = 2;
  c.nu = 2;
  c.dt = 0.01;
  CHECK(ilqr_chain_create(&ch, 0, &c, 10, 8, 7, ILQR_LINEARIZE_DUAL) == ILQR_ERR_BAD_ARG, "chain dtype");
  CHECK(ilqr_chain_create(&ch, 0, &c, 10, 8, ILQR_F64, 9) == ILQR_ERR_BAD_ARG, "chain linearisation");
  CHECK(ilqr_chain_fit(nullptr, nullptr, buf, buf, nullptr, buf, buf, buf, ibuf, ibuf) == ILQR_ERR_BAD_ARG,
        "chain fit null");
  CHECK(ilqr_chain_destroy(nullptr) == ILQR_OK, "chain destroy null");
  ilqr_floating fm = floating_model();
  ilqr_floating_handle* fh = nullptr;
  CHECK(ilqr_floating_create(nullptr, 0, &fm, 10, 2) == ILQR_ERR_BAD_ARG, "floating null");
  CHECK(ilqr_floating_create(&fh, 0, &fm, 0, 2) == ILQR_ERR_BAD_DIMS && !fh, "floating bad dims");
  fm.gravity[2] = -9.81;
  CHECK(ilqr_floating_create(&fh, 0, &fm, 10, 2) == ILQR_ERR_UNSUPPORTED && !fh, "floating gravity");
  fm = floating_model();
  fm.n_joints = 3;
  CHECK(ilqr_floating_create(&fh, 0, &fm, 10, 2) == ILQR_ERR_UNSUPPORTED && !fh, "floating joints");
  CHECK(ilqr_floating_fit(nullptr, nullptr, buf, buf, nullptr, buf, buf, buf, ibuf, ibuf) == ILQR_ERR_BAD_ARG,
        "floating fit null");
  CHECK(ilqr_floating_destroy(nullptr) == ILQR_OK, "floating destroy null");
  std::printf("no-GPU paths: %d failed checks\n", fails);
}

// a small LQ batch: A = I + small, B small, Q/R/Qf diagonal
struct LQ {
  int B, T, nx = 12, nu = 4;
  std::vector<double> A, Bm, Q, R, Qf, x, u;
  LQ(int b, int t) : B(b), T(t) {
    A.assign((size_t)B * nx * nx, 0.0);
    Bm.assign((size_t)B * nx * nu, 0.0);
    Q.assign((size_t)B * nx * nx, 0.0);
    R.assign((size_t)B * nu * nu, 0.0);
    Qf.assign((size_t)B * nx * nx, 0.0);
    x.assign((size_t)B * (T + 1) * nx, 0.0);
    u.assign((size_t)B * T * nu, 0.0);
    for (int b = 0; b < B; ++b) {
      for (int i = 0; i < nx; ++i) {
        A[(size_t)b * nx * nx + i * nx + i] = 1.0;
        if (i + 6 < nx) A[(size_t)b * nx * nx + i * nx + i + 6] = 0.05;
        Q[(size_t)b * nx * nx + i * nx + i] = 1.0 + 0.01 * b;
        Qf[(size_t)b * nx * nx + i * nx + i] = 10.0;
      }
      for (int i = 0; i < nu; ++i) {
        R[(size_t)b * nu * nu + i * nu + i] = 0.1;
        Bm[(size_t)b * nx * nu + (8 + i) * nu + i] = 0.05;
      }
      for (int t = 0; t <= T; ++t)
        for (int i = 0; i < 3; ++i) x[((size_t)b * (T + 1) + t) * nx + i] = 0.5 - 0.1 * i;
    }
  }
};

static void gpu_paths_body(int ndev);

// Device memory the process holds (total − free on device 0), after a synchronise.
static size_t device_bytes_in_use() {
  size_t fr = 0, tot = 0;
  hipDeviceSynchronize();
  if (hipMemGetInfo(&fr, &tot) != 0) return 0;
  return tot - fr;
}

static void gpu_paths(int ndev) {
  // every handle and buffer a round of the GPU paths creates is released before the round
  // returns: a later round leaves the device memory in use where it found it. (The first
  // round's delta is the HIP runtime's own one-time allocations — code objects loaded at
  // first launch, the private-segment (scratch) pool — which it keeps until exit.) Under
  // ASan's default quarantine the freed device blocks stay parked in the quarantine until
  // exit, so the check runs with quarantine_size_mb=0 (tools/san/run_gpu.sh)
  // and is only reported otherwise.
  (void)hipSetDevice(0);
  (void)hipFree(nullptr);
  size_t use[4];
  use[0] = device_bytes_in_use();
  for (int r = 1; r <= 3; ++r) {
    gpu_paths_body(ndev);
    use[r] = device_bytes_in_use();
  }
  const long long delta = (long long)use[3] - (long long)use[2];
  const char* opts = getenv("ASAN_OPTIONS");
  const bool no_quarantine = opts && strstr(opts, "quarantine_size_mb=0");
  std::printf("device memory in use: %zu B at start; after rounds 1, 2, 3: %zu, %zu, %zu B (round 1: the "
              "runtime's one-time allocations; round 3 − round 2: %lld B)%s\n", use[0], use[1], use[2], use[3], delta,
              no_quarantine || !opts ? "" : " [quarantine on: freed blocks held, not checked]");
  // a leak of ours would repeat every round; the runtime's sub-allocator works in 2 MiB chunks
  if (no_quarantine || !opts) CHECK(delta <= (2ll << 20), "every device buffer and handle released");
}

static void gpu_paths_body(int ndev) {
  const int B = 96, T = 20, it = 4;
  LQ lq(B, T);
  const size_t xb = lq.x.size() * 8, ub = lq.u.size() * 8;
  // one handle: host data through ilqr_memcpy_*, fit_ex with a full history, iterate
  ilqr_handle* h = nullptr;
  CHECK(ilqr_create(&h, 0, 12, 4, T, B) == ILQR_OK, "create");
  CHECK(ilqr_set_schedule(h, ILQR_SCHED_FUSED | ILQR_SCHED_BACKWARD_WAVE) == ILQR_ERR_BAD_ARG, "schedule combo");
  CHECK(ilqr_set_schedule(h, 1 << 20) == ILQR_ERR_BAD_ARG, "schedule bits");
  CHECK(ilqr_set_schedule(h, ILQR_SCHED_RING_FORWARD | ILQR_SCHED_FUSED | ILQR_SCHED_BACKWARD_BLOCK) == ILQR_OK,
        "schedule");
  void *dA, *dB, *dQ, *dR, *dQf, *dx, *du, *dxo, *duo, *dc, *di, *ds, *hc, *ht, *ha, *hd;
  for (void** q : {&dA, &dQ, &dQf}) ilqr_malloc(h, (size_t)B * 144 * 8, q);
  ilqr_malloc(h, (size_t)B * 48 * 8, &dB);
  ilqr_malloc(h, (size_t)B * 16 * 8, &dR);
  for (void** q : {&dx, &dxo}) ilqr_malloc(h, xb, q);
  for (void** q : {&du, &duo}) ilqr_malloc(h, ub, q);
  ilqr_malloc(h, B * 8, &dc);
  ilqr_malloc(h, B * 4, &di);
  ilqr_malloc(h, B * 4, &ds);
  for (void** q : {&hc, &ha, &hd}) ilqr_malloc(h, (size_t)it * B * 8, q);
  ilqr_malloc(h, (size_t)it * B * 4, &ht);
  ilqr_memcpy_h2d(h, dA, lq.A.data(), lq.A.size() * 8);
  ilqr_memcpy_h2d(h, dB, lq.Bm.data(), lq.Bm.size() * 8);
  ilqr_memcpy_h2d(h, dQ, lq.Q.data(), lq.Q.size() * 8);
  ilqr_memcpy_h2d(h, dR, lq.R.data(), lq.R.size() * 8);
  ilqr_memcpy_h2d(h, dQf, lq.Qf.data(), lq.Qf.size() * 8);
  ilqr_memcpy_h2d(h, dx, lq.x.data(), xb);
  ilqr_memcpy_h2d(h, du, lq.u.data(), ub);
  ilqr_problem p{ILQR_PROBLEM_LQ, 0, (double*)dA, (double*)dB, (double*)dQ, (double*)dR, (double*)dQf};
  ilqr_options o;
  ilqr_default_options(&o);
  o.max_iter = it;
  o.tol = -1.0;
  ilqr_history hs{(double*)hc, (int32_t*)ht, (double*)ha, (double*)hd};
  const ilqr_status fs = ilqr_fit_ex(h, &p, &o, (double*)dx, (double*)du, nullptr, (double*)dxo, (double*)duo,
                                     (double*)dc, (int32_t*)di, (int32_t*)ds, &hs);
  CHECK(fs == ILQR_OK || fs == ILQR_ERR_LS_EXHAUSTED, "fit_ex %d", (int)fs);
  std::vector<double> cost(B), hcost((size_t)it * B);
  ilqr_memcpy_d2h(h, cost.data(), dc, B * 8);
  ilqr_memcpy_d2h(h, hcost.data(), hc, hcost.size() * 8);
  for (int b = 0; b < B; ++b) CHECK(std::isfinite(cost[b]), "cost %d", b);
  CHECK(std::isfinite(hcost[0]), "history cost");
  CHECK(ilqr_iterate(h, &p, &o, (double*)dx, (double*)du, nullptr, (double*)dxo, (double*)duo, nullptr,
                     (double*)dc, nullptr, nullptr, (int32_t*)ds) == ILQR_OK, "iterate");
  CHECK(ilqr_sync(h) == ILQR_OK, "sync");
  for (void* q : {dA, dB, dQ, dR, dQf, dx, du, dxo, duo, dc, di, ds, hc, ht, ha, hd}) ilqr_free(h, q);
  ilqr_destroy(h);

  // multi-device: host path, then the resident calls (their host threads are what the
  // thread sanitizer watches), warm start, gather into pinned memory
  std::vector<int> devs(4);
  for (int i = 0; i < 4; ++i) devs[i] = i % ndev;
  ilqr_multi* m = nullptr;
  CHECK(ilqr_multi_create(&m, devs.data(), 4, 12, 4, T, B) == ILQR_OK, "multi create");
  // the single handle's schedule: its shards (B / 4 below BW4_MIN_BATCH) would otherwise
  // take the one-trajectory-per-wave backward, whose bits differ
  CHECK(ilqr_multi_set_schedule(m, ILQR_SCHED_RING_FORWARD | ILQR_SCHED_FUSED | ILQR_SCHED_BACKWARD_BLOCK) ==
            ILQR_OK, "multi schedule");
  ilqr_problem hp{ILQR_PROBLEM_LQ, 0, lq.A.data(), lq.Bm.data(), lq.Q.data(), lq.R.data(), lq.Qf.data()};
  std::vector<double> xo(lq.x.size()), uo(lq.u.size()), co(B);
  std::vector<int32_t> io(B), so(B);
  ilqr_status ms = ilqr_multi_fit(m, &hp, &o, lq.x.data(), lq.u.data(), nullptr, xo.data(), uo.data(), co.data(),
                                  io.data(), so.data());
  CHECK(ms == ILQR_OK || ms == ILQR_ERR_LS_EXHAUSTED, "multi fit %d", (int)ms);
  for (int b = 0; b < B; ++b) CHECK(co[b] == cost[b], "multi fit cost %d: %g vs %g", b, co[b], cost[b]);
  CHECK(ilqr_multi_set_problem(m, &hp) == ILQR_OK, "multi set_problem");
  CHECK(ilqr_multi_load(m, lq.x.data(), lq.u.data(), nullptr) == ILQR_OK, "multi load");
  CHECK(ilqr_multi_fit_resident(m, &o, 7, nullptr) == ILQR_ERR_BAD_ARG, "multi flags");
  ms = ilqr_multi_fit_resident(m, &o, 0, nullptr);
  CHECK(ms == ILQR_OK || ms == ILQR_ERR_LS_EXHAUSTED, "multi fit_resident %d", (int)ms);
  double* pinned = nullptr;
  CHECK(ilqr_host_alloc(B * 8, (void**)&pinned) == ILQR_OK, "host alloc");
  CHECK(ilqr_multi_gather(m, nullptr, nullptr, pinned, nullptr, nullptr) == ILQR_OK, "multi gather");
  for (int b = 0; b < B; ++b) CHECK(pinned[b] == cost[b], "resident cost %d", b);
  ms = ilqr_multi_fit_resident(m, &o, ILQR_MULTI_WARM_START, nullptr);
  CHECK(ms == ILQR_OK || ms == ILQR_ERR_LS_EXHAUSTED, "multi warm start %d", (int)ms);
  CHECK(ilqr_multi_gather(m, xo.data(), uo.data(), pinned, io.data(), so.data()) == ILQR_OK, "multi gather all");
  ilqr_host_free(pinned);
  ilqr_multi_destroy(m);

  // the floating-base family: the script's rest state, a 3-iteration fit of 3 trajectories
  {
    const int FB = 3, FT = 10;
    ilqr_floating fm = floating_model();
    ilqr_floating_handle* fh = nullptr;
    CHECK(ilqr_floating_create(&fh, 0, &fm, FT, FB) == ILQR_OK, "floating create");
    std::vector<double> fx((size_t)FB * (FT + 1) * 16, 0.0), fu((size_t)FB * FT * 8, 0.0);
    void *dfx, *dfu, *dfxo, *dfuo, *dfc;
    ilqr_handle* mh = nullptr;  // device-memory helper
    CHECK(ilqr_create(&mh, 0, 16, 8, FT, 1) == ILQR_OK, "helper create");
    for (void** q : {&dfx, &dfxo}) ilqr_malloc(mh, fx.size() * 8, q);
    for (void** q : {&dfu, &dfuo}) ilqr_malloc(mh, fu.size() * 8, q);
    ilqr_malloc(mh, FB * 8, &dfc);
    for (int b = 0; b < FB; ++b) {
      double* x0 = fx.data() + (size_t)b * (FT + 1) * 16;
      x0[2] = 1.0;
      x0[3] = 0.5;
      x0[4] = 0.75;
      x0[5] = 1.0;
      x0[8 + b] = 0.01;
    }
    ilqr_memcpy_h2d(mh, dfx, fx.data(), fx.size() * 8);
    ilqr_memcpy_h2d(mh, dfu, fu.data(), fu.size() * 8);
    // x_init = the rollout of u = 0 (the script's state_traj), one step at a time
    for (int t = 0; t < FT; ++t)
      for (int b = 0; b < FB; ++b) {
        double* xb = (double*)dfx + (size_t)b * (FT + 1) * 16;
        CHECK(ilqr_floating_dynamics(fh, xb + t * 16, (double*)dfu, xb + (t + 1) * 16, 1) == ILQR_OK, "dyn");
      }
    ilqr_options fo;
    ilqr_default_options(&fo);
    fo.max_iter = 3;
    const ilqr_status fs2 = ilqr_floating_fit(fh, &fo, (double*)dfx, (double*)dfu, nullptr, (double*)dfxo,
                                              (double*)dfuo, (double*)dfc, nullptr, nullptr);
    CHECK(fs2 == ILQR_OK, "floating fit %d", (int)fs2);
    std::vector<double> fc(FB);
    ilqr_memcpy_d2h(mh, fc.data(), dfc, FB * 8);
    for (int b = 0; b < FB; ++b) CHECK(std::isfinite(fc[b]), "floating cost %d", b);
    for (void* q : {dfx, dfu, dfxo, dfuo, dfc}) ilqr_free(mh, q);
    ilqr_destroy(mh);
    CHECK(ilqr_floating_destroy(fh) == ILQR_OK, "floating destroy");
  }
  std::printf("GPU paths (%d device(s)): %d failed checks\n", ndev, fails);
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);  // every line out before a crash at exit
  no_gpu_paths();
  int n = 0;
  if (hipGetDeviceCount(&n) == 0 && n > 0) gpu_paths(n);
  else {
    // the valid calls fail cleanly without a device: ILQR_ERR_HIP, nothing leaked
    ilqr_handle* h = nullptr;
    CHECK(ilqr_create(&h, 0, 12, 4, 10, 8) == ILQR_ERR_HIP && !h, "create without a GPU");
    ilqr_multi* m = nullptr;
    int devs[2] = {0, 1};
    CHECK(ilqr_multi_create(&m, devs, 2, 12, 4, 10, 8) == ILQR_ERR_HIP && !m, "multi create without a GPU");
    ilqr_floating fm = floating_model();
    ilqr_floating_handle* fh = nullptr;
    CHECK(ilqr_floating_create(&fh, 0, &fm, 10, 2) == ILQR_ERR_HIP && !fh, "floating create without a GPU");
    std::printf("no GPU visible: GPU paths skipped, create paths fail with ILQR_ERR_HIP (%d failed checks)\n", fails);
  }
  std::printf("abi sanitizer driver: %s\n", fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}
