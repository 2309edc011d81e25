// Multi-GPU fit in one process (the `ilqr_fit_multi` of §8b): the
// batch is split into contiguous per-device blocks, every device gets its own
// ilqr_handle and device-resident shard buffers (allocated once at create), and one
// host thread per device runs H2D copy → ilqr_fit → D2H concurrently. Trajectories
// are independent, so there is no device-to-device traffic in the solve; host
// inputs and outputs hold the whole batch. (The one-process-per-GPU path with the
// RCCL all-gather of costs is ilqr_amd.dist + bench.py.)
#include <hip/hip_runtime.h>

#include <string>
#include <thread>
#include <vector>

#include "../../include/ilqr.h"

namespace {

struct Shard {
  int device = 0;
  int b0 = 0, nb = 0;  // global trajectory range [b0, b0 + nb)
  ilqr_handle* h = nullptr;
  double *A = nullptr, *B = nullptr, *Q = nullptr, *R = nullptr, *Qf = nullptr;
  double *x = nullptr, *u = nullptr, *xt = nullptr, *xo = nullptr, *uo = nullptr, *cost = nullptr;
  int32_t *iters = nullptr, *status = nullptr;
  hipStream_t stream = nullptr;
};

}  // namespace

struct ilqr_multi {
  int nx = 0, nu = 0, T = 0, batch = 0;
  std::vector<Shard> shards;
};

namespace {

thread_local std::string g_multi_error;

int severity(ilqr_status s) {  // which status the call reports when shards differ
  switch (s) {
    case ILQR_OK: return 0;
    case ILQR_ERR_LS_EXHAUSTED: return 1;
    case ILQR_ERR_NAN: return 2;
    default: return 3;  // hard errors first
  }
}

void free_shard(Shard& s) {
  if (s.h) ilqr_destroy(s.h);
  (void)hipSetDevice(s.device);
  for (double* p : {s.A, s.B, s.Q, s.R, s.Qf, s.x, s.u, s.xt, s.xo, s.uo, s.cost}) (void)hipFree(p);
  (void)hipFree(s.iters);
  (void)hipFree(s.status);
  if (s.stream) (void)hipStreamDestroy(s.stream);
  s = Shard{};
}

// one device's part of ilqr_multi_fit
ilqr_status run_shard(const ilqr_multi* m, Shard& s, const ilqr_problem* p, const ilqr_options* o,
                      const double* x_init, const double* u_init, const double* x_traj,
                      double* x_out, double* u_out, double* cost, int32_t* iters, int32_t* status) {
  if (s.nb == 0) return ILQR_OK;
  if (hipSetDevice(s.device) != hipSuccess) return ILQR_ERR_HIP;
  const int nx = m->nx, nu = m->nu, T = m->T;
  const size_t b0 = (size_t)s.b0, nb = (size_t)s.nb;
  const size_t xs = (size_t)(T + 1) * nx, us = (size_t)T * nu;
  auto h2d = [&](double* dst, const double* src, size_t per) {
    return hipMemcpyAsync(dst, src + b0 * per, sizeof(double) * nb * per, hipMemcpyHostToDevice, s.stream);
  };
  hipError_t e = hipSuccess;
  ilqr_problem dp = *p;
  if (p->kind == ILQR_PROBLEM_LQ) {
    if (e == hipSuccess) e = h2d(s.A, p->A, (size_t)nx * nx);
    if (e == hipSuccess) e = h2d(s.B, p->B, (size_t)nx * nu);
    if (e == hipSuccess) e = h2d(s.Q, p->Q, (size_t)nx * nx);
    if (e == hipSuccess) e = h2d(s.R, p->R, (size_t)nu * nu);
    if (e == hipSuccess) e = h2d(s.Qf, p->Qf, (size_t)nx * nx);
    dp.A = s.A;
    dp.B = s.B;
    dp.Q = s.Q;
    dp.R = s.R;
    dp.Qf = s.Qf;
  }
  if (e == hipSuccess) e = h2d(s.x, x_init, xs);
  if (e == hipSuccess) e = h2d(s.u, u_init, us);
  if (e == hipSuccess && x_traj) e = h2d(s.xt, x_traj, xs);
  if (e != hipSuccess) return ILQR_ERR_HIP;
  const ilqr_status st = ilqr_fit(s.h, &dp, o, s.x, s.u, x_traj ? s.xt : nullptr, s.xo, s.uo, s.cost,
                                  s.iters, s.status);
  if (st != ILQR_OK && st != ILQR_ERR_NAN && st != ILQR_ERR_LS_EXHAUSTED) return st;
  auto d2h = [&](void* dst, const void* src, size_t bytes) {
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s.stream);
  };
  if (e == hipSuccess) e = d2h(x_out + b0 * xs, s.xo, sizeof(double) * nb * xs);
  if (e == hipSuccess) e = d2h(u_out + b0 * us, s.uo, sizeof(double) * nb * us);
  if (e == hipSuccess && cost) e = d2h(cost + b0, s.cost, sizeof(double) * nb);
  if (e == hipSuccess && iters) e = d2h(iters + b0, s.iters, sizeof(int32_t) * nb);
  if (e == hipSuccess && status) e = d2h(status + b0, s.status, sizeof(int32_t) * nb);
  if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
  return e == hipSuccess ? st : ILQR_ERR_HIP;
}

}  // namespace

extern "C" {

ilqr_status ilqr_multi_create(ilqr_multi** out, const int* devices, int n_devices, int nx, int nu,
                              int T, int batch) {
  if (!out || !devices || n_devices <= 0) return ILQR_ERR_BAD_ARG;
  *out = nullptr;
  if (nx <= 0 || nu <= 0 || T <= 0 || batch <= 0) return ILQR_ERR_BAD_DIMS;
  auto* m = new ilqr_multi;
  m->nx = nx;
  m->nu = nu;
  m->T = T;
  m->batch = batch;
  m->shards.resize(n_devices);
  ilqr_status st = ILQR_OK;
  for (int i = 0; i < n_devices && st == ILQR_OK; ++i) {
    Shard& s = m->shards[i];
    s.device = devices[i];
    s.b0 = (int)((long long)batch * i / n_devices);
    s.nb = (int)((long long)batch * (i + 1) / n_devices) - s.b0;
    if (s.nb == 0) continue;
    if (hipSetDevice(s.device) != hipSuccess) { st = ILQR_ERR_HIP; break; }
    if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) { st = ILQR_ERR_HIP; break; }
    if ((st = ilqr_create(&s.h, s.device, nx, nu, T, s.nb)) != ILQR_OK) break;
    if ((st = ilqr_set_stream(s.h, s.stream)) != ILQR_OK) break;
    const size_t nb = (size_t)s.nb, xs = (size_t)(T + 1) * nx, us = (size_t)T * nu;
    hipError_t e = hipSuccess;
    auto al = [&](auto** q, size_t n) { if (e == hipSuccess) e = hipMalloc(q, sizeof(**q) * n); };
    al(&s.A, nb * nx * nx);
    al(&s.B, nb * nx * nu);
    al(&s.Q, nb * nx * nx);
    al(&s.R, nb * nu * nu);
    al(&s.Qf, nb * nx * nx);
    al(&s.x, nb * xs);
    al(&s.xt, nb * xs);
    al(&s.xo, nb * xs);
    al(&s.u, nb * us);
    al(&s.uo, nb * us);
    al(&s.cost, nb);
    al(&s.iters, nb);
    al(&s.status, nb);
    if (e != hipSuccess) st = ILQR_ERR_HIP;
  }
  if (st != ILQR_OK) {
    g_multi_error = "ilqr_multi_create failed on a device";
    for (Shard& s : m->shards) free_shard(s);
    delete m;
    return st;
  }
  *out = m;
  return ILQR_OK;
}

ilqr_status ilqr_multi_destroy(ilqr_multi* m) {
  if (!m) return ILQR_OK;
  for (Shard& s : m->shards) free_shard(s);
  delete m;
  return ILQR_OK;
}

ilqr_status ilqr_multi_set_schedule(ilqr_multi* m, int flags) {
  if (!m) return ILQR_ERR_BAD_ARG;
  for (Shard& s : m->shards)
    if (s.h) {
      const ilqr_status st = ilqr_set_schedule(s.h, flags);
      if (st != ILQR_OK) return st;
    }
  return ILQR_OK;
}

ilqr_status ilqr_multi_fit(ilqr_multi* m, const ilqr_problem* p, const ilqr_options* o,
                           const double* x_init, const double* u_init, const double* x_traj,
                           double* x_out, double* u_out, double* cost, int32_t* iters,
                           int32_t* status) {
  if (!m || !p || !x_init || !u_init || !x_out || !u_out) return ILQR_ERR_BAD_ARG;
  if (p->kind == ILQR_PROBLEM_LQ && (!p->A || !p->B || !p->Q || !p->R || !p->Qf)) return ILQR_ERR_BAD_ARG;
  if (!ilqr_supported(p->kind, m->nx, m->nu)) return ILQR_ERR_UNSUPPORTED;
  const int n = (int)m->shards.size();
  std::vector<ilqr_status> res(n, ILQR_OK);
  std::vector<std::thread> th;
  th.reserve(n);
  for (int i = 0; i < n; ++i)
    th.emplace_back([&, i] {
      res[i] = run_shard(m, m->shards[i], p, o, x_init, u_init, x_traj, x_out, u_out, cost, iters, status);
    });
  for (auto& t : th) t.join();
  ilqr_status worst = ILQR_OK;
  for (ilqr_status s : res)
    if (severity(s) > severity(worst)) worst = s;
  return worst;
}

int ilqr_multi_devices(const ilqr_multi* m) { return m ? (int)m->shards.size() : 0; }

}  // extern "C"
