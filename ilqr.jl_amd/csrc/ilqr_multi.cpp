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
#include <utility>
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
  // fit history scratch (max_iter, nb) per shard, grown on demand (ilqr_multi_fit_resident)
  double *hcost = nullptr, *halpha = nullptr, *hdu2 = nullptr;
  int32_t* htrials = nullptr;
  int hcap = 0;  // iterations the scratch holds
  hipStream_t stream = nullptr;
};

}  // namespace

struct ilqr_multi {
  int nx = 0, nu = 0, T = 0, batch = 0;
  std::vector<Shard> shards;
  int32_t kind = 0;        // problem set by ilqr_multi_set_problem (0: none yet)
  bool loaded = false;     // trajectories loaded (ilqr_multi_load) or left by a fit
  bool have_result = false;
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
  for (double* p : {s.A, s.B, s.Q, s.R, s.Qf, s.x, s.u, s.xt, s.xo, s.uo, s.cost, s.hcost, s.halpha, s.hdu2})
    (void)hipFree(p);
  (void)hipFree(s.iters);
  (void)hipFree(s.status);
  (void)hipFree(s.htrials);
  if (s.stream) (void)hipStreamDestroy(s.stream);
  s = Shard{};
}

ilqr_status hip_status(hipError_t e) { return e == hipSuccess ? ILQR_OK : ILQR_ERR_HIP; }

// the problem descriptor of a shard: its resident per-instance LQ data; the 2-link arm
// has none
ilqr_problem shard_problem(int32_t kind, const Shard& s) {
  if (kind == ILQR_PROBLEM_LQ) return ilqr_problem{kind, 0, s.A, s.B, s.Q, s.R, s.Qf};
  return ilqr_problem{kind, 0, nullptr, nullptr, nullptr, nullptr, nullptr};
}

// Per-device steps of the multi-device calls (each runs on the shard's thread, on the
// shard's stream). Host arrays hold the whole batch; shard i's block starts at b0.
ilqr_status shard_set_problem(const ilqr_multi* m, Shard& s, const ilqr_problem* p) {
  if (s.nb == 0) return ILQR_OK;
  if (hipSetDevice(s.device) != hipSuccess) return ILQR_ERR_HIP;
  const int nx = m->nx, nu = m->nu;
  const size_t b0 = (size_t)s.b0, nb = (size_t)s.nb;
  auto h2d = [&](double* dst, const double* src, size_t per) {
    return hipMemcpyAsync(dst, src + b0 * per, sizeof(double) * nb * per, hipMemcpyHostToDevice, s.stream);
  };
  hipError_t e = hipSuccess;
  if (p->kind == ILQR_PROBLEM_LQ) {
    if (e == hipSuccess) e = h2d(s.A, p->A, (size_t)nx * nx);
    if (e == hipSuccess) e = h2d(s.B, p->B, (size_t)nx * nu);
    if (e == hipSuccess) e = h2d(s.Q, p->Q, (size_t)nx * nx);
    if (e == hipSuccess) e = h2d(s.R, p->R, (size_t)nu * nu);
    if (e == hipSuccess) e = h2d(s.Qf, p->Qf, (size_t)nx * nx);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
  return hip_status(e);
}

ilqr_status shard_load(const ilqr_multi* m, Shard& s, const double* x, const double* u, const double* x_traj) {
  if (s.nb == 0) return ILQR_OK;
  if (hipSetDevice(s.device) != hipSuccess) return ILQR_ERR_HIP;
  const size_t b0 = (size_t)s.b0, nb = (size_t)s.nb;
  const size_t xs = (size_t)(m->T + 1) * m->nx, us = (size_t)m->T * m->nu;
  auto h2d = [&](double* dst, const double* src, size_t per) {
    return hipMemcpyAsync(dst, src + b0 * per, sizeof(double) * nb * per, hipMemcpyHostToDevice, s.stream);
  };
  hipError_t e = hipSuccess;
  if (x) e = h2d(s.x, x, xs);
  if (e == hipSuccess && u) e = h2d(s.u, u, us);
  if (e == hipSuccess && x_traj) e = h2d(s.xt, x_traj, xs);
  if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
  return hip_status(e);
}

// fit from the shard's resident (x, u) into its resident results (xo, uo, cost, …)
ilqr_status shard_fit(const ilqr_multi* m, Shard& s, const ilqr_options* o, bool use_x_traj,
                      const ilqr_history* hist) {
  if (s.nb == 0) return ILQR_OK;
  if (hipSetDevice(s.device) != hipSuccess) return ILQR_ERR_HIP;
  const ilqr_problem dp = shard_problem(m->kind, s);
  // the history's shard block: its columns b0 .. b0+nb of each (max_iter, batch) array,
  // written through a per-shard (max_iter, nb) device scratch and copied out below
  ilqr_history sh{};
  if (hist) sh = ilqr_history{hist->cost ? s.hcost : nullptr, hist->trials ? s.htrials : nullptr,
                              hist->alpha ? s.halpha : nullptr, hist->du2 ? s.hdu2 : nullptr};
  const ilqr_status st = ilqr_fit_ex(s.h, &dp, o, s.x, s.u, use_x_traj ? s.xt : nullptr, s.xo, s.uo, s.cost,
                                     s.iters, s.status, hist ? &sh : nullptr);
  (void)m;
  return st;
}

ilqr_status shard_gather(const ilqr_multi* m, Shard& s, double* x_out, double* u_out, double* cost,
                         int32_t* iters, int32_t* status) {
  if (s.nb == 0) return ILQR_OK;
  if (hipSetDevice(s.device) != hipSuccess) return ILQR_ERR_HIP;
  const size_t b0 = (size_t)s.b0, nb = (size_t)s.nb;
  const size_t xs = (size_t)(m->T + 1) * m->nx, us = (size_t)m->T * m->nu;
  auto d2h = [&](void* dst, const void* src, size_t bytes) {
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s.stream);
  };
  hipError_t e = hipSuccess;
  if (x_out) e = d2h(x_out + b0 * xs, s.xo, sizeof(double) * nb * xs);
  if (e == hipSuccess && u_out) e = d2h(u_out + b0 * us, s.uo, sizeof(double) * nb * us);
  if (e == hipSuccess && cost) e = d2h(cost + b0, s.cost, sizeof(double) * nb);
  if (e == hipSuccess && iters) e = d2h(iters + b0, s.iters, sizeof(int32_t) * nb);
  if (e == hipSuccess && status) e = d2h(status + b0, s.status, sizeof(int32_t) * nb);
  if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
  return hip_status(e);
}

// run fn(shard) on one host thread per shard; the most severe status
template <class F>
ilqr_status each_shard(ilqr_multi* m, F fn) {
  const int n = (int)m->shards.size();
  std::vector<ilqr_status> res(n, ILQR_OK);
  std::vector<std::thread> th;
  th.reserve(n);
  for (int i = 0; i < n; ++i) th.emplace_back([&, i] { res[i] = fn(m->shards[i]); });
  for (auto& t : th) t.join();
  ilqr_status worst = ILQR_OK;
  for (ilqr_status s : res)
    if (severity(s) > severity(worst)) worst = s;
  return worst;
}

ilqr_status check_problem(const ilqr_multi* m, const ilqr_problem* p) {
  if (!p) return ILQR_ERR_BAD_ARG;
  if (p->kind == ILQR_PROBLEM_LQ && (!p->A || !p->B || !p->Q || !p->R || !p->Qf)) return ILQR_ERR_BAD_ARG;
  if (!ilqr_supported(p->kind, m->nx, m->nu)) return ILQR_ERR_UNSUPPORTED;
  return ILQR_OK;
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

ilqr_status ilqr_multi_set_problem(ilqr_multi* m, const ilqr_problem* host_problem) {
  if (!m) return ILQR_ERR_BAD_ARG;
  ilqr_status st = check_problem(m, host_problem);
  if (st != ILQR_OK) return st;
  st = each_shard(m, [&](Shard& s) { return shard_set_problem(m, s, host_problem); });
  m->kind = st == ILQR_OK ? host_problem->kind : 0;
  return st;
}

ilqr_status ilqr_multi_load(ilqr_multi* m, const double* x, const double* u, const double* x_traj) {
  if (!m || (!x && !u && !x_traj) || (!m->loaded && (!x || !u))) return ILQR_ERR_BAD_ARG;
  const ilqr_status st = each_shard(m, [&](Shard& s) { return shard_load(m, s, x, u, x_traj); });
  if (st == ILQR_OK) m->loaded = true;
  return st;
}

ilqr_status ilqr_multi_fit_resident(ilqr_multi* m, const ilqr_options* o, int flags,
                                    const ilqr_history* history) {
  if (!m || !m->kind || (flags & ~(ILQR_MULTI_WARM_START | ILQR_MULTI_USE_X_TRAJ)) != 0) return ILQR_ERR_BAD_ARG;
  if ((flags & ILQR_MULTI_WARM_START) ? !m->have_result : !m->loaded) return ILQR_ERR_BAD_ARG;
  const ilqr_history* hist = history;
  if (hist && !hist->cost && !hist->trials && !hist->alpha && !hist->du2) hist = nullptr;
  ilqr_options def;
  ilqr_default_options(&def);
  const int max_iter = (o ? o : &def)->max_iter;
  if (hist && max_iter > 0) {  // per-shard history scratch, allocated on first use
    for (Shard& s : m->shards) {
      if (s.nb == 0 || s.hcap >= max_iter) continue;
      if (hipSetDevice(s.device) != hipSuccess) return ILQR_ERR_HIP;
      for (double* q : {s.hcost, s.halpha, s.hdu2}) (void)hipFree(q);
      (void)hipFree(s.htrials);
      s.hcost = s.halpha = s.hdu2 = nullptr;
      s.htrials = nullptr;
      s.hcap = 0;
      const size_t n = (size_t)max_iter * s.nb;
      hipError_t e = hipMalloc(&s.hcost, sizeof(double) * n);
      if (e == hipSuccess) e = hipMalloc(&s.halpha, sizeof(double) * n);
      if (e == hipSuccess) e = hipMalloc(&s.hdu2, sizeof(double) * n);
      if (e == hipSuccess) e = hipMalloc(&s.htrials, sizeof(int32_t) * n);
      if (e != hipSuccess) return ILQR_ERR_HIP;
      s.hcap = max_iter;
    }
  }
  const ilqr_status st = each_shard(m, [&](Shard& s) -> ilqr_status {
    if ((flags & ILQR_MULTI_WARM_START) && s.nb) {  // the previous result is the new start
      std::swap(s.x, s.xo);
      std::swap(s.u, s.uo);
    }
    // The shard's (max_iter, nb) record ↔ columns b0 .. b0+nb of the caller's
    // (max_iter, batch) arrays (device memory of any device: peer copies). The scratch
    // is first loaded with the caller's columns, so rows past the shard's last iteration
    // (the fit's poll stopped the loop) go back as they were (include/ilqr.h).
    auto cp_hist = [&](bool out) -> hipError_t {
      auto cp = [&](void* user, void* scratch, size_t w) {
        char* u = (char*)user + w * s.b0;
        return out ? hipMemcpy2DAsync(u, w * m->batch, scratch, w * s.nb, w * s.nb, max_iter,
                                      hipMemcpyDefault, s.stream)
                   : hipMemcpy2DAsync(scratch, w * s.nb, u, w * m->batch, w * s.nb, max_iter,
                                      hipMemcpyDefault, s.stream);
      };
      hipError_t e = hipSuccess;
      if (hist->cost) e = cp(hist->cost, s.hcost, sizeof(double));
      if (e == hipSuccess && hist->trials) e = cp(hist->trials, s.htrials, sizeof(int32_t));
      if (e == hipSuccess && hist->alpha) e = cp(hist->alpha, s.halpha, sizeof(double));
      if (e == hipSuccess && hist->du2) e = cp(hist->du2, s.hdu2, sizeof(double));
      if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
      return e;
    };
    const bool rec = hist && s.nb && max_iter > 0;
    if (rec) {
      if (hipSetDevice(s.device) != hipSuccess || cp_hist(false) != hipSuccess) return ILQR_ERR_HIP;
    }
    ilqr_status r = shard_fit(m, s, o, (flags & ILQR_MULTI_USE_X_TRAJ) != 0, hist);
    if ((r == ILQR_OK || r == ILQR_ERR_NAN || r == ILQR_ERR_LS_EXHAUSTED) && rec && cp_hist(true) != hipSuccess)
      r = ILQR_ERR_HIP;
    return r;
  });
  m->have_result = severity(st) <= severity(ILQR_ERR_NAN);
  return st;
}

ilqr_status ilqr_multi_gather(ilqr_multi* m, double* x_out, double* u_out, double* cost, int32_t* iters,
                              int32_t* status) {
  if (!m || !m->have_result) return ILQR_ERR_BAD_ARG;
  return each_shard(m, [&](Shard& s) { return shard_gather(m, s, x_out, u_out, cost, iters, status); });
}

ilqr_status ilqr_multi_fit(ilqr_multi* m, const ilqr_problem* p, const ilqr_options* o,
                           const double* x_init, const double* u_init, const double* x_traj,
                           double* x_out, double* u_out, double* cost, int32_t* iters,
                           int32_t* status) {
  if (!m || !p || !x_init || !u_init || !x_out || !u_out) return ILQR_ERR_BAD_ARG;
  ilqr_status st = check_problem(m, p);
  if (st != ILQR_OK) return st;
  // host in, host out: every call moves the problem and the trajectories both ways
  // (the device-resident calls above keep them on the devices)
  st = each_shard(m, [&](Shard& s) -> ilqr_status {
    ilqr_status r = shard_set_problem(m, s, p);
    if (r == ILQR_OK) r = shard_load(m, s, x_init, u_init, x_traj);
    if (r != ILQR_OK) return r;
    const ilqr_problem dp = shard_problem(p->kind, s);
    if (s.nb == 0) return ILQR_OK;
    r = ilqr_fit(s.h, &dp, o, s.x, s.u, x_traj ? s.xt : nullptr, s.xo, s.uo, s.cost, s.iters, s.status);
    if (r != ILQR_OK && r != ILQR_ERR_NAN && r != ILQR_ERR_LS_EXHAUSTED) return r;
    const ilqr_status g = shard_gather(m, s, x_out, u_out, cost, iters, status);
    return g != ILQR_OK ? g : r;
  });
  m->kind = severity(st) <= severity(ILQR_ERR_NAN) ? p->kind : 0;
  m->loaded = m->have_result = m->kind != 0;
  return st;
}

int ilqr_multi_devices(const ilqr_multi* m) { return m ? (int)m->shards.size() : 0; }

ilqr_status ilqr_host_alloc(size_t bytes, void** ptr) {
  if (!ptr) return ILQR_ERR_BAD_ARG;
  *ptr = nullptr;
  return hip_status(hipHostMalloc(ptr, bytes > 0 ? bytes : 1, hipHostMallocDefault));
}

ilqr_status ilqr_host_free(void* ptr) { return ptr ? hip_status(hipHostFree(ptr)) : ILQR_OK; }

}  // extern "C"
