// C ABI of libilqr_hip.so (include/ilqr.h): handle/workspace management, argument
// validation with the reference's error behaviour mapped to status codes, and the
// fit driver (src/forward_pass.jl:148-179) on top of the fused iteration kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "../../include/ilqr.h"
#include "ilqr_internal.h"

constexpr int BW4_MIN_BATCH = 2048;  // default backward kernel switch (see bw_wave)

struct ilqr_handle {
  int device = 0;
  int nx = 0, nu = 0, T = 0, batch = 0;
  hipStream_t stream = nullptr;
  // workspace (fit): ping-pong trajectories, gains, per-trajectory state
  double* xbuf[2] = {nullptr, nullptr};
  double* ubuf[2] = {nullptr, nullptr};
  double* K = nullptr;
  double* d = nullptr;
  double* prev_cost = nullptr;
  double* du2 = nullptr;
  int32_t* trials = nullptr;
  int32_t* status = nullptr;
  int32_t* res_parity = nullptr;
  int32_t* iters = nullptr;
  int32_t* host_status = nullptr;  // pinned host copy of a status array (fold_status)
  // fit's convergence poll: running-trajectory counts of the last two iterations,
  // written by the device into host-mapped memory, each behind an event
  // [2] = fit's call-status flags (gather_kernel: bit 0 NaN, bit 1 exhausted line search)
  int32_t* host_running = nullptr;
  int32_t* dev_running = nullptr;  // device alias of host_running
  int32_t* dev_flags = nullptr;    // gather_kernel's device call-status word
  hipEvent_t ev_poll[2] = {nullptr, nullptr};
  ilqr::HostWait host_wait;        // the end-of-fit wait (wait_host_seq)
  ilqr::HostWait poll_wait;        // the per-iteration convergence polls (wait_event)
  // LQ problems of another shape (nx ≤ 12, nu ≤ 4) run zero-padded on an inner
  // (12, 4) handle (created on the first such call): zero rows/columns of A, B, Q, R,
  // Qf, x, u decouple exactly, so the real entries are the (12, 4) kernels' bits.
  ilqr_handle* pad = nullptr;
  double *pA = nullptr, *pB = nullptr, *pQ = nullptr, *pR = nullptr, *pQf = nullptr;
  double *px = nullptr, *pu = nullptr, *pxt = nullptr, *pxn = nullptr, *pun = nullptr;
  double *pd = nullptr, *pK = nullptr;
  // 2-link arm: per-step linearisation workspace J = [A|B] (T × 24 × batch)
  double* J = nullptr;
  // pipelining: the batch is split into `nchunks` chunks; chunk i's forward pass
  // runs on `side` while chunk i+1's backward runs on `stream`
  hipStream_t side = nullptr;
  int nchunks = 1;
  // LQ family schedule (ilqr_set_schedule): fit through the pipelined kernel (forward
  // of half the workgroups overlapping the backward of the other half), and the
  // forward of sequential iterations through the LDS-ring kernel
  bool pipelined = false;
  bool fw_ring = true;
  bool fw_mfma = false;  // ILQR_SCHED_FORWARD_MFMA: the ring forward on the 4-block f64 MFMA
  // backward + forward of an iteration in one launch (ILQR_SCHED_FUSED, default on),
  // with the four-trajectories-per-wave backward and the ring forward only: 166 → 159 µs
  // per headline iteration (no kernel boundary)
  bool fused = true;
  // backward kernel of the LQ family: ILQR_SCHED_BACKWARD_WAVE (or PIPELINED) forces
  // one trajectory per wave, ILQR_SCHED_BACKWARD_BLOCK four per wave; by default four
  // per wave from BW4_MIN_BATCH trajectories up (below it there are fewer waves than
  // SIMDs and the shorter per-wave chain of the one-trajectory kernel wins:
  // profiles/r01/bw4_scan.txt)
  bool bw_wave = false;
  // the fused LQ iteration's cooperative line search (ILQR_SCHED_SEQUENTIAL_SEARCH
  // turns it off): per-trajectory records, candidate costs, the publication list and
  // its counters (zeroed here, re-armed by every launch's last wave)
  bool coop = true;
  ilqr::LSCoopRec* coop_rec = nullptr;
  double* coop_cost = nullptr;
  double* coop_du2 = nullptr;
  uint64_t* coop_list = nullptr;
  int32_t* coop_ctl = nullptr;
  uint32_t coop_gen = 0;  // fused launches so far (the list's generation tag)
  uint32_t fit_seq = 0;   // fits so far (tags the host call-status word, wait_fit)
  double* coop_sx = nullptr;  // the search's scratch rollouts (LSCoop::sx / su)
  double* coop_su = nullptr;
  ilqr::LSCoop* coop_dev = nullptr;  // the struct of the above, in device memory
  int bound[3] = {0, 0, 0};
  hipEvent_t ev_bw[2] = {nullptr, nullptr};
  hipEvent_t ev_fw[2] = {nullptr, nullptr};
};

namespace {

thread_local std::string g_last_error;

ilqr_status hip_fail(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return ILQR_ERR_HIP;
}

#define HIP_TRY(expr)                                  \
  do {                                                 \
    hipError_t e_ = (expr);                            \
    if (e_ != hipSuccess) return hip_fail(e_, #expr);  \
  } while (0)

ilqr::LQParams lq_params(const ilqr_problem* p) {
  return ilqr::LQParams{p->A, p->B, p->Q, p->R, p->Qf};
}

constexpr int PAD_NX = 12, PAD_NU = 4;  // the compiled LQ shape padded problems run at

bool lq_paddable(int nx, int nu) {
  return !ilqr::lq_supported(nx, nu) && nx <= PAD_NX && nu <= PAD_NU &&
         ilqr::lq_supported(PAD_NX, PAD_NU);
}

ilqr_status check_problem(const ilqr_handle* h, const ilqr_problem* p) {
  if (!h || !p) return ILQR_ERR_BAD_ARG;
  if (p->kind == ILQR_PROBLEM_LQ) {
    if (!p->A || !p->B || !p->Q || !p->R || !p->Qf) return ILQR_ERR_BAD_ARG;
    if (!ilqr::lq_supported(h->nx, h->nu) && !lq_paddable(h->nx, h->nu)) return ILQR_ERR_UNSUPPORTED;
    return ILQR_OK;
  }
  if (p->kind == ILQR_PROBLEM_TWO_LINK) {
    // the arm is fully defined by the reference script: no per-instance data
    if (p->A || p->B || p->Q || p->R || p->Qf) return ILQR_ERR_BAD_ARG;
    if (!ilqr::tl_supported(h->nx, h->nu) || !h->J) return ILQR_ERR_UNSUPPORTED;
    return ILQR_OK;
  }
  return ILQR_ERR_UNSUPPORTED;
}

bool two_link(const ilqr_problem* p) { return p->kind == ILQR_PROBLEM_TWO_LINK; }

bool padded(const ilqr_handle* h, const ilqr_problem* p) {
  return p->kind == ILQR_PROBLEM_LQ && lq_paddable(h->nx, h->nu);
}

ilqr::LSParams ls_params(const ilqr_options* o) {
  ilqr_options def;
  ilqr_default_options(&def);
  if (!o) o = &def;
  return ilqr::LSParams{o->mu, o->alpha0, o->shrink, o->tol, o->max_trials};
}

ilqr_status join(ilqr_handle* h, const ilqr_problem* p);

// the LQ iteration runs as one lq_iter_fused4 launch (enqueue_iteration)
bool fused_path(const ilqr_handle* h, const ilqr_problem* p) {
  return !two_link(p) && h->nchunks == 1 && h->fused && !h->bw_wave && h->fw_ring && h->nx == 12 &&
         h->nu == 4;
}

// Enqueue one fit iteration for the whole batch: backward(c) on the handle's
// stream, forward(c) on the side stream after it. With `chain`, backward(c) first
// waits for the previous iteration's forward(c) (same trajectories); otherwise the
// call ends by making the handle's stream wait for every forward (join).
ilqr_status enqueue_iteration(ilqr_handle* h, const ilqr_problem* p, const ilqr::IterArgs& a,
                              const ilqr::LSParams& ls, bool chain, const ilqr_history* hist = nullptr) {
  if (two_link(p)) {  // one stream: linearise, backward, forward
    HIP_TRY(ilqr::launch_tl_iteration(ilqr::two_link_params(), h->nu, h->batch, h->T, a, h->J, ls,
                                      h->stream));
    return ILQR_OK;
  }
  const ilqr::LQParams P = lq_params(p);
  if (h->nchunks == 1) {  // one stream, no cross-stream events (each hand-off costs ~10 µs)
    if (fused_path(h, p)) {
      ilqr::IterArgs ac = a;
      // only a launch that gets the list also re-arms it (ctl[(gen + 1) & 1] = 0): a
      // sequential-search launch between two cooperative ones must not advance the
      // generation, or the next cooperative launch would count in a half nobody zeroed
      // Against prev_cost = +Inf (a cold iteration, fit's first) trial 1 accepts every
      // finite cost (forward_pass.jl:77-80): nothing would be published, so the launch
      // runs the sequential search (the same bits) without the search's exit test.
      const bool coop = h->coop && a.prev_cost && !a.init;
      ac.coop = coop ? h->coop_dev : nullptr;
      ac.coop_ctl = coop ? h->coop_ctl : nullptr;
      ac.coop_gen = coop ? ++h->coop_gen : h->coop_gen;
      HIP_TRY(ilqr::launch_lq_iter_fused4(P, h->batch, h->T, ac, ls, h->stream, h->fw_mfma));
      return ILQR_OK;
    }
    HIP_TRY(ilqr::launch_lq_iter_backward(h->nx, h->nu, P, 0, h->batch, h->T, a, ls.mu, h->stream, h->bw_wave));
    HIP_TRY(ilqr::launch_lq_iter_forward(h->nx, h->nu, P, 0, h->batch, h->T, a, ls, h->stream, h->fw_ring,
                                         h->fw_mfma));
    return ILQR_OK;
  }
  for (int c = 0; c < h->nchunks; ++c) {
    const int b0 = h->bound[c], b1 = h->bound[c + 1];
    if (chain) HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_fw[c], 0));
    HIP_TRY(ilqr::launch_lq_iter_backward(h->nx, h->nu, P, b0, b1, h->T, a, ls.mu, h->stream, h->bw_wave));
    HIP_TRY(hipEventRecord(h->ev_bw[c], h->stream));
    HIP_TRY(hipStreamWaitEvent(h->side, h->ev_bw[c], 0));
    HIP_TRY(ilqr::launch_lq_iter_forward(h->nx, h->nu, P, b0, b1, h->T, a, ls, h->side));
    if (hist)  // chunk c's record before ev_fw[c]: its next backward (it may set NAN) waits
               // for this chunk's record only, and still overlaps the next chunk's forward
      HIP_TRY(ilqr::launch_record_history(
          b1 - b0, a.iter, a.status + b0, a.iters + b0, a.trials + b0, a.new_cost + b0, a.du2 + b0, false,
          ls.alpha0, ls.shrink, hist->cost ? hist->cost + b0 : nullptr, hist->trials ? hist->trials + b0 : nullptr,
          hist->alpha ? hist->alpha + b0 : nullptr, hist->du2 ? hist->du2 + b0 : nullptr, h->side, h->batch));
    HIP_TRY(hipEventRecord(h->ev_fw[c], h->side));
  }
  if (!chain) return join(h, p);
  return ILQR_OK;
}

ilqr_status join(ilqr_handle* h, const ilqr_problem* p) {
  if (two_link(p) || h->nchunks == 1) return ILQR_OK;
  for (int c = 0; c < h->nchunks; ++c) HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_fw[c], 0));
  return ILQR_OK;
}

ilqr_status check_options(const ilqr_options* o) {
  if (!o) return ILQR_OK;
  if (o->max_trials < 1 || o->max_iter < 0) return ILQR_ERR_BAD_ARG;
  if (!(o->shrink > 0.0 && o->shrink < 1.0) || !(o->alpha0 > 0.0) || std::isnan(o->mu))
    return ILQR_ERR_BAD_ARG;
  return ILQR_OK;
}

// Reduce per-trajectory status to the call status (host copy, synchronising).
ilqr_status fold_status(ilqr_handle* h, const int32_t* dev_status) {
  int32_t* st = h->host_status;  // pinned: one DMA, no staging copy
  HIP_TRY(hipMemcpyAsync(st, dev_status, sizeof(int32_t) * h->batch, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  bool nan = false, ls = false;
  for (int b = 0; b < h->batch; ++b) {
    nan |= st[b] == ILQR_TRAJ_NAN;
    ls |= st[b] == ILQR_TRAJ_LS_EXHAUSTED;
  }
  return nan ? ILQR_ERR_NAN : (ls ? ILQR_ERR_LS_EXHAUSTED : ILQR_OK);
}

// Inner (12, 4) handle and padded scratch, created on the first padded call (the
// only allocation outside ilqr_create); stream and schedule follow the outer handle.
ilqr_status ensure_pad(ilqr_handle* h) {
  if (!h->pad) {
    ilqr_handle* in = nullptr;
    const ilqr_status st = ilqr_create(&in, h->device, PAD_NX, PAD_NU, h->T, h->batch);
    if (st != ILQR_OK) return st;
    h->pad = in;
    const size_t B = (size_t)h->batch, T = (size_t)h->T;
    hipError_t e = hipSuccess;
    auto al = [&](double** q, size_t n) { if (e == hipSuccess) e = hipMalloc(q, sizeof(double) * n); };
    al(&h->pA, B * PAD_NX * PAD_NX);
    al(&h->pB, B * PAD_NX * PAD_NU);
    al(&h->pQ, B * PAD_NX * PAD_NX);
    al(&h->pR, B * PAD_NU * PAD_NU);
    al(&h->pQf, B * PAD_NX * PAD_NX);
    al(&h->px, B * (T + 1) * PAD_NX);
    al(&h->pxt, B * (T + 1) * PAD_NX);
    al(&h->pxn, B * (T + 1) * PAD_NX);
    al(&h->pu, B * T * PAD_NU);
    al(&h->pun, B * T * PAD_NU);
    al(&h->pd, B * T * PAD_NU);
    al(&h->pK, B * T * PAD_NU * PAD_NX);
    if (e != hipSuccess) return hip_fail(e, "ilqr: padded workspace");
  }
  h->pad->stream = h->stream;
  h->pad->pipelined = h->pipelined;
  h->pad->fused = h->fused;
  h->pad->fw_ring = h->fw_ring;
  h->pad->fw_mfma = h->fw_mfma;
  h->pad->bw_wave = h->bw_wave;
  h->pad->coop = h->coop;
  return ILQR_OK;
}

// (N, R, C) → (N, R2, C2) zero-padded, and back
ilqr_status pad3(ilqr_handle* h, const double* src, double* dst, size_t N, int R, int C, int R2, int C2) {
  HIP_TRY(ilqr::launch_pad3(src, dst, N, R, C, R2, C2, h->stream));
  return ILQR_OK;
}
ilqr_status unpad3(ilqr_handle* h, const double* src, double* dst, size_t N, int R, int C, int R2, int C2) {
  HIP_TRY(ilqr::launch_unpad3(src, dst, N, R, C, R2, C2, h->stream));
  return ILQR_OK;
}

#define ILQR_TRY(expr)                    \
  do {                                    \
    const ilqr_status s_ = (expr);        \
    if (s_ != ILQR_OK) return s_;         \
  } while (0)

// pad the LQ problem data into the scratch and describe it
ilqr_status pad_problem(ilqr_handle* h, const ilqr_problem* p, ilqr_problem* pp) {
  const size_t B = (size_t)h->batch;
  const int n = h->nx, m = h->nu;
  ILQR_TRY(pad3(h, p->A, h->pA, B, n, n, PAD_NX, PAD_NX));
  ILQR_TRY(pad3(h, p->B, h->pB, B, n, m, PAD_NX, PAD_NU));
  ILQR_TRY(pad3(h, p->Q, h->pQ, B, n, n, PAD_NX, PAD_NX));
  ILQR_TRY(pad3(h, p->R, h->pR, B, m, m, PAD_NU, PAD_NU));
  ILQR_TRY(pad3(h, p->Qf, h->pQf, B, n, n, PAD_NX, PAD_NX));
  *pp = *p;
  pp->A = h->pA;
  pp->B = h->pB;
  pp->Q = h->pQ;
  pp->R = h->pR;
  pp->Qf = h->pQf;
  return ILQR_OK;
}
// trajectories: x-like (B, T+1, nx), u-like (B, T, nu), gains K (B·T, nu, nx)
ilqr_status pad_x(ilqr_handle* h, const double* x, double* px) {
  return pad3(h, x, px, (size_t)h->batch, h->T + 1, h->nx, h->T + 1, PAD_NX);
}
ilqr_status pad_u(ilqr_handle* h, const double* u, double* pu) {
  return pad3(h, u, pu, (size_t)h->batch, h->T, h->nu, h->T, PAD_NU);
}
ilqr_status unpad_x(ilqr_handle* h, const double* px, double* x) {
  return unpad3(h, px, x, (size_t)h->batch, h->T + 1, h->nx, h->T + 1, PAD_NX);
}
ilqr_status unpad_u(ilqr_handle* h, const double* pu, double* u) {
  return unpad3(h, pu, u, (size_t)h->batch, h->T, h->nu, h->T, PAD_NU);
}

// The end of a fit: the stream's last kernel stores this fit's number into a wait word
// (ilqr::wait_host_seq below).
// `units`: the fit iterations enqueued since the host last waited on this fit.
hipError_t wait_fit(ilqr_handle* h, uint32_t seq, int units, hipStream_t s) {
  return ilqr::wait_host_seq(h->host_running + 2, seq, units, s, &h->host_wait);
}

}  // namespace

// The stream's last kernel of a fit (gather_flags_kernel) stores the fit's number into
// the host-mapped call-status word as it runs, after every earlier kernel of the stream
// completed (in-order stream): when the word carries the number, the outputs are written.
// The host waits on that word by ilqr_wait.h's policy (spin around the expected end, nap
// only through the bulk of a wait expected to exceed 1 ms, sized per iteration). A
// headline-size fit (≈450 µs) never naps; a long one (a config-5 default fit, 2-9 ms; the
// floating family's fits; every shard thread of ilqr_multi) holds no core. The fit
// drivers' per-iteration convergence polls wait the same way on their events (wait_event;
// the next iteration is already queued). hipEventSynchronize busy-waits on this ROCm
// whatever the event's flags (profiles/r05/event_wait_probe_r05.log), so no runtime sync
// is left on these paths. ILQR_FIT_WAIT=sync in the environment forces the stream sync (A/B).
hipError_t ilqr::wait_host_seq(const volatile int32_t* w, uint32_t seq, int units, hipStream_t s,
                               HostWait* hw) {
  static const bool spin = [] {
    const char* e = getenv("ILQR_FIT_WAIT");
    return !(e && strcmp(e, "sync") == 0);
  }();
  if (!spin) return hipStreamSynchronize(s);
  auto done = [&] { return ((uint32_t)__atomic_load_n(w, __ATOMIC_ACQUIRE) >> 2) == seq; };
  hipError_t e = nap_spin_wait(hw, units, hipSuccess, hipErrorNotReady, done, [&] {
    const hipError_t q = hipStreamQuery(s);  // idle, busy (NotReady) or an execution error
    return q == hipSuccess && !done() ? hipErrorLaunchFailure : q;  // idle without the word: lost
  });
  return e != hipSuccess ? e : hipPeekAtLastError();  // a launch error of this thread
}

hipError_t ilqr::wait_event(hipEvent_t ev, HostWait* hw) {
  hipError_t q = hipErrorNotReady;
  auto done = [&] { return (q = hipEventQuery(ev)) != hipErrorNotReady; };
  const hipError_t e = nap_spin_wait(hw, 1, hipSuccess, hipErrorNotReady, done, [&] { return q = hipEventQuery(ev); });
  return e != hipSuccess ? e : q;
}

extern "C" {

int ilqr_abi_version(void) { return ILQR_ABI_VERSION; }

const char* ilqr_status_string(ilqr_status s) {
  switch (s) {
    case ILQR_OK: return "ok";
    case ILQR_ERR_BAD_DIMS: return "bad dimensions (size(x,1) must equal size(u,1)+1)";
    case ILQR_ERR_BAD_ARG: return "bad argument";
    case ILQR_ERR_UNSUPPORTED: return "unsupported problem kind or (nx, nu)";
    case ILQR_ERR_HIP: return "HIP runtime error";
    case ILQR_ERR_NAN: return "NaN in a trajectory";
    case ILQR_ERR_LS_EXHAUSTED: return "line search exhausted";
  }
  return "unknown status";
}

const char* ilqr_last_error(void) { return g_last_error.c_str(); }

void ilqr_default_options(ilqr_options* o) {
  if (!o) return;
  o->max_iter = 100;     // forward_pass.jl:152
  o->max_trials = 64;    // reference is unbounded (forward_pass.jl:70); 0.5^63 ≈ 1e-19
  o->tol = 1e-6;         // forward_pass.jl:152
  o->mu = 0.01;          // backward_pass.jl:214
  o->alpha0 = 1.0;       // forward_pass.jl:66
  o->shrink = 0.5;       // forward_pass.jl:82
}

int ilqr_supported(int32_t kind, int nx, int nu) {
  if (kind == ILQR_PROBLEM_LQ) return (ilqr::lq_supported(nx, nu) || lq_paddable(nx, nu)) ? 1 : 0;
  if (kind == ILQR_PROBLEM_TWO_LINK) return ilqr::tl_supported(nx, nu) ? 1 : 0;
  if (kind == ILQR_PROBLEM_TILES) return ilqr::tiles_supported(nx, nu) ? 1 : 0;
  if (kind == ILQR_PROBLEM_CHAIN) return (nx % 2 == 0) ? ilqr_chain_supported(nx / 2, nu) : 0;
  return 0;
}

ilqr_status ilqr_create(ilqr_handle** out, int device, int nx, int nu, int T, int batch) {
  if (!out) return ILQR_ERR_BAD_ARG;
  *out = nullptr;
  if (nx <= 0 || nu <= 0 || T <= 0 || batch <= 0) return ILQR_ERR_BAD_DIMS;
  HIP_TRY(hipSetDevice(device));
  auto* h = new ilqr_handle;
  h->device = device;
  h->nx = nx;
  h->nu = nu;
  h->T = T;
  h->batch = batch;
  h->bw_wave = batch < BW4_MIN_BATCH;
  const size_t B = (size_t)batch;
  hipError_t e = hipSuccess;
  for (int i = 0; i < 2 && e == hipSuccess; ++i) {
    e = hipMalloc(&h->xbuf[i], sizeof(double) * B * (T + 1) * nx);
    if (e == hipSuccess) e = hipMalloc(&h->ubuf[i], sizeof(double) * B * T * nu);
  }
  if (e == hipSuccess) e = hipMalloc(&h->K, sizeof(double) * B * T * nu * nx);
  if (e == hipSuccess) e = hipMalloc(&h->d, sizeof(double) * B * T * nu);
  if (e == hipSuccess) e = hipMalloc(&h->prev_cost, sizeof(double) * B);
  if (e == hipSuccess) e = hipMalloc(&h->du2, sizeof(double) * B);
  if (e == hipSuccess) e = hipMalloc(&h->trials, sizeof(int32_t) * B);
  if (e == hipSuccess) e = hipMalloc(&h->status, sizeof(int32_t) * B);
  if (e == hipSuccess) e = hipMalloc(&h->res_parity, sizeof(int32_t) * B);
  if (e == hipSuccess) e = hipMalloc(&h->iters, sizeof(int32_t) * B);
  if (e == hipSuccess) e = hipHostMalloc(&h->host_status, sizeof(int32_t) * B, hipHostMallocDefault);
  if (e == hipSuccess)
    e = hipHostMalloc(&h->host_running, sizeof(int32_t) * 4, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&h->dev_running, h->host_running, 0);
  if (e == hipSuccess) e = hipMalloc(&h->dev_flags, sizeof(int32_t) * 2);
  if (e == hipSuccess) e = hipMemset(h->dev_flags, 0, sizeof(int32_t) * 2);
  for (int c = 0; c < 2 && e == hipSuccess; ++c) e = hipEventCreateWithFlags(&h->ev_poll[c], hipEventDisableTiming);
  if (e == hipSuccess && nx == 12 && nu == 4) {
    e = hipMalloc(&h->coop_rec, sizeof(ilqr::LSCoopRec) * B);
    if (e == hipSuccess) e = hipMalloc(&h->coop_cost, sizeof(double) * B * ilqr::COOP_MAX_TRIALS);
    if (e == hipSuccess) e = hipMalloc(&h->coop_du2, sizeof(double) * B * ilqr::COOP_MAX_TRIALS);
    if (e == hipSuccess) e = hipMalloc(&h->coop_list, sizeof(uint64_t) * B);
    if (e == hipSuccess) e = hipMalloc(&h->coop_ctl, sizeof(int32_t) * 2);
    if (e == hipSuccess) e = hipMemset(h->coop_list, 0, sizeof(uint64_t) * B);  // generation 0: stale
    if (e == hipSuccess) e = hipMemset(h->coop_ctl, 0, sizeof(int32_t) * 2);
    if (e == hipSuccess) e = hipMalloc(&h->coop_dev, sizeof(ilqr::LSCoop));
    // scratch rollouts for the first searches of a launch (32-bit buffer offsets: the
    // x part must stay under 2 GiB, else no scratch)
    const int nsl = std::min(batch, ilqr::COOP_SCRATCH_SLOTS);
    const size_t sxb = sizeof(double) * nsl * ilqr::COOP_MAX_TRIALS * (size_t)(T + 1) * nx;
    const size_t sub = sizeof(double) * nsl * ilqr::COOP_MAX_TRIALS * (size_t)T * nu;
    bool scratch = sxb < (size_t(1) << 31);
    // the scratch (≈260 MB at T = 1000) is a speed-up, not a need: without it the search
    // rolls the final trial out again (nslots = 0), so a failed allocation is not an error
    if (e == hipSuccess && scratch && hipMalloc(&h->coop_sx, sxb) != hipSuccess) scratch = false;
    if (e == hipSuccess && scratch && hipMalloc(&h->coop_su, sub) != hipSuccess) scratch = false;
    if (!scratch) {
      (void)hipGetLastError();  // clear the failed allocation's error
      (void)hipFree(h->coop_sx);
      (void)hipFree(h->coop_su);
      h->coop_sx = nullptr;
      h->coop_su = nullptr;
    }
    if (e == hipSuccess) {
      const ilqr::LSCoop c{h->coop_rec, h->coop_cost, h->coop_du2, h->coop_list, h->coop_ctl,
                           h->coop_sx,  h->coop_su,   scratch ? nsl : 0};
      e = hipMemcpy(h->coop_dev, &c, sizeof(c), hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
  }
  if (e == hipSuccess && ilqr::tl_supported(nx, nu))
    e = hipMalloc(&h->J, sizeof(double) * ilqr::tl_workspace_doubles(batch, T));
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking);
  for (int c = 0; c < 2 && e == hipSuccess; ++c) {
    e = hipEventCreateWithFlags(&h->ev_bw[c], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_fw[c], hipEventDisableTiming);
  }
  if (e == hipSuccess) {
    // Two chunks (chunk c's forward on the side stream overlapping chunk c+1's
    // backward) only when each chunk still fills every SIMD with 4 backward waves:
    // measured at B = 4096 on MI355X, halves at 2 waves/SIMD run 14 % slower and
    // the cross-stream hand-offs cost ~10 µs each, a net loss.
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    const int full_gen = 4 * 4 * (cus > 0 ? cus : 256);
    h->nchunks = batch >= 2 * full_gen ? 2 : 1;
    h->bound[0] = 0;
    h->bound[h->nchunks] = batch;
    if (h->nchunks == 2) h->bound[1] = batch / 2;
  }
  if (e != hipSuccess) {
    ilqr_destroy(h);
    return hip_fail(e, "ilqr_create: hipMalloc");
  }
  *out = h;
  return ILQR_OK;
}

ilqr_status ilqr_destroy(ilqr_handle* h) {
  if (!h) return ILQR_OK;
  (void)hipSetDevice(h->device);
  for (int i = 0; i < 2; ++i) {
    (void)hipFree(h->xbuf[i]);
    (void)hipFree(h->ubuf[i]);
  }
  (void)hipFree(h->K);
  (void)hipFree(h->d);
  (void)hipFree(h->prev_cost);
  (void)hipFree(h->du2);
  (void)hipFree(h->trials);
  (void)hipFree(h->status);
  (void)hipFree(h->res_parity);
  (void)hipFree(h->iters);
  if (h->host_status) (void)hipHostFree(h->host_status);
  if (h->host_running) (void)hipHostFree(h->host_running);
  (void)hipFree(h->dev_flags);
  (void)hipFree(h->coop_rec);
  (void)hipFree(h->coop_cost);
  (void)hipFree(h->coop_du2);
  (void)hipFree(h->coop_list);
  (void)hipFree(h->coop_sx);
  (void)hipFree(h->coop_su);
  (void)hipFree(h->coop_ctl);
  (void)hipFree(h->coop_dev);
  for (int c = 0; c < 2; ++c)
    if (h->ev_poll[c]) (void)hipEventDestroy(h->ev_poll[c]);
  if (h->pad) {
    (void)ilqr_destroy(h->pad);
    for (double* q : {h->pA, h->pB, h->pQ, h->pR, h->pQf, h->px, h->pu, h->pxt, h->pxn, h->pun, h->pd, h->pK})
      (void)hipFree(q);
  }
  (void)hipFree(h->J);
  for (int c = 0; c < 2; ++c) {
    if (h->ev_bw[c]) (void)hipEventDestroy(h->ev_bw[c]);
    if (h->ev_fw[c]) (void)hipEventDestroy(h->ev_fw[c]);
  }
  if (h->side) (void)hipStreamDestroy(h->side);
  delete h;
  return ILQR_OK;
}

ilqr_status ilqr_set_stream(ilqr_handle* h, void* s) {
  if (!h) return ILQR_ERR_BAD_ARG;
  h->stream = (hipStream_t)s;
  return ILQR_OK;
}

ilqr_status ilqr_set_schedule(ilqr_handle* h, int flags) {
  if (!h || (flags & ~(ILQR_SCHED_PIPELINED | ILQR_SCHED_RING_FORWARD | ILQR_SCHED_BACKWARD_WAVE |
                      ILQR_SCHED_BACKWARD_BLOCK | ILQR_SCHED_FUSED | ILQR_SCHED_FORWARD_MFMA |
                      ILQR_SCHED_SEQUENTIAL_SEARCH)) != 0)
    return ILQR_ERR_BAD_ARG;
  // every combination check before any handle state changes
  if ((flags & ILQR_SCHED_FUSED) && (flags & (ILQR_SCHED_BACKWARD_WAVE | ILQR_SCHED_PIPELINED)))
    return ILQR_ERR_BAD_ARG;
  if ((flags & ILQR_SCHED_BACKWARD_BLOCK) && (flags & (ILQR_SCHED_BACKWARD_WAVE | ILQR_SCHED_PIPELINED)))
    return ILQR_ERR_BAD_ARG;
  for (ilqr_handle* t : {h, h->pad}) {
    if (!t) continue;
    t->pipelined = (flags & ILQR_SCHED_PIPELINED) != 0;
    t->fused = (flags & ILQR_SCHED_FUSED) != 0;
    t->fw_ring = (flags & ILQR_SCHED_RING_FORWARD) != 0;
    t->fw_mfma = (flags & ILQR_SCHED_FORWARD_MFMA) != 0;
    t->coop = (flags & ILQR_SCHED_SEQUENTIAL_SEARCH) == 0;
    t->bw_wave = (flags & (ILQR_SCHED_BACKWARD_WAVE | ILQR_SCHED_PIPELINED)) != 0 ||
                 (!(flags & ILQR_SCHED_BACKWARD_BLOCK) && h->batch < BW4_MIN_BATCH);
  }
  return ILQR_OK;
}

ilqr_status ilqr_sync(ilqr_handle* h) {
  if (!h) return ILQR_ERR_BAD_ARG;
  HIP_TRY(hipStreamSynchronize(h->stream));
  return ILQR_OK;
}

ilqr_status ilqr_backward(ilqr_handle* h, const ilqr_problem* p, const ilqr_options* o,
                          const double* x, const double* u, double* d, double* K,
                          int32_t* status) {
  ilqr_status st = check_problem(h, p);
  if (st != ILQR_OK) return st;
  if ((st = check_options(o)) != ILQR_OK) return st;
  if (!x || !u || !d || !K) return ILQR_ERR_BAD_ARG;
  HIP_TRY(hipSetDevice(h->device));
  if (padded(h, p)) {
    ILQR_TRY(ensure_pad(h));
    ilqr_problem pp;
    ILQR_TRY(pad_problem(h, p, &pp));
    ILQR_TRY(pad_x(h, x, h->px));
    ILQR_TRY(pad_u(h, u, h->pu));
    // with a status array the inner call folds it (and synchronises)
    const ilqr_status bst = ilqr_backward(h->pad, &pp, o, h->px, h->pu, h->pd, h->pK, status);
    if (bst != ILQR_OK && bst != ILQR_ERR_NAN) return bst;
    ILQR_TRY(unpad_u(h, h->pd, d));
    ILQR_TRY(unpad3(h, h->pK, K, (size_t)h->batch * h->T, h->nu, h->nx, PAD_NU, PAD_NX));
    if (status) HIP_TRY(hipStreamSynchronize(h->stream));
    return bst;
  }
  if (two_link(p))
    HIP_TRY(ilqr::launch_tl_backward(ilqr::two_link_params(), h->nu, h->batch, h->T, x, u, h->J, d, K,
                                     status, ls_params(o).mu, h->stream));
  else
    HIP_TRY(ilqr::launch_lq_backward(h->nx, h->nu, lq_params(p), h->batch, h->T, x, u, d, K,
                                     status, ls_params(o).mu, h->stream, h->bw_wave));
  return status ? fold_status(h, status) : ILQR_OK;
}

ilqr_status ilqr_backward_tiles(ilqr_handle* h, const ilqr_tiles* tl, const ilqr_options* o,
                                double* d, double* K, int32_t* status) {
  if (!h || !tl) return ILQR_ERR_BAD_ARG;
  ilqr_status st = check_options(o);
  if (st != ILQR_OK) return st;
  if (!ilqr::tiles_supported(h->nx, h->nu)) return ILQR_ERR_UNSUPPORTED;
  if (!tl->A || !tl->B || !tl->lx || !tl->lu || !tl->lxx || !tl->luu || !tl->lfx || !tl->lfxx ||
      !d || !K)
    return ILQR_ERR_BAD_ARG;
  HIP_TRY(hipSetDevice(h->device));
  const ilqr::TileParams P{tl->A, tl->B, tl->lx, tl->lu, tl->lxx, tl->lux, tl->luu, tl->lfx, tl->lfxx};
  HIP_TRY(ilqr::launch_tiles_backward(h->nx, h->nu, P, h->batch, h->T, d, K, status,
                                      ls_params(o).mu, h->stream));
  return status ? fold_status(h, status) : ILQR_OK;
}

ilqr_status ilqr_linearize(ilqr_handle* h, const ilqr_problem* p, const double* x, const double* u,
                           double* A, double* B) {
  const ilqr_status st = check_problem(h, p);
  if (st != ILQR_OK) return st;
  if (!A || !B) return ILQR_ERR_BAD_ARG;
  HIP_TRY(hipSetDevice(h->device));
  if (two_link(p)) {
    if (!x || !u) return ILQR_ERR_BAD_ARG;
    HIP_TRY(ilqr::launch_tl_jacobian(ilqr::two_link_params(), h->nu, h->batch, h->T, x, u, A, B, h->stream));
  } else {  // LQ of any supported or padded shape: the caller's (nx, nu) matrices as given
    HIP_TRY(ilqr::launch_lq_linearize(h->nx, h->nu, lq_params(p), h->batch, h->T, A, B, h->stream));
  }
  return ILQR_OK;
}

ilqr_status ilqr_forward(ilqr_handle* h, const ilqr_problem* p, const ilqr_options* o,
                         const double* x, const double* u, const double* x_traj,
                         const double* d, const double* K, const double* prev_cost,
                         double* x_new, double* u_new, double* new_cost, int32_t* trials,
                         int32_t* status) {
  ilqr_status st = check_problem(h, p);
  if (st != ILQR_OK) return st;
  if ((st = check_options(o)) != ILQR_OK) return st;
  if (!x || !u || !d || !K || !prev_cost || !x_new || !u_new || !new_cost) return ILQR_ERR_BAD_ARG;
  HIP_TRY(hipSetDevice(h->device));
  if (padded(h, p)) {
    ILQR_TRY(ensure_pad(h));
    ilqr_problem pp;
    ILQR_TRY(pad_problem(h, p, &pp));
    ILQR_TRY(pad_x(h, x, h->px));
    ILQR_TRY(pad_u(h, u, h->pu));
    if (x_traj) ILQR_TRY(pad_x(h, x_traj, h->pxt));
    ILQR_TRY(pad_u(h, d, h->pd));
    ILQR_TRY(pad3(h, K, h->pK, (size_t)h->batch * h->T, h->nu, h->nx, PAD_NU, PAD_NX));
    const ilqr_status fst = ilqr_forward(h->pad, &pp, o, h->px, h->pu, x_traj ? h->pxt : nullptr,
                                         h->pd, h->pK, prev_cost, h->pxn, h->pun, new_cost, trials,
                                         status);
    if (fst != ILQR_OK && fst != ILQR_ERR_NAN && fst != ILQR_ERR_LS_EXHAUSTED) return fst;
    ILQR_TRY(unpad_x(h, h->pxn, x_new));
    ILQR_TRY(unpad_u(h, h->pun, u_new));
    if (status) HIP_TRY(hipStreamSynchronize(h->stream));
    return fst;
  }
  if (two_link(p))
    HIP_TRY(ilqr::launch_tl_forward(ilqr::two_link_params(), h->nu, h->batch, h->T, x, u, x_traj, d, K,
                                    prev_cost, x_new, u_new, new_cost, trials, status,
                                    ls_params(o), h->stream));
  else
    HIP_TRY(ilqr::launch_lq_forward(h->nx, h->nu, lq_params(p), h->batch, h->T, x, u, x_traj, d,
                                    K, prev_cost, x_new, u_new, new_cost, trials, status,
                                    ls_params(o), h->stream, h->fw_ring, h->fw_mfma));
  return status ? fold_status(h, status) : ILQR_OK;
}

ilqr_status ilqr_iterate(ilqr_handle* h, const ilqr_problem* p, const ilqr_options* o,
                         const double* x, const double* u, const double* x_traj, double* x_new,
                         double* u_new, const double* prev_cost, double* new_cost, double* du2,
                         int32_t* trials,
                         int32_t* status) {
  ilqr_status st = check_problem(h, p);
  if (st != ILQR_OK) return st;
  if ((st = check_options(o)) != ILQR_OK) return st;
  if (!x || !u || !x_new || !u_new || !new_cost || !status) return ILQR_ERR_BAD_ARG;
  HIP_TRY(hipSetDevice(h->device));
  if (padded(h, p)) {
    ILQR_TRY(ensure_pad(h));
    ilqr_problem pp;
    ILQR_TRY(pad_problem(h, p, &pp));
    ILQR_TRY(pad_x(h, x, h->px));
    ILQR_TRY(pad_u(h, u, h->pu));
    if (x_traj) ILQR_TRY(pad_x(h, x_traj, h->pxt));
    ILQR_TRY(ilqr_iterate(h->pad, &pp, o, h->px, h->pu, x_traj ? h->pxt : nullptr, h->pxn, h->pun,
                          prev_cost, new_cost, du2, trials, status));
    ILQR_TRY(unpad_x(h, h->pxn, x_new));
    return unpad_u(h, h->pun, u_new);
  }
  ilqr::IterArgs a{};
  a.x = x;
  a.u = u;
  a.xtraj = x_traj;
  a.xnew = x_new;
  a.unew = u_new;
  a.K = h->K;
  a.d = h->d;
  a.prev_cost = prev_cost;
  a.new_cost = new_cost;
  a.du2 = du2;
  a.trials = trials;
  a.status = status;
  a.res_parity = nullptr;
  a.iters = nullptr;
  a.parity = 0;
  a.iter = 0;
  return enqueue_iteration(h, p, a, ls_params(o), /*chain=*/false);
}

ilqr_status ilqr_fit(ilqr_handle* h, const ilqr_problem* p, const ilqr_options* o,
                     const double* x_init, const double* u_init, const double* x_traj,
                     double* x_out, double* u_out, double* cost, int32_t* iters,
                     int32_t* status) {
  return ilqr_fit_ex(h, p, o, x_init, u_init, x_traj, x_out, u_out, cost, iters, status, nullptr);
}

ilqr_status ilqr_fit_ex(ilqr_handle* h, const ilqr_problem* p, const ilqr_options* o,
                        const double* x_init, const double* u_init, const double* x_traj,
                        double* x_out, double* u_out, double* cost, int32_t* iters,
                        int32_t* status, const ilqr_history* hist) {
  if (hist && !hist->cost && !hist->trials && !hist->alpha && !hist->du2) hist = nullptr;
  ilqr_status st = check_problem(h, p);
  if (st != ILQR_OK) return st;
  if ((st = check_options(o)) != ILQR_OK) return st;
  if (!x_init || !u_init || !x_out || !u_out) return ILQR_ERR_BAD_ARG;
  ilqr_options def;
  ilqr_default_options(&def);
  if (!o) o = &def;
  HIP_TRY(hipSetDevice(h->device));
  if (padded(h, p)) {
    ILQR_TRY(ensure_pad(h));
    ilqr_problem pp;
    ILQR_TRY(pad_problem(h, p, &pp));
    ILQR_TRY(pad_x(h, x_init, h->px));
    ILQR_TRY(pad_u(h, u_init, h->pu));
    if (x_traj) ILQR_TRY(pad_x(h, x_traj, h->pxt));
    const ilqr_status fst = ilqr_fit_ex(h->pad, &pp, o, h->px, h->pu, x_traj ? h->pxt : nullptr,
                                        h->pxn, h->pun, cost, iters, status, hist);
    if (fst != ILQR_OK && fst != ILQR_ERR_NAN && fst != ILQR_ERR_LS_EXHAUSTED) return fst;
    ILQR_TRY(unpad_x(h, h->pxn, x_out));
    ILQR_TRY(unpad_u(h, h->pun, u_out));
    HIP_TRY(hipStreamSynchronize(h->stream));  // fit returns with its outputs written
    return fst;
  }
  hipStream_t s = h->stream;
  // prev_cost = Inf (forward_pass.jl:159), status OK, result "the input", iters 0: by
  // the first iteration's kernel itself on the fused LQ path, else by a kernel here
  // the pipelined schedule interleaves two iterations per launch: a fit that records
  // its history runs the sequential schedule instead (the same bits)
  const bool pipe = !two_link(p) && h->pipelined && !hist;
  const bool init_in_iter = fused_path(h, p) && !pipe && o->max_iter > 0;
  if (!init_in_iter)
    HIP_TRY(ilqr::launch_fit_init(h->batch, h->prev_cost, h->status, h->res_parity, h->iters, s));
  volatile int32_t* flags = h->host_running + 2;
  *flags = 0;
  const ilqr::LSParams ls = ls_params(o);
  // Iteration `it` reads x̄ⁱ (the caller's x_init/u_init for it = 1, no copy; else
  // the handle's buffer (it−1)&1) and writes buffer it&1 (x̄ⁱ, ūⁱ = x̄ⁱ⁺¹, ūⁱ⁺¹,
  // :174-175). `parity` records where a trajectory's result lies when it stops:
  // ilqr::PARITY_INPUT for the caller's buffers.
  // The last iteration writes the caller's x_out / u_out directly (the gather then
  // copies only trajectories that stopped earlier) unless they overlap an input.
  const size_t xbytes = sizeof(double) * (size_t)h->batch * (h->T + 1) * h->nx;
  const size_t ubytes = sizeof(double) * (size_t)h->batch * h->T * h->nu;
  auto overlap = [](const void* a, size_t na, const void* b, size_t nb) {
    const char *pa = (const char*)a, *pb = (const char*)b;
    return b && pa < pb + nb && pb < pa + na;
  };
  const bool direct = o->max_iter > 0 && !overlap(x_out, xbytes, x_init, xbytes) &&
                      !overlap(x_out, xbytes, x_traj, xbytes) && !overlap(u_out, ubytes, u_init, ubytes) &&
                      !overlap(x_out, xbytes, u_init, ubytes) && !overlap(u_out, ubytes, x_init, xbytes) &&
                      !overlap(u_out, ubytes, x_traj, xbytes);
  auto iter_args = [&](int it) {
    const int par = (it - 1) & 1;
    const bool last = direct && it == o->max_iter;
    ilqr::IterArgs a{};
    a.x = it == 1 ? x_init : h->xbuf[par];
    a.u = it == 1 ? u_init : h->ubuf[par];
    a.xtraj = x_traj;
    a.xnew = last ? x_out : h->xbuf[par ^ 1];
    a.unew = last ? u_out : h->ubuf[par ^ 1];
    a.K = h->K;
    a.d = h->d;
    a.prev_cost = h->prev_cost;  // in place: prev_cost = new_cost (:168)
    a.new_cost = h->prev_cost;
    a.du2 = h->du2;
    a.trials = h->trials;
    a.status = h->status;
    a.res_parity = h->res_parity;
    a.iters = h->iters;
    a.parity = it == 1 ? ilqr::PARITY_INPUT : par;
    a.iter = it;
    a.init = init_in_iter && it == 1;
    return a;
  };
  if (pipe) {
    // Launch `it` runs iteration it for role-B workgroups and forward(it−1) +
    // backward(it) for role A; launch max_iter+1 drains A's last forward.
    for (int it = 1; it <= o->max_iter + 1; ++it) {
      int flags = 0;
      if (it <= o->max_iter) flags |= ilqr::PIPE_A_BW_FLAG | ilqr::PIPE_B_FLAG;
      if (it >= 2) flags |= ilqr::PIPE_A_FW_FLAG;
      if (!flags) continue;
      HIP_TRY(ilqr::launch_lq_iter_pipe(h->nx, h->nu, lq_params(p), h->batch, h->T, iter_args(it),
                                        iter_args(it - 1), ls, flags, s));
    }
  }
  // With a convergence test (tol ≥ 0) the loop stops enqueueing once every trajectory
  // has stopped, like the reference's `break` (:171): after iteration it a one-block
  // kernel writes the running count to host-mapped memory behind an event, and the host
  // reads iteration it−1's count while the GPU runs iteration it (no idle gap; at most
  // one iteration of already-stopped waves is enqueued past the last useful one).
  const bool poll = o->tol >= 0.0 && o->max_iter > 2;
  int enqueued = pipe ? o->max_iter : 0, waited = 0;  // iterations (the end-of-fit wait's units)
  for (int it = 1; !pipe && it <= o->max_iter; ++it) {  // forward_pass.jl:161
    // iterations chain per chunk: chunk 0's next backward overlaps chunk 1's forward
    const ilqr_status st = enqueue_iteration(h, p, iter_args(it), ls, /*chain=*/true, hist);
    if (st != ILQR_OK) return st;
    enqueued = it;
    // the history record and the count run behind every chunk's forward without
    // joining the main stream (a join would keep chunk 0's next backward from
    // overlapping chunk 1's forward): the forwards of all chunks are in order on the
    // side stream
    const hipStream_t ps = (two_link(p) || h->nchunks == 1) ? s : h->side;
    // (chunked: enqueue_iteration recorded each chunk right behind its forward)
    if (hist && ps == s)
      HIP_TRY(ilqr::launch_record_history(h->batch, it, h->status, h->iters, h->trials, h->prev_cost, h->du2,
                                          false, ls.alpha0, ls.shrink, hist->cost, hist->trials, hist->alpha,
                                          hist->du2, ps));
    if (!poll || it == o->max_iter) continue;
    HIP_TRY(ilqr::launch_count_running(h->batch, h->status, h->dev_running + (it & 1), ps));
    HIP_TRY(hipEventRecord(h->ev_poll[it & 1], ps));
    if (it >= 2) {
      HIP_TRY(ilqr::wait_event(h->ev_poll[(it - 1) & 1], &h->poll_wait));
      waited = it - 1;
      if (__atomic_load_n(h->host_running + ((it - 1) & 1), __ATOMIC_ACQUIRE) == 0) break;
    }
  }
  {
    const ilqr_status st = join(h, p);
    if (st != ILQR_OK) return st;
  }
  // still-running trajectories (max_iter reached) return the last accepted iterate,
  // the one the last iteration wrote (the input when max_iter = 0)
  const int last = o->max_iter == 0 ? ilqr::PARITY_INPUT : (direct ? ilqr::PARITY_OUT : (o->max_iter & 1));
  uint32_t seq = (++h->fit_seq) & 0x3fffffffu;
  if (seq == 0) seq = h->fit_seq = 1;  // 0 is the word's cleared value
  HIP_TRY(ilqr::launch_gather_result(h->batch, h->T, h->nx, h->nu, x_init, u_init, h->xbuf[0],
                                     h->ubuf[0], h->xbuf[1], h->ubuf[1], h->res_parity, h->status,
                                     last, h->prev_cost, h->iters, x_out, u_out, cost, iters,
                                     status, h->dev_flags, h->dev_running + 2, s, seq));
  HIP_TRY(wait_fit(h, seq, enqueued - waited, s));
  const int32_t f = __atomic_load_n(h->host_running + 2, __ATOMIC_ACQUIRE);
  return (f & 1) ? ILQR_ERR_NAN : ((f & 2) ? ILQR_ERR_LS_EXHAUSTED : ILQR_OK);
}

ilqr_status ilqr_malloc(ilqr_handle* h, size_t bytes, void** ptr) {
  if (!h || !ptr) return ILQR_ERR_BAD_ARG;
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipMalloc(ptr, bytes));
  return ILQR_OK;
}

ilqr_status ilqr_free(ilqr_handle* h, void* ptr) {
  if (!h) return ILQR_ERR_BAD_ARG;
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipFree(ptr));
  return ILQR_OK;
}

ilqr_status ilqr_memcpy_h2d(ilqr_handle* h, void* dst, const void* src, size_t bytes) {
  if (!h || !dst || !src) return ILQR_ERR_BAD_ARG;
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return ILQR_OK;
}

ilqr_status ilqr_memcpy_d2h(ilqr_handle* h, void* dst, const void* src, size_t bytes) {
  if (!h || !dst || !src) return ILQR_ERR_BAD_ARG;
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return ILQR_OK;
}

ilqr_status ilqr_selftest(int device, int32_t* failures) {
  const int f = ilqr::run_selftest(device);
  if (f < 0) {
    g_last_error = "selftest: HIP error";
    return ILQR_ERR_HIP;
  }
  if (failures) *failures = f;
  return ILQR_OK;
}

}  // extern "C"
