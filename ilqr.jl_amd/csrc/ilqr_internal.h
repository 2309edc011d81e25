// Internal interface between the C ABI (ilqr_abi.cpp) and the HIP kernels
// (ilqr_lq.hip). Not installed; see include/ilqr.h for the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "ilqr_wait.h"

namespace ilqr {

// Per-instance LQ problem data, device pointers, row-major, trajectory slowest.
struct LQParams {
  const double* A;   // (B, nx, nx)
  const double* B;   // (B, nx, nu)
  const double* Q;   // (B, nx, nx)
  const double* R;   // (B, nu, nu)
  const double* Qf;  // (B, nx, nx)
};

struct LSParams {
  double mu;       // regulariser added to H (backward_pass.jl:214)
  double alpha0;   // first line-search step (forward_pass.jl:66)
  double shrink;   // step factor (forward_pass.jl:82)
  double tol;      // convergence threshold on Σ(Δu)² (forward_pass.jl:171)
  int max_trials;  // line-search cap
};

// Cooperative line search of the fused LQ iteration (lq_coop_search, ilqr_fwd_ring.h;
// DESIGN.md §4): a trajectory still open after its first trial is published to a list,
// and every wave of the launch that is done with its own trajectories evaluates the
// remaining trials of published ones, four candidates per grab. Needs max_trials ≤ 64
// (one mask bit per trial).
struct LSCoopRec {  // per trajectory, agent-scope atomics only
  int32_t next;     // next trial to hand out
  int32_t best;     // smallest accepted trial (max_trials + 1: none yet)
  int32_t stop;     // smallest rejected trial whose α·δu vanished (max_trials + 1: none)
  int32_t fin;      // 0 → 1 by the wave that finalises the trajectory
  uint64_t mask;    // bit j − 1: trial j evaluated
  int32_t slot;     // its position in the launch's list (written before the entry)
  int32_t pad;
};
struct LSCoop {
  LSCoopRec* rec;     // (B); nullptr: the sequential search of the ring forward
  double* cost;       // (B, 64) each evaluated trial's cost
  double* du2;        // (B, 64) each evaluated trial's Σ(ū − u)²
  uint64_t* list;     // (B) published trajectories: launch generation << 32 | trajectory
                      // (an entry of another generation is stale: not written yet)
  int32_t* ctl;       // [gen & 1]: list length of launch `gen` (the launch zeroes the other)
  // Rollouts of every evaluated trial of the first `nslots` searches of a launch (list
  // positions < nslots): (nslots, 64, T+1, nx) and (nslots, 64, T, nu). Their finaliser
  // copies the accepted trial's instead of rolling it out again.
  double* sx;
  double* su;
  int32_t nslots;     // 0: no scratch (every finaliser rolls out)
};
#ifndef ILQR_COOP_SCRATCH_SLOTS  // A/B builds only
#define ILQR_COOP_SCRATCH_SLOTS 32
#endif
constexpr int COOP_SCRATCH_SLOTS = ILQR_COOP_SCRATCH_SLOTS;
// coop_find reads (next, best) and (stop, fin) as one 64-bit word each
static_assert(sizeof(LSCoopRec) == 32 && offsetof(LSCoopRec, best) == 4 && offsetof(LSCoopRec, stop) == 8 &&
                  offsetof(LSCoopRec, fin) == 12 && offsetof(LSCoopRec, mask) == 16,
              "LSCoopRec layout");
constexpr int COOP_MAX_TRIALS = 64;

// Buffers of one fused iteration (fit loop body).
struct IterArgs {
  const double* x;      // (B, T+1, nx) current iterate
  const double* u;      // (B, T, nu)
  const double* xtraj;  // (B, T+1, nx) or nullptr (zeros)
  double* xnew;         // (B, T+1, nx) next iterate
  double* unew;         // (B, T, nu)
  double* K;            // (B, T, nu, nx) gains workspace
  double* d;            // (B, T, nu)
  const double* prev_cost;  // (B) in; nullptr = +Inf (fit's first iteration, forward_pass.jl:159)
  double* new_cost;         // (B) out: cost of the accepted rollout (may alias prev_cost)
  double* du2;          // (B) out, may be null
  int32_t* trials;      // (B) out, may be null
  int32_t* status;      // (B) in/out (non-zero = skip)
  int32_t* res_parity;  // (B) out, may be null: buffer parity holding the result when a trajectory stops
  int32_t* iters;       // (B) out, may be null: last iteration index that processed the trajectory
  int parity;           // parity of (x, u) in the fit ping-pong
  int iter;             // 1-based iteration index (fit)
  int init;             // fit's first iteration on the fused LQ kernel: the kernel itself sets
                        // prev_cost = Inf, status OK, res_parity = input, iters = 0 (fit_init)
  const LSCoop* coop;   // the fused LQ kernel's cooperative line search (device memory, one
                        // per handle; read only when the search starts, so its pointers
                        // hold no SGPRs through the backward pass); nullptr: off
  uint32_t coop_gen;    // the launch's generation (per handle, counts cooperative launches)
  int32_t* coop_ctl;    // == coop->ctl, in the kernel arguments: a wave's exit test at the end
                        // of its own work is ONE load (no dependent load of *coop first)
};

// Returns hipSuccess or the launch error. All launches are asynchronous on `s`.
hipError_t launch_lq_backward(int nx, int nu, const LQParams& p, int B, int T, const double* x,
                              const double* u, double* d, double* K, int32_t* status, double mu,
                              hipStream_t s, bool wave = false);
// (12, 4) goes to the four-trajectories-per-wave kernel (ilqr_bw4.hip) unless
// `wave` (ILQR_SCHED_BACKWARD_WAVE) selects the one-trajectory-per-wave kernel
// (launch_lq_backward_v6), which the pipelined schedule's fused kernel also runs.
hipError_t launch_lq_backward4(const LQParams& p, int B, int T, const double* x, const double* u,
                               double* d, double* K, int32_t* status, double mu, hipStream_t s);
hipError_t launch_lq_iter_backward4(const LQParams& p, int B, int T, const IterArgs& a, double mu,
                                    hipStream_t s);
// backward (four trajectories per wave) + LDS-ring forward of one fit iteration in one
// launch, (12, 4) only; the same bits as the two launches
hipError_t launch_lq_iter_fused4(const LQParams& p, int B, int T, const IterArgs& a, const LSParams& ls,
                                 hipStream_t s, bool mfma = false);
hipError_t launch_lq_backward_v6(int nx, int nu, const LQParams& p, int B, int T, const double* x,
                                 const double* u, double* d, double* K, int32_t* status, double mu,
                                 hipStream_t s);
hipError_t launch_lq_forward(int nx, int nu, const LQParams& p, int B, int T, const double* x,
                             const double* u, const double* xtraj, const double* d,
                             const double* K, const double* prev_cost, double* xnew,
                             double* unew, double* new_cost, int32_t* trials, int32_t* status,
                             const LSParams& ls, hipStream_t s, bool ring = false, bool mfma = false);
// The two halves of one fit iteration over trajectories [b0, b1) (pointers in
// `a` and `p` address the whole batch).
hipError_t launch_lq_iter_backward(int nx, int nu, const LQParams& p, int b0, int b1, int T,
                                   const IterArgs& a, double mu, hipStream_t s, bool wave = false);
hipError_t launch_lq_iter_forward(int nx, int nu, const LQParams& p, int b0, int b1, int T,
                                  const IterArgs& a, const LSParams& ls, hipStream_t s,
                                  bool ring = false, bool mfma = false);
// Pipelined fit iteration (DESIGN.md §fit driver): role-B workgroups run iteration
// `cur` (backward then forward), role-A workgroups the forward of iteration `prev`
// then the backward of `cur`; flags select the phases (PIPE_* below).
constexpr int PIPE_A_FW_FLAG = 1, PIPE_A_BW_FLAG = 2, PIPE_B_FLAG = 4;
hipError_t launch_lq_iter_pipe(int nx, int nu, const LQParams& p, int B, int T, const IterArgs& cur,
                               const IterArgs& prev, const LSParams& ls, int flags, hipStream_t s);
// Result buffer codes of the fit ping-pong: 0 / 1 the handle's buffers, PARITY_INPUT
// the caller's x_init / u_init (iteration 1 reads them in place).
constexpr int PARITY_INPUT = 2;
// ... and PARITY_OUT the caller's x_out / u_out (fit's last iteration writes there
// directly when they do not alias the inputs, so the gather copies only trajectories
// that stopped earlier)
constexpr int PARITY_OUT = 3;
// fit's per-trajectory state: prev_cost = +Inf, status OK, res_parity INPUT, iters 0.
hipError_t launch_fit_init(int B, double* prev_cost, int32_t* status, int32_t* res_parity,
                           int32_t* iters, hipStream_t s);
// x_out[b] = the buffer res_parity[b] names (final_parity for still-running ones,
// whose status becomes MAX_ITER), and u; cost/iters/status copied out (each may be
// null). The call-status bits go through dflags (two zeroed device words, re-armed by
// the kernel) into `flags` (host-mapped, may be null) as (seq << 2) | bits.
hipError_t launch_gather_result(int B, int T, int nx, int nu, const double* xin, const double* uin,
                                const double* x0, const double* u0, const double* x1,
                                const double* u1, const int32_t* res_parity, int32_t* status,
                                int final_parity, const double* fit_cost, const int32_t* fit_iters,
                                double* x_out, double* u_out, double* cost_out,
                                int32_t* iters_out, int32_t* status_out, int32_t* dflags,
                                int32_t* flags, hipStream_t s, uint32_t seq = 0);
// (N, R, C) row-major → (N, R2, C2) zero-padded (R2 ≥ R, C2 ≥ C), and back.
hipError_t launch_pad3(const double* src, double* dst, size_t N, int R, int C, int R2, int C2,
                       hipStream_t s);
hipError_t launch_unpad3(const double* src, double* dst, size_t N, int R, int C, int R2, int C2,
                         hipStream_t s);
hipError_t launch_fill_i32(int32_t* p, int n, int32_t v, hipStream_t s);
hipError_t launch_fill_f64(double* p, int n, double v, hipStream_t s);
// fit's per-iteration record (ilqr_history, include/ilqr.h) of iteration `it`, from the
// per-trajectory words the iteration kernels left (iters[b] == it: the trajectory ran
// it; cost = the in-place prev_cost; status after the iteration). Cost/du2 arrays of
// the family's dtype (f32: float), α formed in that dtype as the forward formed it.
// `stride`: the history arrays' row length (0: B); a chunk of the batch passes its
// offset pointers, its own B and the whole batch as the stride.
hipError_t launch_record_history(int B, int it, const int32_t* status, const int32_t* iters,
                                 const int32_t* trials, const void* cost, const void* du2, bool f32,
                                 double alpha0, double shrink, double* h_cost, int32_t* h_trials,
                                 double* h_alpha, double* h_du2, hipStream_t s, int stride = 0);
// linearize_dynamics (ilqr_linearize): A (B, T, nx, nx), Bm (B, T, nx, nu) — the LQ
// instance's matrices at every step
hipError_t launch_lq_linearize(int nx, int nu, const LQParams& p, int B, int T, double* A, double* Bm,
                               hipStream_t s);
// *out = #trajectories with status OK (out may be host-mapped memory)
hipError_t launch_count_running(int B, const int32_t* status, int32_t* out, hipStream_t s);
// The last launch of a fit (gather_flags_kernel): dflags[0] (a gather's call-status
// bits, re-armed) into the host-mapped word `flags` as (seq << 2) | bits.
hipError_t launch_publish_flags(int32_t* dflags, int32_t* flags, uint32_t seq, hipStream_t s);
// The host's end of a fit: wait until the host-mapped word carries `seq` in bits 2..31,
// `units` = the fit iterations the wait covers (the policy: ilqr_wait.h; ILQR_FIT_WAIT=sync
// forces the stream sync). wait_event: the same for an event (the fit drivers' polls, one
// iteration each). One HostWait per waiting site of a handle.
hipError_t wait_host_seq(const volatile int32_t* word, uint32_t seq, int units, hipStream_t s, HostWait* hw);
hipError_t wait_event(hipEvent_t ev, HostWait* hw);
bool lq_supported(int nx, int nu);

// Caller-supplied derivative tiles (ilqr_tiles in include/ilqr.h), device pointers.
struct TileParams {
  const double *A, *B, *lx, *lu, *lxx, *lux, *luu, *lfx, *lfxx;  // lux may be null (zeros)
};
bool tiles_supported(int nx, int nu);
hipError_t launch_tiles_backward(int nx, int nu, const TileParams& p, int B, int T, double* d,
                                 double* K, int32_t* status, double mu, hipStream_t s);

// 2-link arm (ILQR_PROBLEM_TWO_LINK, test/2_link_example/2_link_helper_functions.jl):
// the constants of the reference script, computed on the host in its expression order.
struct TwoLinkParams {
  double alpha, beta, delta;  // inertia parameters (:11-13)
  double dt;                  // RK4 step Δt (:14)
  double tgt0, tgt1;          // θ* = InverseKinematics(target_tool_loc) (:16-26)
};
TwoLinkParams two_link_params();
bool tl_supported(int nx, int nu);  // (4, 2), and (4, 1): f(x, [u₁, 0])
size_t tl_workspace_doubles(int B, int T);  // linearisation workspace J
// backward = linearise every (b, t) into J, then the Riccati recursion
hipError_t launch_tl_backward(const TwoLinkParams& P, int nu, int B, int T, const double* x,
                              const double* u, double* J, double* d, double* K, int32_t* status,
                              double mu, hipStream_t s);
hipError_t launch_tl_forward(const TwoLinkParams& P, int nu, int B, int T, const double* x,
                             const double* u, const double* xtraj, const double* d,
                             const double* K, const double* prev_cost, double* xnew,
                             double* unew, double* new_cost, int32_t* trials, int32_t* status,
                             const LSParams& ls, hipStream_t s);
// linearize_dynamics at every (b, t) in the caller's layout (ilqr_linearize):
// A (B, T, 4, 4), Bm (B, T, 4, nu), the backward's Dual<4+nu> arithmetic
hipError_t launch_tl_jacobian(const TwoLinkParams& P, int nu, int B, int T, const double* x,
                              const double* u, double* A, double* Bm, hipStream_t s);
// one fit iteration (linearise, backward, forward) for trajectories with status OK
hipError_t launch_tl_iteration(const TwoLinkParams& P, int nu, int B, int T, const IterArgs& a,
                               double* J, const LSParams& ls, hipStream_t s);
int run_selftest(int device);  // number of failed checks, or -1 on HIP error

}  // namespace ilqr
