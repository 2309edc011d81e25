/*
 * ilqr.h — C ABI of the MI355X-native batched iLQR hot path (libilqr_hip.so).
 *
 * Drop-in boundary for aabouman/iLQR.jl's backward/forward passes. The
 * reference has no FFI (it is pure Julia); each entry point below replaces one
 * Julia function of the reference and is what a Julia `ccall` shim binds
 * (julia/iLQRHIP.jl):
 *
 *   ilqr_backward  <- iLQR.backward_pass   /root/reference/src/backward_pass.jl:324-357
 *   ilqr_forward   <- iLQR.forward_pass    /root/reference/src/forward_pass.jl:55-93
 *   ilqr_fit       <- iLQR.fit             /root/reference/src/forward_pass.jl:148-179
 *   ilqr_iterate   <- one iteration of fit's loop body, forward_pass.jl:162-175
 *                     (backward_pass + forward_pass fused in one launch)
 *   ilqr_linearize <- iLQR.linearize_dynamics, trajectory form  backward_pass.jl:25-40
 *
 * The reference's callbacks (dynamicsf, immediate_cost, final_cost; documented
 * at src/backward_pass.jl:11-19,54-70,122-127) are Julia closures that cannot
 * run on the device; they are replaced by a problem descriptor (ilqr_problem)
 * naming a device-side problem family. ILQR_PROBLEM_LQ is
 *   dynamicsf(x,u)      = A x + B u
 *   immediate_cost(x,u) = xᵀ Q x + uᵀ R u
 *   final_cost(x)       = xᵀ Qf x
 * with per-instance (per-trajectory) A, B, Q, R, Qf. ILQR_PROBLEM_TWO_LINK is the
 * reference's 2-link arm, test/2_link_example/2_link_helper_functions.jl:1-108
 * (nx = 4, nu = 2): RK4 (Δt = 0.01) of the arm dynamics with its CoriolisMatrix,
 * ℓ(x,u) = |θ* − θ|² + |u|², ℓ_f(x) = |θ* − θ|², θ* = InverseKinematics([0.6, −0.5]);
 * it has no per-instance data (A..Qf must be NULL) and is linearised on the
 * device by forward-mode dual numbers (what ForwardDiff does in the reference).
 *
 * Data layout (all arrays are DEVICE pointers, fp64, C row-major, trajectory
 * slowest; the same memory is a Julia column-major Array with the dimension
 * list reversed):
 *   x      (batch, T+1, nx)     Julia Array{Float64,3} (nx, T+1, batch)
 *   u, d   (batch, T,   nu)     Julia (nu, T, batch)
 *   K      (batch, T, nu, nx)   K[b,t] is the reference's Ks[t,:,:] (nu × nx)
 *   A      (batch, nx, nx)      B (batch, nx, nu)   Q, Qf (batch, nx, nx)   R (batch, nu, nu)
 *   cost, prev_cost (batch)     status, trials, iters (batch) int32
 *
 * Errors: every call returns an ilqr_status; no exceptions or aborts cross the
 * ABI. ILQR_ERR_BAD_DIMS replaces the reference's `@assert N == M+1`
 * (backward_pass.jl:329, forward_pass.jl:62,156). NaNs (the reference's
 * `@assert !any(isnan, ...)`, backward_pass.jl:353-354, forward_pass.jl:89-90)
 * are reported per trajectory in `status` (ILQR_TRAJ_NAN) and as
 * ILQR_ERR_NAN from ilqr_fit/ilqr_backward/ilqr_forward when any trajectory hit one.
 *
 * Threading: a handle is bound to one device and one HIP stream; calls are
 * asynchronous on that stream except where noted; different handles may be
 * used from different threads.
 */
#ifndef ILQR_H_
#define ILQR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ILQR_ABI_VERSION 2

typedef enum {
  ILQR_OK = 0,
  ILQR_ERR_BAD_DIMS = 1,      /* shape mismatch (reference: @assert N == M+1)          */
  ILQR_ERR_BAD_ARG = 2,       /* null pointer / bad option value                       */
  ILQR_ERR_UNSUPPORTED = 3,   /* (nx, nu) or problem kind not built into this library  */
  ILQR_ERR_HIP = 4,           /* HIP runtime error (see ilqr_last_error)               */
  ILQR_ERR_NAN = 5,           /* a trajectory produced NaN (reference: AssertionError) */
  ILQR_ERR_LS_EXHAUSTED = 6   /* a line search hit max_trials (reference: loops forever) */
} ilqr_status;

/* per-trajectory status word */
enum {
  ILQR_TRAJ_OK = 0,
  ILQR_TRAJ_CONVERGED = 1,
  ILQR_TRAJ_MAX_ITER = 2,
  ILQR_TRAJ_LS_EXHAUSTED = 3,
  ILQR_TRAJ_NAN = 4
};

typedef enum {
  ILQR_PROBLEM_LQ = 1,
  ILQR_PROBLEM_TWO_LINK = 2,
  ILQR_PROBLEM_TILES = 3, /* ilqr_backward_tiles only (caller-supplied derivatives) */
  ILQR_PROBLEM_CHAIN = 4  /* URDF serial chain: the ilqr_chain_* entry points below   */
} ilqr_problem_kind;

typedef struct {
  int32_t kind;        /* ilqr_problem_kind */
  int32_t reserved;
  const double* A;     /* (batch, nx, nx); LQ only, NULL for TWO_LINK */
  const double* B;     /* (batch, nx, nu) */
  const double* Q;     /* (batch, nx, nx) */
  const double* R;     /* (batch, nu, nu) */
  const double* Qf;    /* (batch, nx, nx) */
} ilqr_problem;

/* Per-step derivative tiles of an ARBITRARY problem along (x, u): what the
 * reference's derivative calls return — linearize_dynamics (backward_pass.jl:25-40),
 * immediate_cost_quadratization (:81-109), final_cost_quadratization (:134-153) —
 * evaluated by the caller (e.g. ForwardDiff on the host, as the reference does).
 * Device pointers, fp64, row-major, trajectory slowest. */
typedef struct {
  const double* A;     /* (batch, T, nx, nx)  ∂f/∂x at (x_t, u_t)          */
  const double* B;     /* (batch, T, nx, nu)  ∂f/∂u                         */
  const double* lx;    /* (batch, T, nx)      𝐪 = ∇ₓℓ                       */
  const double* lu;    /* (batch, T, nu)      𝐫 = ∇ᵤℓ                       */
  const double* lxx;   /* (batch, T, nx, nx)  𝐐 = ∇²ₓₓℓ                     */
  const double* lux;   /* (batch, T, nu, nx)  𝐏 = ∂(∇ᵤℓ)/∂x, NULL = zeros   */
  const double* luu;   /* (batch, T, nu, nu)  𝐑 = ∇²ᵤᵤℓ                     */
  const double* lfx;   /* (batch, nx)         ∇ℓ_f(x_N)                     */
  const double* lfxx;  /* (batch, nx, nx)     ∇²ℓ_f(x_N)                    */
} ilqr_tiles;

typedef struct {
  int32_t max_iter;    /* fit: forward_pass.jl:152 default 100                         */
  int32_t max_trials;  /* line-search cap (reference: unbounded, forward_pass.jl:70)   */
  double tol;          /* fit: forward_pass.jl:152 default 1e-6                         */
  double mu;           /* H regulariser, backward_pass.jl:214 (0.01)                    */
  double alpha0;       /* first step, forward_pass.jl:66 (1.0)                           */
  double shrink;       /* step factor, forward_pass.jl:82 (0.5)                           */
} ilqr_options;

typedef struct ilqr_handle ilqr_handle;

int ilqr_abi_version(void);
const char* ilqr_status_string(ilqr_status s);
/* last HIP error text recorded by this thread (empty string if none) */
const char* ilqr_last_error(void);
void ilqr_default_options(ilqr_options* opts);
/* 1 if (nx, nu) has a compiled kernel for `kind` */
int ilqr_supported(int32_t kind, int nx, int nu);

/* Bind a handle to `device`, preallocating the workspace (trajectory ping-pong
 * buffers, gains, per-trajectory state) for problems of this shape. Hot calls
 * never allocate. */
ilqr_status ilqr_create(ilqr_handle** out, int device, int nx, int nu, int T, int batch);
ilqr_status ilqr_destroy(ilqr_handle* h);
/* HIP stream (hipStream_t) the handle launches on; NULL = the null stream. */
ilqr_status ilqr_set_stream(ilqr_handle* h, void* hip_stream);
ilqr_status ilqr_sync(ilqr_handle* h);
/* Launch schedule of ilqr_backward / ilqr_iterate / ilqr_fit for the LQ family (bit
 * flags):
 *   ILQR_SCHED_RING_FORWARD  the forward pass streams its per-step inputs HBM → LDS
 *                            ahead of use (default on);
 *   ILQR_SCHED_BACKWARD_WAVE the backward pass runs one trajectory per wave on the
 *                            16x16x4 MFMA tile (the v6 kernel);
 *   ILQR_SCHED_BACKWARD_BLOCK the backward pass runs four trajectories per wave on
 *                            the 4x4x4 4-block MFMA (the v7 kernel). With neither
 *                            flag the handle picks BLOCK from 2048 trajectories up
 *                            and WAVE below (fewer waves than SIMDs);
 *   ILQR_SCHED_PIPELINED     fit runs one kernel per iteration in which half of the
 *                            workgroups do forward(i-1) then backward(i) while the
 *                            other half do backward(i) then forward(i) (default off;
 *                            implies ILQR_SCHED_BACKWARD_WAVE);
 *   ILQR_SCHED_FUSED         ilqr_iterate / ilqr_fit run each iteration as ONE kernel:
 *                            every wave does the backward pass of its four trajectories
 *                            then their ring forward pass (with the BLOCK backward and
 *                            the ring forward; ignored otherwise; not with WAVE or
 *                            PIPELINED). A new handle starts with RING_FORWARD | FUSED.
 *   ILQR_SCHED_FORWARD_MFMA  the ring forward pass (and the fused kernel's) runs its
 *                            mat-vecs on the 4-block f64 MFMA in the backward's layout
 *                            instead of DPP row broadcasts: the same function, other
 *                            rounding (agrees to 1e-12).
 *   ILQR_SCHED_SEQUENTIAL_SEARCH the fused iteration runs the line search wave by
 *                            wave, trial after trial (forward_pass.jl:70-87 as written).
 *                            Without it (the default) a trajectory still open after
 *                            trial 1 has its remaining trials evaluated four at a time
 *                            by every wave of the launch with nothing else to do,
 *                            ending at the first accepted trial or as soon as α·δu
 *                            vanishes at every step (each later trial is then the same
 *                            rollout): the same x̄, ū, cost, Σ(ū − u)², trial count and
 *                            status, bit for bit (max_trials ≤ 64, else
 *                            sequential).
 * Schedules with the same backward kernel return the same bits; the two backward
 * kernels agree to rounding. Unknown bits, or BLOCK with WAVE or
 * PIPELINED → ILQR_ERR_BAD_ARG. */
#define ILQR_SCHED_PIPELINED 1
#define ILQR_SCHED_RING_FORWARD 2
#define ILQR_SCHED_BACKWARD_WAVE 4
#define ILQR_SCHED_BACKWARD_BLOCK 8
#define ILQR_SCHED_FUSED 16
#define ILQR_SCHED_FORWARD_MFMA 32
#define ILQR_SCHED_SEQUENTIAL_SEARCH 64
ilqr_status ilqr_set_schedule(ilqr_handle* h, int flags);

/* iLQR.backward_pass (backward_pass.jl:324-357): gains d (batch,T,nu) and
 * K (batch,T,nu,nx) for every trajectory. With a status array (batch) the call
 * synchronises and returns ILQR_ERR_NAN if any trajectory produced a NaN gain;
 * with status == NULL it is asynchronous and reports nothing. */
ilqr_status ilqr_backward(ilqr_handle* h, const ilqr_problem* p, const ilqr_options* o,
                          const double* x, const double* u, double* d, double* K,
                          int32_t* status);

/* iLQR.backward_pass for arbitrary closures: the Riccati recursion of
 * backward_pass.jl:335-357 (optimal_controller_param, feedback_parameters,
 * step_back) on caller-supplied derivative tiles (ilqr_tiles); same outputs and
 * status behaviour as ilqr_backward. Shapes: ilqr_supported(ILQR_PROBLEM_TILES, nx, nu):
 * every nx ≤ 16, nu ≤ 8 (the reference's RBD caller, animate_RBD_2_link.jl:31, is 16 × 8
 * at T = 1000), any T. */
ilqr_status ilqr_backward_tiles(ilqr_handle* h, const ilqr_tiles* tiles, const ilqr_options* o,
                                double* d, double* K, int32_t* status);

/* iLQR.linearize_dynamics (backward_pass.jl:25-40) at every step of every
 * trajectory, the trajectory form test/test_linearize_dynamics.jl:10-14 calls:
 * A (batch, T, nx, nx) = ∂f/∂x and B (batch, T, nx, nu) = ∂f/∂u at (x_t, u_t),
 * t = 0 .. T−1 (x (batch, T+1, nx): x_T is not read; u (batch, T, nu)). LQ: f is
 * linear, so every step's A_t, B_t is the instance's A, B exactly (x, u may be NULL).
 * TWO_LINK: forward-mode dual numbers through the RK4 functor, the arithmetic of
 * ilqr_backward's own linearisation. Asynchronous. (Chains: ilqr_chain_linearize.) */
ilqr_status ilqr_linearize(ilqr_handle* h, const ilqr_problem* p, const double* x, const double* u,
                           double* A, double* B);

/* iLQR.forward_pass (forward_pass.jl:55-93): rollout + line search starting
 * from alpha0, accepting the first alpha with prev_cost - new_cost > 0; a
 * trajectory whose search exhausts max_trials gets x_new = x, u_new = u.
 * x_traj may be NULL (zeros); trials may be NULL. status as for ilqr_backward
 * (synchronising when given; ILQR_ERR_LS_EXHAUSTED / ILQR_ERR_NAN). */
ilqr_status ilqr_forward(ilqr_handle* h, const ilqr_problem* p, const ilqr_options* o,
                         const double* x, const double* u, const double* x_traj,
                         const double* d, const double* K, const double* prev_cost,
                         double* x_new, double* u_new, double* new_cost,
                         int32_t* trials, int32_t* status);

/* One iteration of fit's loop (forward_pass.jl:162-175) for every trajectory
 * whose status is ILQR_TRAJ_OK: backward, forward with line search, the
 * convergence test. Reads (x, u), writes (x_new, u_new). prev_cost (batch) is
 * the cost to beat (NULL = +Inf, fit's first iteration, forward_pass.jl:159);
 * new_cost (batch, may alias prev_cost) receives the accepted cost; du2 (batch,
 * may be NULL) receives Σ(ū_new − u)²; status is read (non-zero = skip) and
 * set to CONVERGED / LS_EXHAUSTED / NAN. A trajectory whose line search exhausts
 * max_trials leaves the LAST trial's rollout in (x_new, u_new), as the sequential
 * search of forward_pass.jl:70-87 capped at max_trials would (fit never reads it: an
 * exhausted trajectory keeps its iterate). Asynchronous. The bench "step". */
ilqr_status ilqr_iterate(ilqr_handle* h, const ilqr_problem* p, const ilqr_options* o,
                         const double* x, const double* u, const double* x_traj,
                         double* x_new, double* u_new, const double* prev_cost,
                         double* new_cost, double* du2, int32_t* trials, int32_t* status);

/* iLQR.fit (forward_pass.jl:148-179) for the whole batch. x_init/u_init are
 * the starting trajectories; x_out/u_out receive the result, which — like the
 * reference — is the iterate BEFORE the update that met `tol` (forward_pass.jl:171).
 * x_traj may be NULL. cost (batch) receives the cost of the returned iterate's
 * successor (the reference's last new_cost); iters/status (batch) may be NULL.
 * Returns ILQR_ERR_NAN / ILQR_ERR_LS_EXHAUSTED if any trajectory stopped that
 * way (others still complete). Returns once the fit's last kernel has run: every
 * output is written (the host thread spins, up to 20 ms, then falls back to the
 * stream sync, on a host-mapped word that one-thread kernel writes after every earlier
 * kernel of the stream completed; the runtime may still be retiring that kernel, so
 * work the caller enqueues next on the same stream runs after it as usual). */
ilqr_status ilqr_fit(ilqr_handle* h, const ilqr_problem* p, const ilqr_options* o,
                     const double* x_init, const double* u_init, const double* x_traj,
                     double* x_out, double* u_out, double* cost, int32_t* iters,
                     int32_t* status);

/* Per-iteration record of a fit: what the reference prints on every iteration
 * (`Iteration: i  Total Cost: new_cost`, forward_pass.jl:167) and inside its line
 * search (α, :83-85), kept per trajectory instead of printed. Device
 * arrays of max_iter × batch elements, iteration-major (element [(i−1)·batch + b] is
 * iteration i of trajectory b), each may be NULL:
 *   cost    the accepted rollout's cost (the printed Total Cost); NaN when the
 *           trajectory did not run iteration i (it had stopped) or its search failed
 *   trials  line-search trials of iteration i (0: did not run)
 *   alpha   the accepted step α = alpha0·shrink^(trials−1) (NaN as for cost)
 *   du2     Σ(ū − u)² of the iteration's last trial, the convergence test's quantity
 *           (:171; NaN: did not run)
 * Entries past a fit's last iteration (every trajectory stopped, or the poll broke
 * the loop) are left as they were. */
typedef struct {
  double* cost;
  int32_t* trials;
  double* alpha;
  double* du2;
} ilqr_history;

/* ilqr_fit plus the per-iteration record (history may be NULL: ilqr_fit). */
ilqr_status ilqr_fit_ex(ilqr_handle* h, const ilqr_problem* p, const ilqr_options* o,
                        const double* x_init, const double* u_init, const double* x_traj,
                        double* x_out, double* u_out, double* cost, int32_t* iters,
                        int32_t* status, const ilqr_history* history);

/* ---------------------------------------------------------------------------
 * RBD problem family (ILQR_PROBLEM_CHAIN): a fixed-base serial chain of revolute
 * joints described by a URDF — the reference's RigidBodyDynamics.jl example,
 * test/RBD_2_link_example/RBD_helper_functions.jl:48-116 on test/urdf/2Dof_arm.urdf
 * (BASELINE.json config 5), with the base fixed. nx = 2·n_joints (q, q̇), and
 *   dynamicsf(x, u)     = RK4(dt) of [q̇; M(q) \ (τ − dynamics_bias(q, q̇))]      (:48-79)
 *   immediate_cost(x,u) = Σ q_weightᵢ (targetᵢ − qᵢ)² + Σ r_weightₖ uₖ²         (:85-99)
 *   final_cost(x)       = Σ qf_weightᵢ (targetᵢ − qᵢ)²                          (:105-116)
 * with τ = u (nu = n_joints) or τ = [u₁, 0, …] (nu = 1). Arrays use the layout
 * above in the handle's dtype (ILQR_F32 or ILQR_F64), costs included; the
 * derivatives of dynamicsf are forward-mode duals (ForwardDiff's algorithm,
 * ILQR_LINEARIZE_DUAL) or central differences (ILQR_LINEARIZE_CENTRAL_FD).
 * Compiled shapes: ilqr_chain_supported(); ilqr_chain_dynamics also takes the
 * 6-DoF arm (n_joints = nu = 6).
 * --------------------------------------------------------------------------- */
#define ILQR_CHAIN_MAX_JOINTS 8

typedef enum { ILQR_F64 = 0, ILQR_F32 = 1 } ilqr_dtype;
typedef enum { ILQR_LINEARIZE_DUAL = 0, ILQR_LINEARIZE_CENTRAL_FD = 1 } ilqr_linearization;

typedef struct {
  int32_t n_joints;    /* revolute joints, root to tip (ilqr_amd.urdf.parse_urdf)          */
  int32_t nu;          /* n_joints (every joint driven) or 1 (joint 1 only)               */
  double dt;           /* RK4 step (Δt = 0.01 in the reference script)                    */
  double gravity[3];   /* base-frame gravity (the reference parses with zero gravity)     */
  double joint_rot[ILQR_CHAIN_MAX_JOINTS][9];  /* joint frame → parent body frame, row-major */
  double joint_pos[ILQR_CHAIN_MAX_JOINTS][3];  /* joint origin in the parent body frame      */
  double axis[ILQR_CHAIN_MAX_JOINTS][3];       /* unit axis, joint (= child body) frame     */
  double mass[ILQR_CHAIN_MAX_JOINTS];
  double com[ILQR_CHAIN_MAX_JOINTS][3];        /* COM in the body frame                     */
  double inertia[ILQR_CHAIN_MAX_JOINTS][9];    /* about the COM, body axes, row-major       */
  double target[ILQR_CHAIN_MAX_JOINTS];        /* θ* (target_pose's joint rows)             */
  double q_weight[ILQR_CHAIN_MAX_JOINTS];
  double r_weight[ILQR_CHAIN_MAX_JOINTS];
  double qf_weight[ILQR_CHAIN_MAX_JOINTS];
} ilqr_chain;

typedef struct ilqr_chain_handle ilqr_chain_handle;

/* 1 if the iLQR kernels are compiled for (n_joints, nu) */
int ilqr_chain_supported(int n_joints, int nu);
const char* ilqr_chain_last_error(void);
ilqr_status ilqr_chain_create(ilqr_chain_handle** out, int device, const ilqr_chain* chain, int T,
                              int batch, int32_t dtype, int32_t linearization);
ilqr_status ilqr_chain_destroy(ilqr_chain_handle* h);
ilqr_status ilqr_chain_set_stream(ilqr_chain_handle* h, void* hip_stream);
/* Dynamics evaluator of the iteration kernels (2-joint chains). The recursive
 * Newton-Euler restates RigidBodyDynamics.jl's dynamics_bias / mass_matrix
 * (RBD_helper_functions.jl:61-66); the closed form is the same f(x, u) as a
 * trigonometric polynomial whose coefficients the handle samples from the recursion
 * in fp64 at creation and checks against it at random states (rounding differs).
 * AUTO (a new handle) = the closed form when its check passed, else the recursion;
 * CLOSED_FORM when unavailable → ILQR_ERR_UNSUPPORTED. */
typedef enum {
  ILQR_CHAIN_DYN_AUTO = 0,
  ILQR_CHAIN_DYN_RNEA = 1,
  ILQR_CHAIN_DYN_CLOSED_FORM = 2
} ilqr_chain_dynamics_mode;
ilqr_status ilqr_chain_set_dynamics(ilqr_chain_handle* h, int32_t mode);
/* the evaluator in effect (RNEA or CLOSED_FORM), −1 for a NULL handle */
int32_t ilqr_chain_get_dynamics(const ilqr_chain_handle* h);
/* the closed form's max relative deviation from the recursion at the creation check
 * (fp64; ≥ 1e-9 means the closed form is not used) */
double ilqr_chain_closed_form_error(const ilqr_chain_handle* h);
/* cost_functions.jl's factories (src/cost_functions.jl:5-54), replacing the handle's
 * joint-space costs for 2-joint chains:
 *   simple_final_cost(mechanism, body, point, final_target, weight)(x)
 *       = weight · Σₖ (p_z(q) − final_targetₖ)²                               (:5-27)
 *   simple_immediate_cost(...)(x, u) = Σ uᵢ²  (its arguments are unused)     (:34-54)
 * where p(q) = transform_to_root(state, body) * point is the root-frame position of
 * `point` (given in the frame of body `body`: the link joint `body` moves, 0-based; −1 =
 * the fixed base) at the joint angles q = x[0:n_joints]. The reference differences the
 * point's LAST coordinate (work_space_traj[end]) against every target component
 * (ILQR_CHAIN_COST_SIMPLE keeps that reading); ILQR_CHAIN_COST_SIMPLE_EUCLIDEAN takes
 * Σₖ (pₖ − final_targetₖ)², the squared distance. The reference passes the whole state
 * to set_configuration! (a BoundsError for a fixed base); the joint angles are what it
 * can mean. ILQR_CHAIN_COST_JOINT restores the costs of ilqr_chain_create (point,
 * final_target, weight ignored). Needs the closed-form dynamics (ILQR_ERR_UNSUPPORTED
 * otherwise; ilqr_chain_set_dynamics(RNEA) is refused while a simple cost is set). */
typedef enum {
  ILQR_CHAIN_COST_JOINT = 0,
  ILQR_CHAIN_COST_SIMPLE = 1,
  ILQR_CHAIN_COST_SIMPLE_EUCLIDEAN = 2
} ilqr_chain_cost_mode;
ilqr_status ilqr_chain_set_simple_costs(ilqr_chain_handle* h, int32_t mode, int32_t body,
                                        const double* point, const double* final_target,
                                        double weight);
/* the cost mode in effect, −1 for a NULL handle */
int32_t ilqr_chain_get_cost_mode(const ilqr_chain_handle* h);
ilqr_status ilqr_chain_sync(ilqr_chain_handle* h);
/* dynamicsf for n independent (x, u) pairs: x (n, nx), u (n, nu) → x_next (n, nx) */
ilqr_status ilqr_chain_dynamics(ilqr_chain_handle* h, const void* x, const void* u, void* x_next,
                                int n);
/* linearize_dynamics (backward_pass.jl:25-40) at every (b, t): A (batch, T, nx, nx),
 * B (batch, T, nx, nu) */
ilqr_status ilqr_chain_linearize(ilqr_chain_handle* h, const void* x, const void* u, void* A,
                                 void* B);
/* iLQR.backward_pass / forward_pass / one fit iteration / fit for the chain family;
 * arguments, status and return semantics as ilqr_backward / ilqr_forward /
 * ilqr_iterate / ilqr_fit. */
ilqr_status ilqr_chain_backward(ilqr_chain_handle* h, const ilqr_options* o, const void* x,
                                const void* u, void* d, void* K, int32_t* status);
ilqr_status ilqr_chain_forward(ilqr_chain_handle* h, const ilqr_options* o, const void* x,
                               const void* u, const void* x_traj, const void* d, const void* K,
                               const void* prev_cost, void* x_new, void* u_new, void* new_cost,
                               int32_t* trials, int32_t* status);
ilqr_status ilqr_chain_iterate(ilqr_chain_handle* h, const ilqr_options* o, const void* x,
                               const void* u, const void* x_traj, void* x_new, void* u_new,
                               const void* prev_cost, void* new_cost, void* du2, int32_t* trials,
                               int32_t* status);
ilqr_status ilqr_chain_fit(ilqr_chain_handle* h, const ilqr_options* o, const void* x_init,
                           const void* u_init, const void* x_traj, void* x_out, void* u_out,
                           void* cost, int32_t* iters, int32_t* status);
/* ilqr_chain_fit plus the per-iteration record (ilqr_history, double arrays whatever
 * the handle's dtype; NULL: ilqr_chain_fit). */
ilqr_status ilqr_chain_fit_ex(ilqr_chain_handle* h, const ilqr_options* o, const void* x_init,
                              const void* u_init, const void* x_traj, void* x_out, void* u_out,
                              void* cost, int32_t* iters, int32_t* status,
                              const ilqr_history* history);

/* Multi-GPU fit in one process (what a single-process Julia host
 * uses): the batch is split into contiguous blocks over `devices` (block i holds
 * trajectories [i·batch/n, (i+1)·batch/n)); each device owns a handle and its
 * shard's buffers (allocated at create) and the shards run concurrently, one host
 * thread per device. ilqr_multi_fit takes HOST pointers with the whole batch in
 * the layout above (problem arrays included) and writes the host outputs; the
 * returned status is the most severe shard status (hard errors, then NAN, then
 * LS_EXHAUSTED). Trajectories are independent: no device-to-device traffic. */
typedef struct ilqr_multi ilqr_multi;
ilqr_status ilqr_multi_create(ilqr_multi** out, const int* devices, int n_devices, int nx, int nu,
                              int T, int batch);
ilqr_status ilqr_multi_destroy(ilqr_multi* m);
ilqr_status ilqr_multi_set_schedule(ilqr_multi* m, int flags);
int ilqr_multi_devices(const ilqr_multi* m);
ilqr_status ilqr_multi_fit(ilqr_multi* m, const ilqr_problem* host_problem, const ilqr_options* o,
                           const double* x_init, const double* u_init, const double* x_traj,
                           double* x_out, double* u_out, double* cost, int32_t* iters,
                           int32_t* status);

/* Device-resident multi-device solving (an MPC loop over many instances): the problem
 * and the trajectories stay on their devices between calls; only what the caller asks
 * for crosses PCIe.
 *   ilqr_multi_set_problem  upload the per-instance problem (host arrays, whole batch)
 *                           once; ILQR_PROBLEM_LQ / ILQR_PROBLEM_TWO_LINK;
 *   ilqr_multi_load         upload x (batch, T+1, nx), u (batch, T, nu) and/or x_traj
 *                           (host; NULL keeps what the devices hold; x and u are both
 *                           required the first time);
 *   ilqr_multi_fit_resident fit every shard from the resident (x, u) — or, with
 *                           ILQR_MULTI_WARM_START, from the previous fit's result —
 *                           into resident results; ILQR_MULTI_USE_X_TRAJ uses the loaded
 *                           x_traj. history (may be NULL): ilqr_history of the whole
 *                           batch, device arrays (max_iter, batch) on any device. Same
 *                           status rules as ilqr_multi_fit;
 *   ilqr_multi_gather       copy the last fit's results to host arrays (each may be
 *                           NULL: only what is asked for moves; pinned host memory,
 *                           e.g. from ilqr_host_alloc, moves at full PCIe rate). */
#define ILQR_MULTI_WARM_START 1
#define ILQR_MULTI_USE_X_TRAJ 2
ilqr_status ilqr_multi_set_problem(ilqr_multi* m, const ilqr_problem* host_problem);
ilqr_status ilqr_multi_load(ilqr_multi* m, const double* x, const double* u, const double* x_traj);
ilqr_status ilqr_multi_fit_resident(ilqr_multi* m, const ilqr_options* o, int flags,
                                    const ilqr_history* history);
ilqr_status ilqr_multi_gather(ilqr_multi* m, double* x_out, double* u_out, double* cost, int32_t* iters,
                              int32_t* status);
/* Pinned (page-locked) host memory for the multi-device transfers. */
ilqr_status ilqr_host_alloc(size_t bytes, void** ptr);
ilqr_status ilqr_host_free(void* ptr);

/* ---------------------------------------------------------------------------
 * Floating-base RBD family: the reference's RBD example as its script runs it —
 * test/RBD_2_link_example/RBD_helper_functions.jl:48-116 on test/urdf/2Dof_arm.urdf
 * parsed with `floating = true, gravity = 0` (:7), fitted by animate_RBD_2_link.jl:31
 * (nx = 16, nu = 8, T = 1000). Replaces, for these closures, the whole of
 * iLQR.fit (src/forward_pass.jl:148-179): linearize_dynamics in forward-mode duals
 * (ForwardDiff's algorithm), the cost tiles in closed form, the Riccati recursion of
 * ilqr_backward_tiles, forward_pass with its line search, and fit's bookkeeping, all on
 * the device.
 *   x = [p (MRP, 3); r (3); θ (n_joints); ω (3); v (3); θ̇ (n_joints)], the base twist
 *       (ω, v) in the base frame; u = [base torque (3); base force (3); joint torques]
 *   dynamicsf(x, u)     = RK4(dt) of [pdot_from_w(p, ω); v; θ̇; M(q) \ (u − bias(q, v))]
 *   immediate_cost(x,u) = q_scale·Σᵢ q_weightᵢ(targetᵢ − xᵢ)² + r_scale·Σⱼ r_weightⱼ uⱼ²
 *   final_cost(x)       = qf_scale·Σᵢ qf_weightᵢ(targetᵢ − xᵢ)²   (i over the 6 + n_joints
 *                         pose rows; the script: scales 10, 1, 100000)
 * M by the composite-rigid-body algorithm, the bias by recursive Newton-Euler at q̈ = 0,
 * in body coordinates (RigidBodyDynamics.jl is not vendored: parity against the
 * restatement in tests/closures.py). Arrays are device fp64, row-major:
 * x (batch, T+1, nx), u (batch, T, nu), A (batch, T, nx, nx), B (batch, T, nx, nu).
 * --------------------------------------------------------------------------- */
#define ILQR_FLOATING_MAX_JOINTS 2
#define ILQR_FLOATING_MAX_POSE (6 + ILQR_FLOATING_MAX_JOINTS)

typedef struct {
  int32_t n_joints;    /* revolute joints root to tip (ilqr_floating_supported)            */
  double dt;           /* RK4 step (Δt = 0.01 in the script)                                */
  double gravity[3];   /* must be zero, as the script parses the URDF                      */
  double base_mass;    /* the root link (fixed children merged), base frame               */
  double base_com[3];
  double base_inertia[9];                          /* about the COM, row-major               */
  double joint_rot[ILQR_FLOATING_MAX_JOINTS][9];   /* joint frame → parent body frame        */
  double joint_pos[ILQR_FLOATING_MAX_JOINTS][3];   /* joint origin in the parent body frame  */
  double axis[ILQR_FLOATING_MAX_JOINTS][3];        /* rotation axis, joint (= child) frame   */
  double mass[ILQR_FLOATING_MAX_JOINTS];
  double com[ILQR_FLOATING_MAX_JOINTS][3];
  double inertia[ILQR_FLOATING_MAX_JOINTS][9];
  double target[ILQR_FLOATING_MAX_POSE];           /* target_pose (animate_RBD_2_link.jl:10) */
  double q_weight[ILQR_FLOATING_MAX_POSE];
  double r_weight[ILQR_FLOATING_MAX_POSE];
  double qf_weight[ILQR_FLOATING_MAX_POSE];
  double q_scale, r_scale, qf_scale;
} ilqr_floating;

typedef struct ilqr_floating_handle ilqr_floating_handle;

/* 1 if the kernels are compiled for n_joints (2: the reference's arm) */
int ilqr_floating_supported(int n_joints);
const char* ilqr_floating_last_error(void);
/* ILQR_ERR_UNSUPPORTED for other joint counts or non-zero gravity. Device memory: the
 * iterate, its tiles and the line search's four trial slots, ≈ batch · T · 8.1 KB
 * (8.1 MB per trajectory at T = 1000) at batch > 64; the slots grow to 16 trials a
 * trajectory up to batch 64 and 64 up to batch 4 (12.3 MB per trajectory at T = 1000) */
ilqr_status ilqr_floating_create(ilqr_floating_handle** out, int device, const ilqr_floating* model,
                                 int T, int batch);
ilqr_status ilqr_floating_destroy(ilqr_floating_handle* h);
ilqr_status ilqr_floating_set_stream(ilqr_floating_handle* h, void* hip_stream);
ilqr_status ilqr_floating_sync(ilqr_floating_handle* h);
/* dynamicsf for n independent (x, u) pairs: x (n, nx), u (n, nu) → x_next (n, nx) */
ilqr_status ilqr_floating_dynamics(ilqr_floating_handle* h, const double* x, const double* u,
                                   double* x_next, int n);
/* linearize_dynamics (backward_pass.jl:25-40) at every (b, t) of x (batch, T+1, nx),
 * u (batch, T, nu) → A (batch, T, nx, nx), B (batch, T, nx, nu) */
ilqr_status ilqr_floating_linearize(ilqr_floating_handle* h, const double* x, const double* u,
                                    double* A, double* B);
/* iLQR.backward_pass / forward_pass (backward_pass.jl:324-357, forward_pass.jl:55-93)
 * for every trajectory; arguments, status and return semantics as ilqr_chain_backward /
 * ilqr_chain_forward (x_traj may be NULL; trials and status may be NULL). Synchronise. */
ilqr_status ilqr_floating_backward(ilqr_floating_handle* h, const ilqr_options* o, const double* x,
                                   const double* u, double* d, double* K, int32_t* status);
ilqr_status ilqr_floating_forward(ilqr_floating_handle* h, const ilqr_options* o, const double* x,
                                  const double* u, const double* x_traj, const double* d,
                                  const double* K, const double* prev_cost, double* x_new,
                                  double* u_new, double* new_cost, int32_t* trials, int32_t* status);
/* iLQR.fit (forward_pass.jl:148-179) for every trajectory: arguments, per-trajectory
 * status and the call status as ilqr_fit (x_traj may be NULL: zeros; cost, iters,
 * status may be NULL). Synchronises. */
ilqr_status ilqr_floating_fit(ilqr_floating_handle* h, const ilqr_options* o, const double* x_init,
                              const double* u_init, const double* x_traj, double* x_out,
                              double* u_out, double* cost, int32_t* iters, int32_t* status);
/* ilqr_floating_fit plus the per-iteration record (history may be NULL) */
ilqr_status ilqr_floating_fit_ex(ilqr_floating_handle* h, const ilqr_options* o, const double* x_init,
                                 const double* u_init, const double* x_traj, double* x_out,
                                 double* u_out, double* cost, int32_t* iters, int32_t* status,
                                 const ilqr_history* history);

/* Device memory helpers so a host-language shim (Julia ccall) needs no GPU package. */
ilqr_status ilqr_malloc(ilqr_handle* h, size_t bytes, void** ptr);
ilqr_status ilqr_free(ilqr_handle* h, void* ptr);
ilqr_status ilqr_memcpy_h2d(ilqr_handle* h, void* dst, const void* src, size_t bytes);
ilqr_status ilqr_memcpy_d2h(ilqr_handle* h, void* dst, const void* src, size_t bytes);

/* Diagnostic: runs the cross-lane and MFMA layout self-tests the kernels rely
 * on (permlane swaps, v_mfma_f64_16x16x4 fragment maps) on `device`. */
ilqr_status ilqr_selftest(int device, int32_t* failures);

#ifdef __cplusplus
}
#endif
#endif /* ILQR_H_ */
