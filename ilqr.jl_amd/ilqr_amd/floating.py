"""Floating-base RBD family (include/ilqr.h `ilqr_floating_*`): the reference's RBD example
as its script runs it, every piece of fit on the device.

The reference (test/RBD_2_link_example/) parses test/urdf/2Dof_arm.urdf with
`parse_urdf(urdf; gravity = [0, 0, 0], floating = true)` (RBD_helper_functions.jl:7),
wraps RigidBodyDynamics.jl's mass_matrix / dynamics_bias in an RK4 `dynamicsf`
(:48-79) with MRP attitude, weights the pose error and the inputs (:85-116) and calls
`iLQR.fit` on 16-state / 8-input trajectories of T = 1000 steps
(animate_RBD_2_link.jl:8-32). `FloatingSolver.fit` runs that fit natively:
forward-mode-dual linearisation, the wide tiles Riccati kernel and a line search of
4-64 trials per trajectory at once (each RK4 step split over three waves), against the generic closure path's 0.76 s per
line-search trial (tests/test_gpu_floating.py compares both with the batched closure
oracle).

    problem = rbd_example_problem()
    s = FloatingSolver(problem, T=1000, batch=1)
    x0 = rbd_initial_state()[None]                  # RBD_to_iLQR_state(...) (:22)
    x = s.rollout(x0, u)                            # the script's state_traj (:23-25)
    r = s.fit(x, u, max_iter=100, tol=1e-6)

`floating_closures(problem)` gives the reference-API callables: `ilqr_amd.fit` with them
dispatches here.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .chain import load_robot
from .solver import FitResult, _ptr, _req, alloc_history
from .urdf import Chain

# animate_RBD_2_link.jl:8-10 and RBD_helper_functions.jl:85-116
RBD_DT = 0.01
RBD_TARGET_POSE = (0.0, 0.0, 0.0, 5.0, 1.0, 2.0, 1.0, 0.3)
RBD_Q_WEIGHT = (100.0, 100.0, 100.0, 1.0, 1.0, 1.0, 10.0, 10.0)      # orr, pos, jo (:88)
RBD_R_WEIGHT = (1.0, 1.0, 1.0, 100.0, 100.0, 100.0, 10.0, 10.0)      # (:94)
RBD_QF_WEIGHT = (100.0, 100.0, 100.0, 1000.0, 1000.0, 1000.0, 10.0, 10.0)  # (:109)
RBD_SCALES = (10.0, 1.0, 100000.0)                                   # (:99, :115)


@dataclass
class FloatingProblem:
    """A floating-base chain (root link = the free base) and the script's costs."""
    chain: Chain
    dt: float = RBD_DT
    target: tuple = RBD_TARGET_POSE
    q_weight: tuple = RBD_Q_WEIGHT
    r_weight: tuple = RBD_R_WEIGHT
    qf_weight: tuple = RBD_QF_WEIGHT
    q_scale: float = RBD_SCALES[0]
    r_scale: float = RBD_SCALES[1]
    qf_scale: float = RBD_SCALES[2]

    @property
    def n_joints(self) -> int:
        return self.chain.n

    @property
    def nx(self) -> int:
        return 2 * (6 + self.chain.n)

    @property
    def nu(self) -> int:
        return 6 + self.chain.n

    def struct(self) -> _lib.FloatingStruct:
        ch, n = self.chain, self.chain.n
        if n > _lib.FLOATING_MAX_JOINTS:
            raise ValueError(f"at most {_lib.FLOATING_MAX_JOINTS} joints")
        if not ch.base_mass > 0.0:
            raise ValueError("the root link has no mass: not a floating base")
        s = _lib.FloatingStruct()
        s.n_joints, s.dt = n, float(self.dt)
        s.gravity[:] = [float(v) for v in ch.gravity]
        s.base_mass = float(ch.base_mass)
        s.base_com[:] = [float(v) for v in ch.base_com]
        s.base_inertia[:] = [float(v) for v in np.asarray(ch.base_Ic).reshape(-1)]
        for i in range(n):
            s.joint_rot[i][:] = [float(v) for v in ch.R0[i].reshape(-1)]
            s.joint_pos[i][:] = [float(v) for v in ch.p[i]]
            s.axis[i][:] = [float(v) for v in ch.axis[i]]
            s.mass[i] = float(ch.mass[i])
            s.com[i][:] = [float(v) for v in ch.com[i]]
            s.inertia[i][:] = [float(v) for v in ch.Ic[i].reshape(-1)]
        q = 6 + n
        for name in ("target", "q_weight", "r_weight", "qf_weight"):
            v = np.broadcast_to(np.asarray(getattr(self, name), float), (q,))
            getattr(s, name)[:q] = [float(e) for e in v]
        s.q_scale, s.r_scale, s.qf_scale = float(self.q_scale), float(self.r_scale), float(self.qf_scale)
        return s


def rbd_example_problem() -> FloatingProblem:
    """The reference's RBD script: 2Dof_arm.urdf floating, zero gravity, its costs."""
    return FloatingProblem(load_robot("2dof_arm"))


def rbd_initial_state() -> np.ndarray:
    """RBD_to_iLQR_state(mech_state_to_vec(state)) after set_configuration!(state,
    [0,0,0,1, .5,.75,1, 0,0]) at rest (RBD_helper_functions.jl:9, :29-32): the quaternion
    (w, x, y, z) = (0, 0, 0, 1) → MRP p = (x, y, z)/(1 + w) = (0, 0, 1)."""
    return np.array([0.0, 0.0, 1.0, 0.5, 0.75, 1.0, 0.0, 0.0] + [0.0] * 8)


class FloatingSolver:
    """Device-resident batched iLQR for one FloatingProblem (one ilqr_floating_handle)."""

    def __init__(self, problem: FloatingProblem, T: int, batch: int, device: int = 0):
        self.lib = _lib.load()
        self.p = problem
        self.nx, self.nu = problem.nx, problem.nu
        self.T, self.batch, self.device = T, batch, device
        self.dev = torch.device("cuda", device)
        self._s = problem.struct()
        h = C.c_void_p()
        _lib.check(self.lib.ilqr_floating_create(C.byref(h), device, C.byref(self._s), T, batch),
                   "ilqr_floating_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.ilqr_floating_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _bind(self):
        s = torch.cuda.current_stream(self.dev).cuda_stream
        _lib.check(self.lib.ilqr_floating_set_stream(self.h, C.c_void_p(s)), "ilqr_floating_set_stream")

    def _new(self, *shape, dtype=torch.float64):
        return torch.empty(shape, dtype=dtype, device=self.dev)

    def _xu(self, x, u):
        _req(x, torch.float64, (self.batch, self.T + 1, self.nx), "x")
        _req(u, torch.float64, (self.batch, self.T, self.nu), "u")

    def dynamics(self, x, u):
        """dynamicsf for n independent pairs: x (n, nx), u (n, nu) → (n, nx)."""
        n = x.shape[0]
        _req(x, torch.float64, (n, self.nx), "x")
        _req(u, torch.float64, (n, self.nu), "u")
        out = self._new(n, self.nx)
        self._bind()
        _lib.check(self.lib.ilqr_floating_dynamics(self.h, _ptr(x), _ptr(u), _ptr(out), n),
                   "ilqr_floating_dynamics")
        return out

    def rollout(self, x0, u):
        """x (B, T+1, nx) from x0 (B, nx) under u (B, T, nu) — the script's state_traj
        (animate_RBD_2_link.jl:23-25); T launches."""
        x0 = torch.as_tensor(x0, dtype=torch.float64, device=self.dev)
        u = torch.as_tensor(u, dtype=torch.float64, device=self.dev)
        B, T = u.shape[0], u.shape[1]
        x = self._new(B, T + 1, self.nx)
        x[:, 0] = x0
        for t in range(T):
            x[:, t + 1] = self.dynamics(x[:, t].contiguous(), u[:, t].contiguous())
        return x

    def linearize(self, x, u):
        """(A (B,T,nx,nx), B (B,T,nx,nu)) = linearize_dynamics at every (b, t)."""
        self._xu(x, u)
        A = self._new(self.batch, self.T, self.nx, self.nx)
        Bm = self._new(self.batch, self.T, self.nx, self.nu)
        self._bind()
        _lib.check(self.lib.ilqr_floating_linearize(self.h, _ptr(x), _ptr(u), _ptr(A), _ptr(Bm)),
                   "ilqr_floating_linearize")
        return A, Bm

    def backward(self, x, u, options=None):
        """iLQR.backward_pass → (d (B,T,nu), K (B,T,nu,nx), status (B,)); synchronises."""
        self._xu(x, u)
        d = self._new(self.batch, self.T, self.nu)
        K = self._new(self.batch, self.T, self.nu, self.nx)
        st = self._new(self.batch, dtype=torch.int32)
        o = options or _lib.default_options()
        self._bind()
        _lib.check(self.lib.ilqr_floating_backward(self.h, C.byref(o), _ptr(x), _ptr(u), _ptr(d), _ptr(K),
                                                   _ptr(st)), "ilqr_floating_backward", allow=(_lib.ERR_NAN,))
        return d, K, st

    def forward(self, x, u, d, K, prev_cost, x_traj=None, options=None):
        """iLQR.forward_pass → (x̄, ū, new_cost, trials, status); synchronises."""
        self._xu(x, u)
        B, T = self.batch, self.T
        _req(d, torch.float64, (B, T, self.nu), "d")
        _req(K, torch.float64, (B, T, self.nu, self.nx), "K")
        _req(prev_cost, torch.float64, (B,), "prev_cost")
        if x_traj is not None:
            _req(x_traj, torch.float64, (B, T + 1, self.nx), "x_traj")
        xn, un = torch.empty_like(x), torch.empty_like(u)
        cost = self._new(B)
        trials = self._new(B, dtype=torch.int32)
        st = self._new(B, dtype=torch.int32)
        o = options or _lib.default_options()
        self._bind()
        _lib.check(self.lib.ilqr_floating_forward(self.h, C.byref(o), _ptr(x), _ptr(u), _ptr(x_traj), _ptr(d),
                                                  _ptr(K), _ptr(prev_cost), _ptr(xn), _ptr(un), _ptr(cost),
                                                  _ptr(trials), _ptr(st)),
                   "ilqr_floating_forward", allow=(_lib.ERR_NAN, _lib.ERR_LS_EXHAUSTED))
        return xn, un, cost, trials, st

    def fit(self, x_init, u_init, max_iter=100, tol=1e-6, x_traj=None, options=None,
            history: bool = False) -> FitResult:
        """iLQR.fit (forward_pass.jl:148-179) for the whole batch; synchronises. history:
        also return the per-iteration record (ilqr_floating_fit_ex; FitResult.history)."""
        self._xu(x_init, u_init)
        if x_traj is not None:
            _req(x_traj, torch.float64, (self.batch, self.T + 1, self.nx), "x_traj")
        B = self.batch
        xo, uo = torch.empty_like(x_init), torch.empty_like(u_init)
        cost = self._new(B)
        iters = self._new(B, dtype=torch.int32)
        st = self._new(B, dtype=torch.int32)
        o = options or _lib.default_options(max_iter=max_iter, tol=tol)
        self._bind()
        hist, hst = alloc_history(o.max_iter, B, x_init.device) if history else (None, None)
        cs = _lib.check(self.lib.ilqr_floating_fit_ex(self.h, C.byref(o), _ptr(x_init), _ptr(u_init),
                                                      _ptr(x_traj), _ptr(xo), _ptr(uo), _ptr(cost),
                                                      _ptr(iters), _ptr(st),
                                                      C.byref(hst) if hst is not None else None),
                        "ilqr_floating_fit", allow=(_lib.ERR_NAN, _lib.ERR_LS_EXHAUSTED))
        return FitResult(xo, uo, cost, iters, st, cs, hist)


# -- reference-API callables (recognised by ilqr_amd.fit) ------------------------------------
class FloatingDynamics:
    """dynamicsf(x, u) of a FloatingProblem, evaluated on the device (one launch) on a
    handle cached per (model, device) (cache.py: the reference script calls dynamicsf
    1000 times to build its state_traj, animate_RBD_2_link.jl:23-25). Device tensors
    stay on their device (and come back as tensors); anything else is evaluated on the
    current device and comes back as a numpy array."""

    def __init__(self, problem: FloatingProblem):
        self.problem = problem

    def __call__(self, x, u):
        from . import cache
        on_dev = isinstance(x, torch.Tensor) and x.is_cuda
        dev = x.device if on_dev else torch.device("cuda", torch.cuda.current_device())
        xt = torch.as_tensor(x, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
        ut = torch.as_tensor(u, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
        key = ("floating", dev.index, bytes(self.problem.struct()), 1, 1)
        with torch.cuda.device(dev), \
                cache.workspace(key, lambda: FloatingSolver(self.problem, 1, 1, device=dev.index)) as s:
            y = s.dynamics(xt, ut)[0]
        return y if on_dev else y.cpu().numpy()


class FloatingCost:
    """immediate_cost(x, u) = q_scale·Σ q_weight(target − x)² + r_scale·Σ r_weight·u²
    (RBD_helper_functions.jl:85-100)."""

    def __init__(self, problem: FloatingProblem):
        self.problem = problem

    def __call__(self, x, u):
        p = self.problem
        q = 6 + p.n_joints
        e = np.asarray(p.target, float) - np.asarray(x[:q], float)
        uu = np.asarray(u, float)
        return float(np.sum(e * np.asarray(p.q_weight, float) * e) * p.q_scale
                     + np.sum(uu * np.asarray(p.r_weight, float) * uu) * p.r_scale)


class FloatingFinalCost:
    """final_cost(x) = qf_scale·Σ qf_weight(target − x)² (RBD_helper_functions.jl:106-116)."""

    def __init__(self, problem: FloatingProblem):
        self.problem = problem

    def __call__(self, x):
        p = self.problem
        q = 6 + p.n_joints
        e = np.asarray(p.target, float) - np.asarray(x[:q], float)
        return float(np.sum(e * np.asarray(p.qf_weight, float) * e) * p.qf_scale)


def floating_closures(problem: FloatingProblem):
    """(dynamicsf, immediate_cost, final_cost) of a FloatingProblem."""
    return FloatingDynamics(problem), FloatingCost(problem), FloatingFinalCost(problem)


def floating_problem_of(dynamicsf, immediate_cost, final_cost):
    """The FloatingProblem behind a recognised closure triple, else None."""
    if (isinstance(dynamicsf, FloatingDynamics) and isinstance(immediate_cost, FloatingCost)
            and isinstance(final_cost, FloatingFinalCost)
            and dynamicsf.problem is immediate_cost.problem is final_cost.problem):
        return dynamicsf.problem
    return None
