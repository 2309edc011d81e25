"""RBD problem family (ILQR_PROBLEM_CHAIN): the reference's RigidBodyDynamics.jl
example on a fixed-base serial chain, solved by the ilqr_chain_* kernels.

Reference: test/RBD_2_link_example/RBD_helper_functions.jl (dynamicsf :48-79 —
RK4 of v̇ = M \\ (−dynamics_bias + u); immediate_cost :85-99; final_cost
:105-116), animate_RBD_2_link.jl (Δt = 0.01, target_pose, :8-10) and
test/urdf/2Dof_arm.urdf. BASELINE.json config 5 runs the 2-DoF arm with a fixed
base (nx = 4) in fp32; the reference's floating base (16 states, MRP attitude)
is outside the hot path. The costs keep the reference's joint
rows: Q = 10·diag(jo_cost = 10) → q_weight 100, R = diag(jo_tor_cost = 10) →
r_weight 10, final Q = 1e5·diag(10) → qf_weight 1e6, target θ* = (1.0, 0.3).

`ChainSolver` owns one ilqr_chain_handle; tensors are torch CUDA tensors in the
solver's dtype (float32 or float64), laid out as include/ilqr.h documents.
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from .solver import FitResult, _ptr, _req, alloc_history
from .urdf import Chain, parse_urdf

ROBOTS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "robots")

# the reference's RBD example (RBD_helper_functions.jl:85-116, animate_RBD_2_link.jl:8-10)
RBD_DT = 0.01
RBD_TARGET_JOINTS = (1.0, 0.3)          # target_pose[7:8]
RBD_Q_JOINT = 10.0 * 10.0               # jo_cost 10, euclidean_penalty * 10.0
RBD_R_JOINT = 10.0 * 1.0                # jo_tor_cost 10, torque_penalty * 1.0
RBD_QF_JOINT = 10.0 * 100000.0          # jo_cost 10, euclidean_penalty * 100000.0


def load_robot(name: str) -> Chain:
    """A chain description shipped with the package ('2dof_arm', '6dof_arm'; made from
    the reference's test/urdf by tools/make_robots.py) or a path to a URDF file."""
    if name.endswith(".urdf"):
        return parse_urdf(name)
    with open(os.path.join(ROBOTS, name + ".json")) as f:
        d = json.load(f)
    return Chain(d["names"], np.array(d["R0"]), np.array(d["p"]), np.array(d["axis"]),
                 np.array(d["mass"]), np.array(d["com"]), np.array(d["Ic"]), np.array(d["gravity"]),
                 float(d.get("base_mass", 0.0)), np.array(d.get("base_com", [0.0] * 3), float),
                 np.array(d.get("base_Ic", np.zeros((3, 3)).tolist()), float))


@dataclass
class ChainProblem:
    """A chain plus the joint-space quadratic costs of the reference's RBD example."""
    chain: Chain
    nu: int
    dt: float = RBD_DT
    target: np.ndarray = None
    q_weight: np.ndarray = None
    r_weight: np.ndarray = None
    qf_weight: np.ndarray = None

    def __post_init__(self):
        n = self.chain.n
        if self.nu not in (n, 1):
            raise ValueError("nu must be n_joints (every joint driven) or 1 (joint 1 only)")
        def vec(v, default):
            return np.full(n, default, float) if v is None else np.broadcast_to(np.asarray(v, float), (n,)).copy()
        self.target = vec(self.target, 0.0)
        self.q_weight = vec(self.q_weight, 1.0)
        self.r_weight = vec(self.r_weight, 1.0)
        self.qf_weight = vec(self.qf_weight, 1.0)

    @property
    def n_joints(self):
        return self.chain.n

    @property
    def nx(self):
        return 2 * self.chain.n

    def struct(self) -> _lib.ChainStruct:
        ch, n = self.chain, self.chain.n
        if n > _lib.CHAIN_MAX_JOINTS:
            raise ValueError(f"at most {_lib.CHAIN_MAX_JOINTS} joints")
        s = _lib.ChainStruct()
        s.n_joints, s.nu, s.dt = n, self.nu, self.dt
        s.gravity[:] = [float(v) for v in ch.gravity]
        for i in range(n):
            s.joint_rot[i][:] = [float(v) for v in ch.R0[i].reshape(-1)]
            s.joint_pos[i][:] = [float(v) for v in ch.p[i]]
            s.axis[i][:] = [float(v) for v in ch.axis[i]]
            s.mass[i] = float(ch.mass[i])
            s.com[i][:] = [float(v) for v in ch.com[i]]
            s.inertia[i][:] = [float(v) for v in ch.Ic[i].reshape(-1)]
            s.target[i] = float(self.target[i])
            s.q_weight[i] = float(self.q_weight[i])
            s.r_weight[i] = float(self.r_weight[i])
            s.qf_weight[i] = float(self.qf_weight[i])
        return s


def rbd_2dof_problem(nu: int = 2) -> ChainProblem:
    """BASELINE config 5: the reference's RBD example on 2Dof_arm.urdf with a fixed base.
    nu = 2 (every joint driven, the reference's u ∈ R^nv convention) or nu = 1 (joint 1
    only, BASELINE's 'nᵤ=1' row; not reference-pinned)."""
    return ChainProblem(load_robot("2dof_arm"), nu, RBD_DT, RBD_TARGET_JOINTS, RBD_Q_JOINT,
                        RBD_R_JOINT, RBD_QF_JOINT)


def coupled_2dof_problem(nu: int = 2) -> ChainProblem:
    """A non-degenerate 2-joint chain for parity tests (not a reference robot): the
    2Dof_arm's joint layout with the first joint frame tilted, COMs off the joint
    origins, anisotropic inertias with products of inertia, and gravity on. Unlike the
    2Dof_arm (COMs on the joint axes, 0.5·I inertias, zero gravity: constant
    M = diag(4, 0.5), zero bias), M(q) is dense and q-dependent and the bias carries
    Coriolis and gravity terms, so A's q-columns are nonzero."""
    ch = load_robot("2dof_arm")
    c, s = math.cos(0.3), math.sin(0.3)
    R0 = ch.R0.copy()
    R0[0] = np.array([[1.0, 0.0, 0.0], [0.0, c, -s], [0.0, s, c]])   # joint 1 tilted about x
    com = np.array([[0.10, 0.05, 0.20], [0.30, 0.05, -0.15]])
    Ic = np.array([[[0.40, 0.02, 0.01], [0.02, 0.60, 0.03], [0.01, 0.03, 0.30]],
                   [[0.20, 0.01, -0.02], [0.01, 0.35, 0.015], [-0.02, 0.015, 0.25]]])
    chain = Chain(list(ch.names), R0, ch.p.copy(), ch.axis.copy(), np.array([3.0, 2.0]), com, Ic,
                  np.array([0.0, 0.0, -9.81]))
    return ChainProblem(chain, nu, RBD_DT, RBD_TARGET_JOINTS, RBD_Q_JOINT, RBD_R_JOINT, RBD_QF_JOINT)


def rbd_initial_states(batch: int, n_joints: int = 2, seed0: int = 0):
    """x₀[b] = [q ~ U(−1, 1)^n, q̇ = 0] from numpy.random.default_rng(seed0 + b)."""
    x0 = np.zeros((batch, 2 * n_joints))
    for b in range(batch):
        x0[b, :n_joints] = np.random.default_rng(seed0 + b).uniform(-1.0, 1.0, n_joints)
    return x0


_LIN = {"dual": _lib.LINEARIZE_DUAL, "fd": _lib.LINEARIZE_CENTRAL_FD}


class ChainSolver:
    """Device-resident batched iLQR for one ChainProblem (one ilqr_chain_handle)."""

    def __init__(self, problem: ChainProblem, T: int, batch: int, dtype=torch.float64,
                 linearization: str = "dual", device: int = 0):
        self.lib = _lib.load()
        self.p = problem
        self.nj, self.nu, self.nx = problem.n_joints, problem.nu, problem.nx
        self.T, self.batch, self.device = T, batch, device
        if dtype not in (torch.float32, torch.float64):
            raise TypeError("dtype must be torch.float32 or torch.float64")
        self.dtype = dtype
        self.dev = torch.device("cuda", device)
        self._s = problem.struct()
        h = C.c_void_p()
        _lib.check(self.lib.ilqr_chain_create(C.byref(h), device, C.byref(self._s), T, batch,
                                              _lib.F32 if dtype == torch.float32 else _lib.F64,
                                              _LIN[linearization]), "ilqr_chain_create")
        self.h = h
        self.iterates = bool(self.lib.ilqr_chain_supported(self.nj, self.nu))

    def set_dynamics(self, mode: str):
        """The iteration kernels' dynamics evaluator (2-joint chains): "auto" (the closed
        form when its creation check passed), "rnea" (the recursive Newton-Euler, the
        restatement of RigidBodyDynamics.jl's calls) or "closed_form"."""
        m = {"auto": _lib.CHAIN_DYN_AUTO, "rnea": _lib.CHAIN_DYN_RNEA,
             "closed_form": _lib.CHAIN_DYN_CLOSED_FORM}[mode]
        _lib.check(self.lib.ilqr_chain_set_dynamics(self.h, m), "ilqr_chain_set_dynamics")

    @property
    def dynamics_mode(self) -> str:
        return {_lib.CHAIN_DYN_RNEA: "rnea", _lib.CHAIN_DYN_CLOSED_FORM: "closed_form"}[
            int(self.lib.ilqr_chain_get_dynamics(self.h))]

    @property
    def closed_form_error(self) -> float:
        """Max relative deviation of the closed form from the recursion at creation."""
        return float(self.lib.ilqr_chain_closed_form_error(self.h))

    def set_simple_costs(self, body, point, final_target, weight, euclidean: bool = False):
        """cost_functions.jl's simple_immediate_cost / simple_final_cost in place of the
        problem's joint-space costs (ilqr_chain_set_simple_costs): ℓ = Σ uᵢ² and
        ℓ_f = weight·Σₖ (p_z − final_targetₖ)² for the point `point` of body `body`
        (0-based link index or the name of the joint that moves it; −1 = the base), or
        the squared distance Σₖ (pₖ − final_targetₖ)² with euclidean=True."""
        b = body_index(self.p.chain, body)
        pt = (C.c_double * 3)(*[float(v) for v in np.asarray(point, float).reshape(3)])
        tg = (C.c_double * 3)(*[float(v) for v in np.asarray(final_target, float).reshape(3)])
        mode = _lib.CHAIN_COST_SIMPLE_EUCLIDEAN if euclidean else _lib.CHAIN_COST_SIMPLE
        _lib.check(self.lib.ilqr_chain_set_simple_costs(self.h, mode, b, pt, tg, float(weight)),
                   "ilqr_chain_set_simple_costs")

    def set_joint_costs(self):
        """Back to the ChainProblem's joint-space costs."""
        _lib.check(self.lib.ilqr_chain_set_simple_costs(self.h, _lib.CHAIN_COST_JOINT, 0, None, None, 0.0),
                   "ilqr_chain_set_simple_costs")

    @property
    def cost_mode(self) -> str:
        return {_lib.CHAIN_COST_JOINT: "joint", _lib.CHAIN_COST_SIMPLE: "simple",
                _lib.CHAIN_COST_SIMPLE_EUCLIDEAN: "simple_euclidean"}[
            int(self.lib.ilqr_chain_get_cost_mode(self.h))]

    def close(self):
        if getattr(self, "h", None):
            self.lib.ilqr_chain_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _bind(self):
        s = torch.cuda.current_stream(self.dev).cuda_stream
        _lib.check(self.lib.ilqr_chain_set_stream(self.h, C.c_void_p(s)), "ilqr_chain_set_stream")

    def _new(self, *shape, dtype=None):
        return torch.empty(shape, dtype=dtype or self.dtype, device=self.dev)

    def _xu(self, x, u):
        B, T = self.batch, self.T
        _req(x, self.dtype, (B, T + 1, self.nx), "x")
        _req(u, self.dtype, (B, T, self.nu), "u")

    # -- primitives ----------------------------------------------------------------------
    def dynamics(self, x, u):
        """dynamicsf for n independent pairs: x (n, nx), u (n, nu) → (n, nx)."""
        n = x.shape[0]
        _req(x, self.dtype, (n, self.nx), "x")
        _req(u, self.dtype, (n, self.nu), "u")
        out = self._new(n, self.nx)
        self._bind()
        _lib.check(self.lib.ilqr_chain_dynamics(self.h, _ptr(x), _ptr(u), _ptr(out), n),
                   "ilqr_chain_dynamics")
        return out

    def rollout(self, x0, u):
        """x (B, T+1, nx) from x0 (B, nx) under u (B, T, nu) (T dynamics launches)."""
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
        _lib.check(self.lib.ilqr_chain_linearize(self.h, _ptr(x), _ptr(u), _ptr(A), _ptr(Bm)),
                   "ilqr_chain_linearize")
        return A, Bm

    def backward(self, x, u, options=None):
        """iLQR.backward_pass → (d (B,T,nu), K (B,T,nu,nx), status (B,)); synchronises."""
        self._xu(x, u)
        d = self._new(self.batch, self.T, self.nu)
        K = self._new(self.batch, self.T, self.nu, self.nx)
        st = self._new(self.batch, dtype=torch.int32)
        o = options or _lib.default_options()
        self._bind()
        _lib.check(self.lib.ilqr_chain_backward(self.h, C.byref(o), _ptr(x), _ptr(u), _ptr(d),
                                                _ptr(K), _ptr(st)),
                   "ilqr_chain_backward", allow=(_lib.ERR_NAN,))
        return d, K, st

    def forward(self, x, u, d, K, prev_cost, x_traj=None, options=None):
        """iLQR.forward_pass → (x̄, ū, new_cost, trials, status); synchronises."""
        self._xu(x, u)
        B, T = self.batch, self.T
        _req(d, self.dtype, (B, T, self.nu), "d")
        _req(K, self.dtype, (B, T, self.nu, self.nx), "K")
        _req(prev_cost, self.dtype, (B,), "prev_cost")
        if x_traj is not None:
            _req(x_traj, self.dtype, (B, T + 1, self.nx), "x_traj")
        xn, un = torch.empty_like(x), torch.empty_like(u)
        cost = self._new(B)
        trials = self._new(B, dtype=torch.int32)
        st = self._new(B, dtype=torch.int32)
        o = options or _lib.default_options()
        self._bind()
        _lib.check(self.lib.ilqr_chain_forward(self.h, C.byref(o), _ptr(x), _ptr(u), _ptr(x_traj),
                                               _ptr(d), _ptr(K), _ptr(prev_cost), _ptr(xn),
                                               _ptr(un), _ptr(cost), _ptr(trials), _ptr(st)),
                   "ilqr_chain_forward", allow=(_lib.ERR_NAN, _lib.ERR_LS_EXHAUSTED))
        return xn, un, cost, trials, st

    def iterate(self, x, u, x_new, u_new, prev_cost, status, new_cost, du2=None, trials=None,
                x_traj=None, options=None):
        """One fit iteration (asynchronous): the bench step of config 5."""
        o = options or _lib.default_options()
        _lib.check(self.lib.ilqr_chain_iterate(self.h, C.byref(o), _ptr(x), _ptr(u), _ptr(x_traj),
                                               _ptr(x_new), _ptr(u_new), _ptr(prev_cost),
                                               _ptr(new_cost), _ptr(du2), _ptr(trials),
                                               _ptr(status)), "ilqr_chain_iterate")

    def fit(self, x_init, u_init, max_iter=100, tol=1e-6, x_traj=None, options=None,
            history: bool = False) -> FitResult:
        """iLQR.fit (forward_pass.jl:148-179) for the whole batch; synchronises. history:
        also return the per-iteration record (ilqr_chain_fit_ex; FitResult.history)."""
        self._xu(x_init, u_init)
        B = self.batch
        xo, uo = torch.empty_like(x_init), torch.empty_like(u_init)
        cost = self._new(B)
        iters = self._new(B, dtype=torch.int32)
        st = self._new(B, dtype=torch.int32)
        o = options or _lib.default_options(max_iter=max_iter, tol=tol)
        self._bind()
        hist, hst = alloc_history(o.max_iter, B, x_init.device) if history else (None, None)
        cs = _lib.check(self.lib.ilqr_chain_fit_ex(self.h, C.byref(o), _ptr(x_init), _ptr(u_init),
                                                   _ptr(x_traj), _ptr(xo), _ptr(uo), _ptr(cost),
                                                   _ptr(iters), _ptr(st),
                                                   C.byref(hst) if hst is not None else None),
                        "ilqr_chain_fit", allow=(_lib.ERR_NAN, _lib.ERR_LS_EXHAUSTED))
        return FitResult(xo, uo, cost, iters, st, cs, hist)


# -- reference-API callables (recognised by ilqr_amd.fit & co.) ---------------------------
class ChainDynamics:
    """dynamicsf(x, u) of a ChainProblem, evaluated on the device (one launch)."""

    def __init__(self, problem: ChainProblem):
        self.problem = problem

    def __call__(self, x, u):
        xt = torch.as_tensor(np.asarray(x, float), device="cuda")[None].contiguous()
        ut = torch.as_tensor(np.asarray(u, float), device="cuda")[None].contiguous()
        s = ChainSolver(self.problem, 1, 1, torch.float64)
        try:
            return s.dynamics(xt, ut)[0].cpu().numpy()
        finally:
            s.close()


class ChainCost:
    """immediate_cost(x, u) = Σ q_weightᵢ(θ*ᵢ − θᵢ)² + Σ r_weightₖ uₖ²."""

    def __init__(self, problem: ChainProblem):
        self.problem = problem

    def __call__(self, x, u):
        p = self.problem
        e = p.target - np.asarray(x[: p.n_joints], float)
        return float(np.sum(p.q_weight * e * e) + np.sum(p.r_weight[: p.nu] * np.asarray(u, float) ** 2))


class ChainFinalCost:
    """final_cost(x) = Σ qf_weightᵢ(θ*ᵢ − θᵢ)²."""

    def __init__(self, problem: ChainProblem):
        self.problem = problem

    def __call__(self, x):
        p = self.problem
        e = p.target - np.asarray(x[: p.n_joints], float)
        return float(np.sum(p.qf_weight * e * e))


def chain_closures(problem: ChainProblem):
    """(dynamicsf, immediate_cost, final_cost) of a ChainProblem."""
    return ChainDynamics(problem), ChainCost(problem), ChainFinalCost(problem)


def body_index(chain: Chain, body) -> int:
    """A body of the chain as ilqr_chain_set_simple_costs numbers it: the link joint i
    moves is body i (RigidBodyDynamics' successor of joint i), −1 the fixed base. Takes
    the index or the joint's name."""
    if isinstance(body, str):
        if body not in chain.names:
            raise ValueError(f"no joint named {body!r} (joints: {chain.names})")
        return chain.names.index(body)
    b = int(body)
    if not -1 <= b < chain.n:
        raise ValueError(f"body {b} outside -1..{chain.n - 1}")
    return b


def chain_problem_of(dynamicsf, immediate_cost, final_cost):
    """The ChainProblem behind a recognised closure triple, else None: the problem's own
    joint-space costs, or cost_functions.jl's simple costs on the problem's chain."""
    if not isinstance(dynamicsf, ChainDynamics):
        return None
    p = dynamicsf.problem
    if (isinstance(immediate_cost, ChainCost) and isinstance(final_cost, ChainFinalCost)
            and p is immediate_cost.problem is final_cost.problem):
        return p
    from .cost_functions import simple_costs_of
    if simple_costs_of(p, immediate_cost, final_cost) is not None:
        return p
    return None
