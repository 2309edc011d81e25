"""Problem definitions for the device path, expressed through the reference's
callback API (dynamicsf(x,u), immediate_cost(x,u), final_cost(x) —
/root/reference/src/backward_pass.jl:11-19,54-70,122-127).

The reference's closures are arbitrary Julia functions; the device path needs
a problem family it has a kernel for. These callables ARE valid reference-style
closures (they evaluate with numpy, so the same objects can be handed to a CPU
implementation) and the device API recognises them and ships their parameters
to the GPU instead of calling them.

Family ILQR_PROBLEM_LQ: f(x,u) = A x + B u, ℓ(x,u) = xᵀQx + uᵀRu, ℓ_f(x) = xᵀQf x,
with per-trajectory (batched) A, B, Q, R, Qf.

Family ILQR_PROBLEM_TWO_LINK: the reference's 2-link arm
(test/2_link_example/2_link_helper_functions.jl), fixed constants, nx=4, nu=2.

`quadrotor_batch` builds the headline benchmark instance: a
hover-linearised quadrotor, per-instance randomised with
numpy.random.default_rng(seed=b).
"""
from __future__ import annotations

import math

import numpy as np


def _like(M, x):
    """M as a tensor on x's device when x is a torch tensor (the callables then also
    serve the generic closure path, which differentiates them with torch.func)."""
    if type(x).__module__.startswith("torch"):
        import torch
        return torch.as_tensor(M, dtype=x.dtype, device=x.device)
    return M


class LinearDynamics:
    """dynamicsf(x, u) = A x + B u.  A: (nx,nx) or (batch,nx,nx); B likewise."""

    def __init__(self, A, B):
        self.A = np.asarray(A, dtype=np.float64)
        self.B = np.asarray(B, dtype=np.float64)

    def __call__(self, x, u):
        if self.A.ndim == 3:
            raise TypeError("batched LinearDynamics: select an instance with .instance(b)")
        return _like(self.A, x) @ x + _like(self.B, x) @ u

    def instance(self, b):
        return LinearDynamics(self.A[b], self.B[b]) if self.A.ndim == 3 else self

    @property
    def nx(self):
        return self.A.shape[-1]

    @property
    def nu(self):
        return self.B.shape[-1]


class QuadraticCost:
    """immediate_cost(x, u) = xᵀ Q x + uᵀ R u."""

    def __init__(self, Q, R):
        self.Q = np.asarray(Q, dtype=np.float64)
        self.R = np.asarray(R, dtype=np.float64)

    def __call__(self, x, u):
        if self.Q.ndim == 3:
            raise TypeError("batched QuadraticCost: select an instance with .instance(b)")
        return x @ (_like(self.Q, x) @ x) + u @ (_like(self.R, x) @ u)

    def instance(self, b):
        return QuadraticCost(self.Q[b], self.R[b]) if self.Q.ndim == 3 else self


class QuadraticFinalCost:
    """final_cost(x) = xᵀ Qf x."""

    def __init__(self, Qf):
        self.Qf = np.asarray(Qf, dtype=np.float64)

    def __call__(self, x):
        if self.Qf.ndim == 3:
            raise TypeError("batched QuadraticFinalCost: select an instance with .instance(b)")
        return x @ (_like(self.Qf, x) @ x)

    def instance(self, b):
        return QuadraticFinalCost(self.Qf[b]) if self.Qf.ndim == 3 else self


class LQBatch:
    """Per-instance LQ data, row-major (batch, …) float64 arrays."""

    def __init__(self, A, B, Q, R, Qf):
        self.A, self.B, self.Q, self.R, self.Qf = (np.ascontiguousarray(a, dtype=np.float64)
                                                   for a in (A, B, Q, R, Qf))
        nb, nx, nu = self.B.shape
        assert self.A.shape == (nb, nx, nx) and self.Q.shape == (nb, nx, nx)
        assert self.R.shape == (nb, nu, nu) and self.Qf.shape == (nb, nx, nx)

    @property
    def batch(self):
        return self.B.shape[0]

    @property
    def nx(self):
        return self.B.shape[1]

    @property
    def nu(self):
        return self.B.shape[2]

    def closures(self):
        """(dynamicsf, immediate_cost, final_cost) — the reference's callback triple."""
        return (LinearDynamics(self.A, self.B), QuadraticCost(self.Q, self.R),
                QuadraticFinalCost(self.Qf))

    def slice(self, lo, hi):
        return LQBatch(self.A[lo:hi], self.B[lo:hi], self.Q[lo:hi], self.R[lo:hi], self.Qf[lo:hi])


def lq_from_closures(dynamicsf, immediate_cost, final_cost, batch):
    """Extract LQ parameters from a recognised callback triple, broadcasting
    unbatched parameters over `batch` trajectories."""
    if not (isinstance(dynamicsf, LinearDynamics) and isinstance(immediate_cost, QuadraticCost)
            and isinstance(final_cost, QuadraticFinalCost)):
        raise NotImplementedError(
            "the MI355X path runs the LQ problem family: pass LinearDynamics, QuadraticCost and "
            "QuadraticFinalCost callables (arbitrary closures have no device kernel)")

    def bc(a, shape):
        a = np.asarray(a, dtype=np.float64)
        return np.broadcast_to(a, (batch,) + shape) if a.ndim == 2 else a

    nx, nu = dynamicsf.B.shape[-2], dynamicsf.B.shape[-1]
    return LQBatch(bc(dynamicsf.A, (nx, nx)), bc(dynamicsf.B, (nx, nu)), bc(immediate_cost.Q, (nx, nx)),
                   bc(immediate_cost.R, (nu, nu)), bc(final_cost.Qf, (nx, nx)))


# -- headline instance: hover-linearised quadrotor -----------------
QUAD_G, QUAD_L, QUAD_C, QUAD_DT = 9.81, 0.175, 0.0245, 0.05


def quadrotor_instance(seed: int, dt: float = QUAD_DT):
    """One randomised instance: returns (A, B, Q, R, Qf, x0).

    State [p(3), φ θ ψ (3), v(3), ω(3)], input = 4 rotor-thrust deviations.
    Continuous: ṗ = v, Θ̇ = ω, v̇ = (g θ, −g φ, Σu/m), ω̇ = J⁻¹ (L(u₂−u₄), L(u₃−u₁), c(u₁−u₂+u₃−u₄));
    forward Euler A = I + dt·A_c, B = dt·B_c. Draw order from default_rng(seed):
    m, Jx, Jy, Jz, q(12), r(4), p0(3), Θ0(3)."""
    rng = np.random.default_rng(seed)
    m = rng.uniform(0.4, 0.6)
    Jx, Jy = rng.uniform(2e-3, 3e-3), rng.uniform(2e-3, 3e-3)
    Jz = rng.uniform(3.5e-3, 4.5e-3)
    q = rng.uniform(0.5, 2.0, 12)
    r = rng.uniform(0.05, 0.2, 4)
    p0 = rng.uniform(-1.0, 1.0, 3)
    th0 = rng.uniform(-0.2, 0.2, 3)
    Ac = np.zeros((12, 12))
    Ac[0:3, 6:9] = np.eye(3)
    Ac[3:6, 9:12] = np.eye(3)
    Ac[6, 4] = QUAD_G      # v̇x =  g θ
    Ac[7, 3] = -QUAD_G     # v̇y = −g φ
    Bc = np.zeros((12, 4))
    Bc[8, :] = 1.0 / m                                        # v̇z = Σu / m
    Bc[9, 1], Bc[9, 3] = QUAD_L / Jx, -QUAD_L / Jx            # L(u₂ − u₄)/Jx
    Bc[10, 2], Bc[10, 0] = QUAD_L / Jy, -QUAD_L / Jy          # L(u₃ − u₁)/Jy
    Bc[11, :] = (QUAD_C / Jz) * np.array([1.0, -1.0, 1.0, -1.0])  # c(u₁−u₂+u₃−u₄)/Jz
    A = np.eye(12) + dt * Ac
    B = dt * Bc
    Q = np.diag(q)
    R = np.diag(r)
    Qf = 10.0 * Q
    x0 = np.concatenate([p0, th0, np.zeros(6)])
    return A, B, Q, R, Qf, x0


def quadrotor_batch(batch: int, T: int = 100, seed0: int = 0):
    """Headline workload: `batch` instances with seeds seed0 .. seed0+batch-1.
    Returns (LQBatch, x_init (batch,T+1,12), u_init (batch,T,4)); u_init = 0 and
    x_init is its rollout (dynamically consistent, like animate_2_link.jl:11-16)."""
    A = np.empty((batch, 12, 12))
    B = np.empty((batch, 12, 4))
    Q = np.empty((batch, 12, 12))
    R = np.empty((batch, 4, 4))
    Qf = np.empty((batch, 12, 12))
    x = np.empty((batch, T + 1, 12))
    for i in range(batch):
        A[i], B[i], Q[i], R[i], Qf[i], x[i, 0] = quadrotor_instance(seed0 + i)
    u = np.zeros((batch, T, 4))
    for t in range(T):
        x[:, t + 1] = np.einsum("bij,bj->bi", A, x[:, t])
    return LQBatch(A, B, Q, R, Qf), x, u


def random_lq_batch(batch: int, nx: int, nu: int, T: int, seed: int = 0, dense: bool = True):
    """Dense random LQ instances (stable-ish A, SPD Q/R) for parity tests beyond
    the quadrotor structure; u_init random, x_init its rollout."""
    rng = np.random.default_rng(seed)
    A = np.eye(nx) + 0.05 * rng.standard_normal((batch, nx, nx))
    B = 0.2 * rng.standard_normal((batch, nx, nu))
    if dense:
        Mq = rng.standard_normal((batch, nx, nx))
        Q = 0.1 * np.einsum("bij,bkj->bik", Mq, Mq) / nx + np.eye(nx) * rng.uniform(0.5, 1.5, (batch, 1, 1))
        Mr = rng.standard_normal((batch, nu, nu))
        R = 0.05 * np.einsum("bij,bkj->bik", Mr, Mr) / nu + np.eye(nu) * rng.uniform(0.05, 0.2, (batch, 1, 1))
    else:
        Q = np.einsum("bi,ij->bij", rng.uniform(0.5, 2.0, (batch, nx)), np.eye(nx))
        R = np.einsum("bi,ij->bij", rng.uniform(0.05, 0.2, (batch, nu)), np.eye(nu))
    Qf = 5.0 * Q
    x = np.empty((batch, T + 1, nx))
    x[:, 0] = rng.uniform(-1, 1, (batch, nx))
    u = 0.1 * rng.standard_normal((batch, T, nu))
    for t in range(T):
        x[:, t + 1] = np.einsum("bij,bj->bi", A, x[:, t]) + np.einsum("bij,bj->bi", B, u[:, t])
    return LQBatch(A, B, Q, R, Qf), x, u


# -- family ILQR_PROBLEM_TWO_LINK: the reference's 2-link arm ---------------------
class TwoLinkArm:
    """Constants of test/2_link_example/2_link_helper_functions.jl:4-26 (same
    expression order as the script). The device kernels compute the same numbers
    on the host side of the C ABI; they are repeated here for host-side use."""
    n_links = 2
    l1 = l2 = math.sqrt(2.0) / 2.0
    r1, r2 = 0.5 * l1, 0.5 * l2
    m1 = m2 = 1.0
    Iz1 = 1.0 / 12.0 * m1 * l1 ** 2
    Iz2 = 1.0 / 12.0 * m2 * l2 ** 2
    alpha = Iz1 + Iz2 + m1 * r1 ** 2 + m2 * (l1 ** 2 + r2 ** 2)
    beta = m2 * l1 * r2
    delta = Iz2 + m2 * r2 ** 2
    dt = 0.01
    target_tool_loc = (0.6, -0.5)
    nx, nu = 4, 2

    @classmethod
    def inverse_kinematics(cls, target=None):
        """InverseKinematics (:19-26) → θ* (2,)."""
        x, y = cls.target_tool_loc if target is None else target
        q2 = math.acos((x ** 2 + y ** 2 - cls.l1 ** 2 - cls.l2 ** 2) / (2 * cls.l1 * cls.l2))
        q1 = math.atan2(y, x) - math.atan2(cls.l2 * math.sin(q2), cls.l1 + cls.l2 * math.cos(q2))
        return np.array([q1, q2])


class TwoLinkDynamics:
    """dynamicsf(x, u) of the 2-link arm (:49-79): one RK4 step of
    [θ̇; −(M\\C)θ̇ + M⁻¹u], with the script's CoriolisMatrix (k = 2 term only).
    Host evaluation (float64 numpy) for callers that roll the model out on the
    CPU; the device path never calls it — it runs its own kernel functor."""
    nx, nu = 4, 2

    @staticmethod
    def _f(x, u):
        P = TwoLinkArm
        s2, c2 = math.sin(x[1]), math.cos(x[1])
        m00 = P.alpha + 2 * P.beta * c2
        m01 = P.delta + P.beta * c2
        dm00, dm01 = 2 * P.beta * -s2, P.beta * -s2
        C = np.array([[0.5 * dm00 * x[3], 0.5 * dm01 * x[3]], [0.5 * dm01 * x[3], 0.0]])
        M = np.array([[m00, m01], [m01, P.delta]])
        acc = -np.linalg.solve(M, C) @ x[2:4] + np.linalg.solve(M, np.asarray(u, float))
        return np.array([x[2], x[3], acc[0], acc[1]])

    def __call__(self, x, u):
        x = np.asarray(x, dtype=np.float64)
        dt = TwoLinkArm.dt
        k1 = dt * self._f(x, u)
        k2 = dt * self._f(x + k1 / 2, u)
        k3 = dt * self._f(x + k2 / 2, u)
        k4 = dt * self._f(x + k3, u)
        return x + (1 / 6) * (k1 + 2 * k2 + 2 * k3 + k4)


class TwoLinkDynamicsNu1(TwoLinkDynamics):
    """dynamicsf₁(x, u) = dynamicsf(x, [u₁, 0]) — the nu = 1 variant of the 2-link arm
    that BASELINE.json's configs 1-2 name. Build-defined: the reference
    multiplies inv(M) (2×2) by u (2_link_helper_functions.jl:63-65), so its own
    dynamicsf needs nu = 2; only joint 1 is driven here. Not reference-pinned."""
    nu = 1

    def __call__(self, x, u):
        u = np.asarray(u, dtype=np.float64).reshape(-1)
        return super().__call__(x, np.array([u[0], 0.0]))


class TwoLinkCost:
    """immediate_cost(x, u) = |θ* − θ|² + |u|² (:82-97; the velocity penalty is dead code)."""

    def __call__(self, x, u):
        e = TwoLinkArm.inverse_kinematics() - np.asarray(x[:2], float)
        return float(np.sum(e ** 2) * 1.0 + np.sum(np.asarray(u, float) ** 2) * 1.0)


class TwoLinkFinalCost:
    """final_cost(x) = |θ* − θ|² (:100-108)."""

    def __call__(self, x):
        e = TwoLinkArm.inverse_kinematics() - np.asarray(x[:2], float)
        return float(np.sum(e ** 2) * 1.0)


def two_link_closures(nu: int = 2):
    """(dynamicsf, immediate_cost, final_cost) of test/2_link_example; nu = 1 gives the
    build-defined single-torque variant (TwoLinkDynamicsNu1)."""
    if nu not in (1, 2):
        raise ValueError("the 2-link arm takes nu = 2 (reference) or 1 (joint 1 driven)")
    return (TwoLinkDynamics() if nu == 2 else TwoLinkDynamicsNu1()), TwoLinkCost(), TwoLinkFinalCost()


def is_two_link(dynamicsf, immediate_cost, final_cost) -> bool:
    return (isinstance(dynamicsf, TwoLinkDynamics) and isinstance(immediate_cost, TwoLinkCost)
            and isinstance(final_cost, TwoLinkFinalCost))


def two_link_initial_states(batch: int, seed0: int = 0):
    """Config 2's x₀ batch: x₀[b] = rand(4) from numpy.random.default_rng(seed0 + b)
    (test_iLQR.jl:8 draws rand(4) unseeded; SURVEY.md §8 fixes the seeds)."""
    return np.stack([np.random.default_rng(seed0 + b).random(4) for b in range(batch)])
