"""CPU restatement of the RBD example's dynamics for a fixed-base serial chain —
TEST INFRASTRUCTURE ONLY (the checker of the ILQR_PROBLEM_CHAIN kernels; only
tests/, __graft_entry__.smoke() and bench/tool CPU-baseline legs import it).

Reference: test/RBD_2_link_example/RBD_helper_functions.jl:48-79 wraps
RigidBodyDynamics.jl (not vendored, absent here; RBD.jl's published algorithms:
Featherstone's recursive Newton-Euler for `dynamics_bias`, the mass matrix of
`mass_matrix`) into
    v̇ = M(q) \\ (−dynamics_bias(q, v) + u),  q̇ = v      (:61-66, fixed base: no MRP part)
    x' = RK4(Δt) of [q̇; v̇]                              (:70-78)
and the weighted quadratic costs of :85-116 restricted to the joint coordinates
(`pos = x[1:8]` keeps positions only; the fixed base has no orientation/position
rows). Parity status: RigidBodyDynamics.jl cannot run here — "parity unpinned"
against the reference's executed output; pinned instead by known answers
(tests/test_chain_oracle.py): the 2-DoF arm's closed form M = diag(4, 0.5),
bias = 0 (COMs on the joint origins, isotropic link inertias, zero gravity as the
reference parses it); an independent Jacobian formulation of M
(Σ mJ_vᵀJ_v + J_ωᵀ I J_ω) on the coupled 6-DoF arm; kinetic-energy conservation
of the unforced RK4 rollout; and RNEA(q, v, M⁻¹(τ − b)) = τ.

Every routine is written with scalar-like arithmetic on per-point arrays, so the
same code runs on float64 arrays of shape (P,) (P points at once) and on the
`Jet` forward-mode type below (exact derivatives, what ForwardDiff gives the
reference at src/backward_pass.jl:32-33).
"""
from __future__ import annotations

import numpy as np


class Jet:
    """Forward-mode AD over P points at once: val (P,), der (P, n)."""
    __slots__ = ("val", "der")

    def __init__(self, val, der):
        self.val, self.der = val, der

    @staticmethod
    def _vd(o):
        return (o.val, o.der) if isinstance(o, Jet) else (o, None)

    def __add__(self, o):
        v, d = self._vd(o)
        return Jet(self.val + v, self.der if d is None else self.der + d)

    __radd__ = __add__

    def __sub__(self, o):
        v, d = self._vd(o)
        return Jet(self.val - v, self.der if d is None else self.der - d)

    def __rsub__(self, o):
        return Jet(o - self.val, -self.der)

    def __neg__(self):
        return Jet(-self.val, -self.der)

    def __mul__(self, o):
        v, d = self._vd(o)
        if d is None:
            return Jet(self.val * v, self.der * np.asarray(v)[..., None])
        return Jet(self.val * v, self.der * v[:, None] + d * self.val[:, None])

    __rmul__ = __mul__

    def __truediv__(self, o):
        v, d = self._vd(o)
        if d is None:
            return Jet(self.val / v, self.der / np.asarray(v)[..., None])
        q = self.val / v
        return Jet(q, (self.der - d * q[:, None]) / v[:, None])

    def __rtruediv__(self, o):
        q = o / self.val
        return Jet(q, -self.der * (q / self.val)[:, None])


def sin(a):
    return Jet(np.sin(a.val), a.der * np.cos(a.val)[:, None]) if isinstance(a, Jet) else np.sin(a)


def cos(a):
    return Jet(np.cos(a.val), -a.der * np.sin(a.val)[:, None]) if isinstance(a, Jet) else np.cos(a)


# -- 3-vectors as lists of per-point scalars -------------------------------------------
def _cross(a, b):
    return [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]


def _add(a, b):
    return [a[0] + b[0], a[1] + b[1], a[2] + b[2]]


def _sub(a, b):
    return [a[0] - b[0], a[1] - b[1], a[2] - b[2]]


def _scale(a, s):
    return [a[0] * s, a[1] * s, a[2] * s]


def _matvec(M, v):   # constant 3×3 M (nested lists of Python floats)
    return [M[i][0] * v[0] + M[i][1] * v[1] + M[i][2] * v[2] for i in range(3)]


def _matTvec(M, v):
    return [M[0][i] * v[0] + M[1][i] * v[1] + M[2][i] * v[2] for i in range(3)]


def _fl(a):
    """numpy constants → nested lists of Python floats (numpy scalars would wrap Jets
    into object arrays)."""
    return np.asarray(a, dtype=float).tolist()


def _rod(a, c, s, w):
    """Rodrigues: Rot(a, q)·w = c·w + s·(a × w) + (1 − c)(a·w)·a, a constant unit axis."""
    axw = _cross(a, w)
    adw = a[0] * w[0] + a[1] * w[1] + a[2] * w[2]
    k = (1.0 - c) * adw
    return [c * w[i] + s * axw[i] + k * a[i] for i in range(3)]


class ChainModel:
    """Dynamics of a fixed-base chain (ilqr_amd.urdf.Chain)."""

    def __init__(self, chain, dt=0.01):
        self.ch = chain
        self.n = chain.n
        self.dt = dt
        # rotational inertia about the body origin and the first mass moment
        c = chain.com
        self.Io = np.array([chain.Ic[i] + chain.mass[i] * (float(c[i] @ c[i]) * np.eye(3) - np.outer(c[i], c[i]))
                            for i in range(self.n)])
        self.mc = chain.mass[:, None] * c
        self._R0, self._p, self._ax = _fl(chain.R0), _fl(chain.p), _fl(chain.axis)
        self._Io, self._mc, self._m = _fl(self.Io), _fl(self.mc), _fl(chain.mass)
        self._g = _fl(chain.gravity)

    # parent → child (motion) and child → parent (force) coordinate maps of joint i
    def _to_child(self, i, sc, w):
        c, s = sc[i]
        return _rod(self._ax[i], c, -s, _matTvec(self._R0[i], w))

    def _to_parent(self, i, sc, w):
        c, s = sc[i]
        return _matvec(self._R0[i], _rod(self._ax[i], c, s, w))

    def rnea(self, q, qd, qdd, gravity=True, sc=None):
        """Recursive Newton-Euler inverse dynamics τ = M(q) q̈ + b(q, q̇) (b includes
        gravity when `gravity`); q, qd, qdd are lists of n per-point scalars (qd may
        be None = zero velocity)."""
        n, ch = self.n, self.ch
        if sc is None:
            sc = [(cos(q[i]), sin(q[i])) for i in range(n)]
        zero = 0.0 * qdd[0]
        w, v = [zero] * 3, [zero] * 3
        al = [zero] * 3
        ac = _scale(self._g, -1.0) if gravity else [zero] * 3  # fictitious base accel
        ac = [zero + a for a in ac]
        f_n, f_f = [], []
        for i in range(n):
            a = self._ax[i]
            r = self._p[i]
            # spatial velocity (ω, v_O) of body i in its own frame
            wi = self._to_child(i, sc, w)
            vi = self._to_child(i, sc, _sub(v, _cross(r, w)))
            ali = self._to_child(i, sc, al)
            aci = self._to_child(i, sc, _sub(ac, _cross(r, al)))
            if qd is not None:
                sq = _scale(list(a), qd[i])           # S q̇ (motion subspace · rate)
                wi = _add(wi, sq)
                ali = _add(ali, _cross(wi, sq))       # v ×m (S q̇): angular part
                aci = _add(aci, _cross(vi, sq))       #             linear part
            ali = _add(ali, _scale(list(a), qdd[i]))
            # f = I a + v ×f (I v);  I·(α, a) = (Io α + mc × a, m a − mc × α)
            Io, mc, m = self._Io[i], self._mc[i], self._m[i]
            fn = _add(_matvec(Io, ali), _cross(mc, aci))
            ff = _sub(_scale(aci, m), _cross(mc, ali))
            if qd is not None:
                hn = _add(_matvec(Io, wi), _cross(mc, vi))
                hf = _sub(_scale(vi, m), _cross(mc, wi))
                fn = _add(fn, _add(_cross(wi, hn), _cross(vi, hf)))
                ff = _add(ff, _cross(wi, hf))
            f_n.append(fn)
            f_f.append(ff)
            w, v, al, ac = wi, vi, ali, aci
        tau = [None] * n
        for i in range(n - 1, -1, -1):
            a = self._ax[i]
            tau[i] = a[0] * f_n[i][0] + a[1] * f_n[i][1] + a[2] * f_n[i][2]
            if i > 0:
                pf = self._to_parent(i, sc, f_f[i])
                pn = _add(self._to_parent(i, sc, f_n[i]), _cross(self._p[i], pf))
                f_n[i - 1] = _add(f_n[i - 1], pn)
                f_f[i - 1] = _add(f_f[i - 1], pf)
        return tau

    def mass_matrix(self, q, sc=None):
        """M(q) column by column: M[:, k] = RNEA(q, 0, e_k) without gravity."""
        n = self.n
        if sc is None:
            sc = [(cos(q[i]), sin(q[i])) for i in range(n)]
        zero = 0.0 * q[0]
        cols = []
        for k in range(n):
            e = [zero + (1.0 if j == k else 0.0) for j in range(n)]
            cols.append(self.rnea(q, None, e, gravity=False, sc=sc))
        return [[cols[k][i] for k in range(n)] for i in range(n)]   # M[i][k]

    def dynamics_bias(self, q, qd, sc=None):
        zero = 0.0 * q[0]
        return self.rnea(q, qd, [zero] * self.n, gravity=True, sc=sc)

    @staticmethod
    def _solve(M, b):
        """Gaussian elimination without pivoting (M is SPD)."""
        n = len(b)
        M = [row[:] for row in M]
        b = b[:]
        for k in range(n):
            inv = 1.0 / M[k][k]
            for i in range(k + 1, n):
                l = M[i][k] * inv
                for j in range(k + 1, n):
                    M[i][j] = M[i][j] - l * M[k][j]
                b[i] = b[i] - l * b[k]
        x = [None] * n
        for i in range(n - 1, -1, -1):
            acc = b[i]
            for j in range(i + 1, n):
                acc = acc - M[i][j] * x[j]
            x[i] = acc / M[i][i]
        return x

    def torque(self, u):
        """u (nu entries) → generalized force: nu = n drives every joint, nu = 1 the first only."""
        zero = 0.0 * u[0]
        return [u[i] if i < len(u) else zero for i in range(self.n)]

    def continuous_dynamics(self, x, u):
        """[q̇; v̇] with v̇ = M \\ (−bias + τ) (RBD_helper_functions.jl:61-66)."""
        n = self.n
        q, qd = x[:n], x[n:]
        sc = [(cos(q[i]), sin(q[i])) for i in range(n)]
        M = self.mass_matrix(q, sc)
        b = self.dynamics_bias(q, qd, sc)
        tau = self.torque(u)
        qdd = self._solve(M, [tau[i] - b[i] for i in range(n)])
        return list(qd) + qdd

    def dynamicsf(self, x, u):
        """RK4 (RBD_helper_functions.jl:70-78): x' = x + (k1 + 2k2 + 2k3 + k4)/6."""
        dt = self.dt
        f = self.continuous_dynamics
        k1 = [dt * v for v in f(x, u)]
        k2 = [dt * v for v in f([x[i] + 0.5 * k1[i] for i in range(len(x))], u)]
        k3 = [dt * v for v in f([x[i] + 0.5 * k2[i] for i in range(len(x))], u)]
        k4 = [dt * v for v in f([x[i] + k3[i] for i in range(len(x))], u)]
        return [x[i] + (1.0 / 6.0) * (((k1[i] + 2.0 * k2[i]) + 2.0 * k3[i]) + k4[i]) for i in range(len(x))]

    # -- vectorised front ends over P points --------------------------------------------
    def step(self, X, U):
        """X (P, 2n), U (P, nu) float64 → X' (P, 2n)."""
        out = self.dynamicsf([X[:, i] for i in range(X.shape[1])], [U[:, i] for i in range(U.shape[1])])
        return np.stack(out, axis=1)

    def linearize(self, X, U):
        """Exact Jacobians A (P, nx, nx), B (P, nx, nu) of one RK4 step (forward-mode AD)."""
        P, nx = X.shape
        nu = U.shape[1]
        nd = nx + nu
        xs = [Jet(X[:, i].copy(), np.tile(np.eye(nd)[i], (P, 1))) for i in range(nx)]
        us = [Jet(U[:, i].copy(), np.tile(np.eye(nd)[nx + i], (P, 1))) for i in range(nu)]
        out = self.dynamicsf(xs, us)
        J = np.stack([o.der for o in out], axis=1)  # (P, nx, nd)
        return J[:, :, :nx], J[:, :, nx:]

    def mass_matrix_np(self, q):
        """M for one configuration q (n,), float64."""
        M = self.mass_matrix([np.array([v]) for v in q])
        return np.array([[M[i][k][0] for k in range(self.n)] for i in range(self.n)])

    def bias_np(self, q, qd):
        b = self.dynamics_bias([np.array([v]) for v in q], [np.array([v]) for v in qd])
        return np.array([v[0] for v in b])


# -- independent formulation for the known-answer tests ---------------------------------
def world_frames(chain, q):
    """World-frame forward kinematics, root to tip: (origin, world axis, orientation) of
    every body frame (matrix exponential of the joint axis; independent of the RNEA)."""
    R = np.eye(3)
    o = np.zeros(3)
    frames = []
    for i in range(chain.n):
        o = o + R @ chain.p[i]
        Rj = R @ chain.R0[i]
        a_w = Rj @ chain.axis[i]
        K = np.array([[0, -chain.axis[i][2], chain.axis[i][1]], [chain.axis[i][2], 0, -chain.axis[i][0]],
                      [-chain.axis[i][1], chain.axis[i][0], 0]])
        Rq = np.eye(3) + np.sin(q[i]) * K + (1 - np.cos(q[i])) * K @ K
        R = Rj @ Rq
        frames.append((o.copy(), a_w, R.copy()))
    return frames


def mass_matrix_jacobian(chain, q):
    """M(q) = Σ_i m_i J_vᵢᵀ J_vᵢ + J_ωᵢᵀ (R_i I_ci R_iᵀ) J_ωᵢ from world-frame forward
    kinematics (a formulation independent of the RNEA above)."""
    n = chain.n
    frames = world_frames(chain, q)
    M = np.zeros((n, n))
    for i in range(n):
        oi, _, Ri = frames[i]
        ci = oi + Ri @ chain.com[i]
        Jv = np.zeros((3, n))
        Jw = np.zeros((3, n))
        for j in range(i + 1):
            oj, aj, _ = frames[j]
            Jw[:, j] = aj
            Jv[:, j] = np.cross(aj, ci - oj)
        Iw = Ri @ chain.Ic[i] @ Ri.T
        M += chain.mass[i] * Jv.T @ Jv + Jw.T @ Iw @ Jw
    return M


# -- the reference's RBD costs on the joint coordinates ---------------------------------
class ChainCost:
    """ℓ(x, u) = Σ qwᵢ(θ*ᵢ − θᵢ)² + Σ rwₖ uₖ²  and  ℓ_f(x) = Σ qfwᵢ(θ*ᵢ − θᵢ)²
    (RBD_helper_functions.jl:85-116 on the joint rows: Q = 10·diag(jo_cost = 10),
    R = diag(jo_tor_cost = 10), final Q = 1e5·diag(10)). Analytic derivatives
    (`quad`, `fquad`) are what ForwardDiff returns for these quadratics."""

    def __init__(self, target, qw, rw, qfw):
        self.t = np.asarray(target, float)
        self.qw, self.rw, self.qfw = (np.asarray(v, float) for v in (qw, rw, qfw))
        self.n = len(self.t)

    def immediate(self, x, u):
        """Generic in the element type (floats or oracle.dual duals), like the reference."""
        acc = 0.0
        for i in range(self.n):
            e = float(self.t[i]) - x[i]
            acc = acc + float(self.qw[i]) * e * e
        for k in range(len(u)):
            acc = acc + float(self.rw[k]) * u[k] * u[k]
        return acc

    def final(self, x):
        acc = 0.0
        for i in range(self.n):
            e = float(self.t[i]) - x[i]
            acc = acc + float(self.qfw[i]) * e * e
        return acc

    def quad(self, x, u):
        n, nx, nu = self.n, len(x), len(u)
        e = self.t - np.asarray(x[:n], float)
        qv = np.zeros(nx)
        qv[:n] = -2 * self.qw * e
        Q = np.zeros((nx, nx))
        Q[:n, :n] = np.diag(2 * self.qw)
        r = 2 * self.rw[:nu] * np.asarray(u, float)
        R = np.diag(2 * self.rw[:nu])
        return float(self.immediate(x, u)), qv, r, Q, np.zeros((nu, nx)), R

    def fquad(self, x):
        n, nx = self.n, len(x)
        e = self.t - np.asarray(x[:n], float)
        g = np.zeros(nx)
        g[:n] = -2 * self.qfw * e
        H = np.zeros((nx, nx))
        H[:n, :n] = np.diag(2 * self.qfw)
        return float(self.final(x)), g, H


def chain_closures(model: ChainModel, cost: ChainCost):
    """(dynamicsf, immediate_cost, final_cost) for oracle.ilqr_oracle, with exact
    Jacobians attached (`.jac`, forward-mode AD of the RK4 step)."""

    class Dyn:
        def __call__(self, x, u):
            return model.step(np.asarray(x, float)[None], np.asarray(u, float)[None])[0]

        def jac(self, x, u):
            A, B = model.linearize(np.asarray(x, float)[None], np.asarray(u, float)[None])
            return A[0], B[0]

    class Cost:
        def __call__(self, x, u):
            return cost.immediate(x, u)

        def quad(self, x, u):
            return cost.quad(x, u)

    class Final:
        def __call__(self, x):
            return cost.final(x)

        def fquad(self, x):
            return cost.fquad(x)

    return Dyn(), Cost(), Final()
