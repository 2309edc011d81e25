"""CPU restatement of aabouman/iLQR.jl's hot path — TEST INFRASTRUCTURE ONLY.

This is the checker the HIP path is compared against, never the thing measured
or shipped. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import it.

Parity status: the reference is pure Julia and no Julia toolchain exists in
this container or on the GPU box, so the reference cannot be run here. Its one
recorded EXECUTED output is pinned instead: the animations
test/2_link_example/animate_2_link.jl saved when its authors ran it (shipped in
test/2_link_example/figures/, 91 frames of the T = 900 2-link fit each; frames
extracted into tests/golden/reference_gifs.npz by tests/golden/make_gif_golden.py).
The C restatement's fit of that workload reproduces every frame of the shipped
script's GIF within a third of a pixel (elbow and tool ≤ 0.0035 data units,
tests/test_reference_gifs.py), and this Python restatement equals the C one on the
same workload (1e-9). What the pin resolves (test_gif_pin_sensitivity): the script's
CoriolisMatrix quirk IS visible — the textbook Coriolis matrix misses the frames by
0.039 data units (≈3.5 px, 4× the tolerance); fit's return of the iterate before the
update that met tol is NOT — the other choice moves the frames by < 10⁻⁵, so that quirk
rests on the restatement's algebra and the unit tests alone. Beyond that the restatements are pinned by known-answer tests
derived from the reference's own tests and algebra (tests/test_oracle.py): the
repaired linear-f linearisation property of test/test_linearize_dynamics.jl:24-25,
the LQ closed-form (KKT) fixed point, the 2-link IK constants of
test/2_link_example/2_link_helper_functions.jl:16-26 and the convergence property
`final_cost(x̄_N) < 0.01` of test/test_iLQR.jl:19. The LQ family (the headline) has
no executed reference output anywhere: there the pin is the algebra (KKT) only.

Layout: one trajectory per call, row-per-timestep exactly like the reference:
x is (N, n), u is (T, m) with N = T + 1, δu is (T, m), K is (T, m, n).
Derivatives come from `oracle.dual` (a restatement of ForwardDiff) unless the
closure carries exact analytic derivatives (`.jac`, `.quad`, `.fquad`
attributes set by `lq_closures`), which tests cross-check against the AD.
"""
from __future__ import annotations

import math

import numpy as np

from . import dual

REG_MU = 0.01  # src/backward_pass.jl:214 (fixed regulariser, no adaptation)


# --------------------------------------------------------------------------------
# L1 local models
# --------------------------------------------------------------------------------
def linearize_dynamics(x, u, dynamicsf):
    """src/backward_pass.jl:25-40 — A = ∂f/∂x, B = ∂f/∂u (two ForwardDiff.jacobian)."""
    if hasattr(dynamicsf, "jac"):
        return dynamicsf.jac(x, u)
    A = dual.jacobian(lambda xx: dynamicsf(xx, u), x)
    B = dual.jacobian(lambda uu: dynamicsf(x, uu), u)
    return A, B


def immediate_cost_quadratization(x, u, immediate_cost):
    """src/backward_pass.jl:81-109 — (q, 𝐪, 𝐫, 𝐐, 𝐏 (m×n), 𝐑)."""
    if hasattr(immediate_cost, "quad"):
        return immediate_cost.quad(x, u)
    dLdx = lambda xx, uu: dual.gradient(lambda z: immediate_cost(z, uu), xx)  # :95
    dLdu = lambda xx, uu: dual.gradient(lambda z: immediate_cost(xx, z), uu)  # :96
    q = immediate_cost(x, u)                                                    # :101
    qv = dLdx(x, u)                                                             # :102
    r = dLdu(x, u)                                                              # :103
    Q = dual.hessian(lambda z: immediate_cost(z, u), x)                         # :97,104
    P = dual.jacobian(lambda z: dLdu(z, u), x)                                  # :98,105
    R = dual.hessian(lambda z: immediate_cost(x, z), u)                         # :99,106
    return float(q), qv, r, Q, P, R


def final_cost_quadratization(x, final_cost):
    """src/backward_pass.jl:134-153 — (ℓ_f, ∇ℓ_f, ∇²ℓ_f) at x_N."""
    if hasattr(final_cost, "fquad"):
        return final_cost.fquad(x)
    return (float(final_cost(x)), dual.gradient(final_cost, x), dual.hessian(final_cost, x))


# --------------------------------------------------------------------------------
# L2 Riccati step algebra
# --------------------------------------------------------------------------------
def optimal_controller_param(A, B, r, P, R, s, S):
    """src/backward_pass.jl:177-186."""
    g = r + B.T @ s                  # :181
    G = P + (B.T @ S) @ A            # :182
    H = R + (B.T @ S) @ B            # :183
    return g, G, H


def feedback_parameters(g, G, H, mu=REG_MU):
    """src/backward_pass.jl:207-218 — H_reg = H + 0.01 I; δu = -H_reg\\g; K = -H_reg\\G.
    Julia's `\\` factorises (Cholesky / LU with partial pivoting); numpy's
    LAPACK gesv is LU with partial pivoting — equal up to rounding."""
    n = H.shape[0]
    H_reg = H + mu * np.eye(n)       # :214
    du = -np.linalg.solve(H_reg, g)  # :215
    K = -np.linalg.solve(H_reg, G)   # :216
    return du, K


def step_back(A, q, qv, Q, g, G, H, du, K, s_next, sv_next, S_next):
    """src/backward_pass.jl:262-273 — uses the UNregularised H."""
    s = q + s_next + 0.5 * du @ H @ du + du @ g                                    # :268
    sv = qv + A.T @ sv_next + K.T @ H @ du + K.T @ g + G.T @ du                   # :269
    S = Q + A.T @ S_next @ A + K.T @ H @ K + K.T @ G + G.T @ K                     # :270
    return s, sv, S


# --------------------------------------------------------------------------------
# L3 passes
# --------------------------------------------------------------------------------
def backward_pass(x, u, dynamicsf, immediate_cost, final_cost, mu=REG_MU, symmetrize=False):
    """src/backward_pass.jl:324-357 — returns (δu (T×m), K (T×m×n)).

    symmetrize=False is the literal reference. symmetrize=True replaces 𝐒 by
    (𝐒+𝐒ᵀ)/2 after every step_back — the identity in exact arithmetic. It exists
    because the literal update 𝐒 = 𝐐 + AᵀSA + KᵀHK + KᵀG + GᵀK (:270) amplifies
    the rounding asymmetry of 𝐒 geometrically (E ← AᵀEA + (BK)ᵀE(BK)); on the
    headline quadrotor instances it reaches O(1) after ~32 of 100 steps and H
    turns indefinite. The device path is symmetric by
    construction and is checked against symmetrize=True where the literal
    recursion diverges."""
    N, n = x.shape
    M, m = u.shape
    assert N == M + 1                                                               # :329
    dus = np.zeros((N - 1, m))                                                      # :332
    Ks = np.zeros((N - 1, m, n))                                                    # :333
    qn, qvn, Qn = final_cost_quadratization(x[N - 1], final_cost)                   # :335
    s_next, sv_next, S_next = qn, qvn, Qn                                           # :336
    for i in range(N - 2, -1, -1):                                                  # :339
        A, B = linearize_dynamics(x[i], u[i], dynamicsf)                            # :340
        q, qv, r, Q, P, R = immediate_cost_quadratization(x[i], u[i], immediate_cost)  # :341
        g, G, H = optimal_controller_param(A, B, r, P, R, sv_next, S_next)          # :342
        du, K = feedback_parameters(g, G, H, mu)                                    # :343
        dus[i] = du                                                                 # :345
        Ks[i] = K                                                                   # :346
        s_next, sv_next, S_next = step_back(A, q, qv, Q, g, G, H, du, K,
                                            s_next, sv_next, S_next)                # :348-350
        if symmetrize:
            S_next = 0.5 * (S_next + S_next.T)
    assert not np.isnan(dus).any()                                                  # :353
    assert not np.isnan(Ks).any()                                                   # :354
    return dus, Ks


def total_cost_generator(x_traj, immediate_cost, final_cost):
    """src/forward_pass.jl:182-196 — Σ_i ℓ(x̄ᵢ − x_trajᵢ, ūᵢ) + ℓ_f(x̄_N), sequential sum."""
    def total_cost(xb, ub):
        N = ub.shape[0]
        acc = 0.0
        for i in range(N):
            acc += float(immediate_cost(xb[i] - x_traj[i], ub[i]))
        acc += float(final_cost(xb[-1]))   # raw x̄_N, never offset by x_traj (:192)
        return acc
    return total_cost


class LineSearchExhausted(RuntimeError):
    """The reference's line search (src/forward_pass.jl:70-87) is unbounded; the
    oracle caps it so a test cannot spin forever."""


def forward_pass(x, u, x_traj, dus, Ks, prev_cost, dynamicsf, immediate_cost, final_cost,
                 max_trials=None, alpha0=1.0, shrink=0.5, stats=None):
    """src/forward_pass.jl:55-93 — rollout with α-halving; α scales δu only."""
    M, m = u.shape
    N, n = x.shape
    assert N == M + 1                                                  # :62
    xb = np.zeros((N, n))
    ub = np.zeros((N - 1, m))
    xb[0] = x[0]                                                       # :65
    alpha = alpha0                                                     # :66
    total_cost = total_cost_generator(x_traj, immediate_cost, final_cost)
    trials = 0
    while True:                                                        # :70
        trials += 1
        for k in range(N - 1):                                         # :71
            dx = xb[k] - x[k]                                          # :72
            ub[k] = u[k] + alpha * dus[k] + Ks[k] @ dx                 # :73
            xb[k + 1] = np.asarray(dynamicsf(xb[k], ub[k]), dtype=float)  # :74
        new_cost = total_cost(xb, ub)                                  # :76
        dcost = prev_cost - new_cost                                   # :77
        if dcost > 0:                                                  # :79
            break
        alpha *= shrink                                                # :82
        if max_trials is not None and trials >= max_trials:
            raise LineSearchExhausted(f"no decrease after {trials} trials")
    if stats is not None:
        stats["trials"] = trials
        stats["alpha"] = alpha
    assert not np.isnan(ub).any()                                      # :89
    assert not np.isnan(xb).any()                                      # :90
    return xb, ub, new_cost


# --------------------------------------------------------------------------------
# L4 driver
# --------------------------------------------------------------------------------
def fit(x_init, u_init, dynamicsf, immediate_cost, final_cost, x_traj=None,
        max_iter=100, tol=1e-6, max_trials=None, history=None, mu=REG_MU, symmetrize=False):
    """src/forward_pass.jl:148-179.

    Quirks kept: prev_cost starts at Inf (so iteration 1 accepts α=1 whenever
    the cost is finite); the convergence test runs BEFORE the update, so on
    convergence the PREVIOUS iterate is returned (:171-178)."""
    if not isinstance(max_iter, (int, np.integer)):
        raise TypeError("max_iter::Int64")                            # :152
    xi, ui = np.asarray(x_init, float), np.asarray(u_init, float)
    if x_traj is None:
        x_traj = np.zeros_like(xi)                                     # :151
    N, n = xi.shape
    M, m = ui.shape
    assert N == M + 1, "size(x_init)[2] == size(u_init)[1]"            # :156
    prev_cost = math.inf                                               # :159
    for it in range(1, max_iter + 1):                                  # :161
        dus, Ks = backward_pass(xi, ui, dynamicsf, immediate_cost, final_cost, mu,
                                symmetrize)                                    # :162
        st = {}
        xn, un, new_cost = forward_pass(xi, ui, x_traj, dus, Ks, prev_cost, dynamicsf,
                                        immediate_cost, final_cost, max_trials=max_trials,
                                        stats=st)                      # :163-166
        assert prev_cost > new_cost                                    # :168
        prev_cost = new_cost
        du2 = float(np.sum((un - ui) ** 2))
        if history is not None:
            history.append({"iter": it, "cost": new_cost, "trials": st["trials"], "du2": du2})
        if du2 <= tol:                                                 # :171
            break
        xi, ui = xn, un                                                # :174-175
    return xi, ui                                                      # :178


# --------------------------------------------------------------------------------
# Problem closures used by the parity tests
# --------------------------------------------------------------------------------
def lq_closures(A, B, Q, R, Qf):
    """The headline LQ problem expressed through the reference's callback API
    (SURVEY.md §8d): f(x,u) = A x + B u, ℓ(x,u) = xᵀQx + uᵀRu, ℓ_f(x) = xᵀQf x.
    The closures work on duals too; `.jac/.quad/.fquad` give the exact
    derivatives ForwardDiff would return (linear/quadratic functions)."""
    A, B, Q, R, Qf = (np.asarray(a, float) for a in (A, B, Q, R, Qf))
    Qs, Rs, Qfs = Q + Q.T, R + R.T, Qf + Qf.T
    n, m = B.shape

    def dynamicsf(x, u):
        return A @ x + B @ u

    def immediate_cost(x, u):
        return x @ (Q @ x) + u @ (R @ u)

    def final_cost(x):
        return x @ (Qf @ x)

    dynamicsf.jac = lambda x, u: (A.copy(), B.copy())
    immediate_cost.quad = lambda x, u: (float(immediate_cost(x, u)), Qs @ x, Rs @ u,
                                        Qs.copy(), np.zeros((m, n)), Rs.copy())
    final_cost.fquad = lambda x: (float(final_cost(x)), Qfs @ x, Qfs.copy())
    return dynamicsf, immediate_cost, final_cost


def lq_kkt_solution(A, B, Q, R, Qf, x0, T):
    """Exact minimiser of Σ_t (x_tᵀQx_t + u_tᵀRu_t) + x_Tᵀ Qf x_T s.t. x_{t+1}=Ax_t+Bu_t,
    by eliminating the states (condensed QP, one dense solve). iLQR's fixed point
    has δu ≡ 0, i.e. ∇_u J = 0, so it equals this solution independent of μ."""
    n, m = B.shape
    # x_t = A^t x0 + Σ_{k<t} A^{t-1-k} B u_k  → X = Φ x0 + Γ U
    Phi = np.zeros(((T + 1) * n, n))
    Gam = np.zeros(((T + 1) * n, T * m))
    P = np.eye(n)
    pw = [np.eye(n)]
    for _ in range(T):
        pw.append(A @ pw[-1])
    for t in range(T + 1):
        Phi[t * n:(t + 1) * n] = pw[t]
        for k in range(t):
            Gam[t * n:(t + 1) * n, k * m:(k + 1) * m] = pw[t - 1 - k] @ B
    Qbig = np.zeros(((T + 1) * n, (T + 1) * n))
    for t in range(T):
        Qbig[t * n:(t + 1) * n, t * n:(t + 1) * n] = Q
    Qbig[T * n:, T * n:] = Qf
    Rbig = np.kron(np.eye(T), R)
    Hs = Gam.T @ (Qbig + Qbig.T) @ Gam + (Rbig + Rbig.T)
    gs = Gam.T @ (Qbig + Qbig.T) @ Phi @ x0
    U = -np.linalg.solve(Hs, gs)
    X = Phi @ x0 + Gam @ U
    del P
    return X.reshape(T + 1, n), U.reshape(T, m)


# -- 2-link arm (test/2_link_example/2_link_helper_functions.jl) ---------------------
class TwoLink:
    """Literal restatement of test/2_link_example/2_link_helper_functions.jl:1-108,
    quirks included (Coriolis `for k in length(θ)` → k=2 only; unused velocity
    penalty). Works on floats and on `oracle.dual` duals."""
    n_links = 2                                                         # :4
    l1 = l2 = math.sqrt(2.0) / 2.0                                      # :5
    r1, r2 = 0.5 * l1, 0.5 * l2                                         # :6
    m1 = m2 = 1.0                                                       # :7
    Iz1 = 1.0 / 12.0 * m1 * l1 ** 2                                     # :8
    Iz2 = 1.0 / 12.0 * m2 * l2 ** 2
    alpha = Iz1 + Iz2 + m1 * r1 ** 2 + m2 * (l1 ** 2 + r2 ** 2)         # :11
    beta = m2 * l1 * r2                                                 # :12
    delta = Iz2 + m2 * r2 ** 2                                          # :13
    dt = 0.01                                                           # :14
    target_tool_loc = (0.6, -0.5)                                       # :16

    @classmethod
    def inverse_kinematics(cls, target):                                # :19-26
        x, y = target
        l1, l2 = cls.l1, cls.l2
        q2 = dual.acos((x ** 2 + y ** 2 - l1 ** 2 - l2 ** 2) / (2 * l1 * l2))
        q1 = math.atan2(y, x) - math.atan2(l2 * math.sin(q2), l1 + l2 * math.cos(q2))
        return np.array([q1, q2])

    @classmethod
    def inertia_matrix(cls, th):                                        # :29-33
        a, b, d = cls.alpha, cls.beta, cls.delta
        c2 = dual.cos(th[1])
        M = np.empty((2, 2), dtype=object)
        M[0, 0] = a + 2 * b * c2
        M[0, 1] = d + b * c2
        M[1, 0] = d + b * c2
        M[1, 1] = d
        return M

    @classmethod
    def coriolis_matrix(cls, th, thd):                                  # :36-47
        dM = dual.jacobian(cls.inertia_matrix, th)                      # 4×2, vec column-major
        dM = np.asarray(dM, dtype=object).reshape((2, 2, 2), order="F")  # :38 reshape
        C = np.empty((2, 2), dtype=object)
        k = 1  # `for k in length(θ)` iterates only k = length(θ) = 2 (0-based 1)
        for i in range(2):
            for j in range(2):
                C[i, j] = 1 / 2 * (dM[k, i, j] + dM[j, i, k] - dM[i, k, j]) * thd[k]
        return C

    @classmethod
    def continuous_dynamics(cls, state, wrench):                        # :51-69
        th, thd = state[0:2], state[2:4]
        M = cls.inertia_matrix(th)
        C = cls.coriolis_matrix(th, thd)
        Minv = _inv2(M)
        MC = _solve2(M, C)
        acc = -(MC @ thd) + Minv @ wrench
        return np.array([thd[0], thd[1], acc[0], acc[1]], dtype=object)

    @classmethod
    def dynamicsf(cls, x, u):                                           # :49-79 (RK4)
        dt = cls.dt
        x = np.asarray(x, dtype=object)
        k1 = dt * cls.continuous_dynamics(x, u)
        k2 = dt * cls.continuous_dynamics(x + k1 / 2, u)
        k3 = dt * cls.continuous_dynamics(x + k2 / 2, u)
        k4 = dt * cls.continuous_dynamics(x + k3, u)
        out = x + (1 / 6) * (k1 + 2 * k2 + 2 * k3 + k4)
        if not any(isinstance(v, dual.Dual) for v in out):
            return out.astype(float)
        return out

    @classmethod
    def dynamicsf_nu1(cls, x, u):
        """dynamicsf₁(x, u) = dynamicsf(x, [u₁, 0]): the build-defined nu = 1 variant
        (BASELINE.json configs 1-2; the reference's own dynamicsf needs nu = 2,
        :63-65). Not reference-pinned."""
        return cls.dynamicsf(x, np.array([u[0], 0.0], dtype=object))

    @classmethod
    def immediate_cost(cls, x, u):                                      # :82-97
        tgt = cls.inverse_kinematics(cls.target_tool_loc)
        e = (tgt[0] - x[0]) ** 2 + (tgt[1] - x[1]) ** 2
        torque = sum(ui ** 2 for ui in u)
        return e * 1.0 + torque * 1.0

    @classmethod
    def final_cost(cls, x):                                             # :100-108
        tgt = cls.inverse_kinematics(cls.target_tool_loc)
        e = (tgt[0] - x[0]) ** 2 + (tgt[1] - x[1]) ** 2
        return e * 1.0


def _inv2(M):
    a, b, c, d = M[0, 0], M[0, 1], M[1, 0], M[1, 1]
    det = a * d - b * c
    out = np.empty((2, 2), dtype=object)
    out[0, 0], out[0, 1], out[1, 0], out[1, 1] = d / det, -b / det, -c / det, a / det
    return out


def _solve2(M, C):
    return _inv2(M) @ C


def rollout(x0, u, dynamicsf):
    """Open-loop rollout used to build a dynamically consistent x_init
    (test/2_link_example/animate_2_link.jl:11-16)."""
    T = u.shape[0]
    x = np.zeros((T + 1, len(x0)))
    x[0] = x0
    for t in range(T):
        x[t + 1] = np.asarray(dynamicsf(x[t], u[t]), dtype=float)
    return x
