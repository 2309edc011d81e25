"""Batched CPU restatement of fit for ARBITRARY closures — TEST INFRASTRUCTURE ONLY.

The checker of the generic-closure path (ilqr_amd.api._fit_closures: derivative tiles
→ ilqr_backward_tiles → rollout of the user's dynamics) at sizes the per-trajectory
oracle (ilqr_oracle.fit on oracle.dual scalars) cannot reach in seconds — the
reference's RBD caller is nx = 16, nu = 8, T = 1000
(test/RBD_2_link_example/animate_RBD_2_link.jl:8,19-20,31-32). Same algorithm, same
quirks, batched over trajectories:

  fit            src/forward_pass.jl:148-179   prev_cost = Inf (:159), the convergence
                                               test before the update (:171-178)
  backward_pass  src/backward_pass.jl:324-357  derivative tiles along (x, u) —
                                               linearize_dynamics (:25-40) by the
                                               array-valued forward-mode AD of
                                               oracle.jet (ForwardDiff's algorithm) —
                                               then the C restatement's recursion
                                               (cref.tiles_backward, symmetrised S:
                                               DESIGN.md §3)
  forward_pass   src/forward_pass.jl:55-93     rollout of the numpy closure, α
                                               halving per trajectory, capped at
                                               max_trials (the reference is unbounded)
  total_cost     src/forward_pass.jl:182-196   sequential sum over t from 0.

It is pinned to the per-trajectory restatement (ilqr_oracle.fit) on a small problem by
tests/test_closures.py. Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import anything under oracle/.
"""
from __future__ import annotations

import numpy as np

from . import cref, dual, jet


def dual_quads(immediate_cost, final_cost):
    """Cost quadratizations (backward_pass.jl:81-109, :134-153) by oracle.dual, point
    by point — for small cases and closures written on scalars."""
    def quad(x, u):
        P, nx = x.shape
        nu = u.shape[1]
        lx, lu = np.zeros((P, nx)), np.zeros((P, nu))
        lxx, lux, luu = np.zeros((P, nx, nx)), np.zeros((P, nu, nx)), np.zeros((P, nu, nu))
        for p in range(P):
            xi, ui = x[p], u[p]
            dLdu = lambda z, v: dual.gradient(lambda w: immediate_cost(z, w), v)  # noqa: E731
            lx[p] = dual.gradient(lambda z: immediate_cost(z, ui), xi)                  # :95
            lu[p] = dLdu(xi, ui)                                                         # :96
            lxx[p] = dual.hessian(lambda z: immediate_cost(z, ui), xi)                   # :97
            lux[p] = dual.jacobian(lambda z: dLdu(z, ui), xi)                            # :98
            luu[p] = dual.hessian(lambda v: immediate_cost(xi, v), ui)                   # :99
        return lx, lu, lxx, lux, luu

    def fquad(xN):
        return (np.stack([dual.gradient(final_cost, x) for x in xN]),                   # :142
                np.stack([dual.hessian(final_cost, x) for x in xN]))                    # :143
    return quad, fquad


def derivative_tiles(x, u, dynamicsf, quad, fquad):
    """ilqr_tiles along (x (B, T+1, nx), u (B, T, nu)): A, B by oracle.jet at all B·T
    points in one evaluation of the closure; the cost pieces from quad / fquad."""
    nb, N, nx = x.shape
    T, nu = u.shape[1], u.shape[2]
    xs, us = x[:, :T].reshape(-1, nx), u.reshape(-1, nu)
    A, Bm = jet.jacobians(dynamicsf, xs, us)                          # :32-33
    lx, lu, lxx, lux, luu = quad(xs, us)                               # :95-99
    lfx, lfxx = fquad(x[:, T])                                         # :142-143
    r = lambda a, *s: np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape((nb,) + s))  # noqa: E731
    return {"A": r(A, T, nx, nx), "B": r(Bm, T, nx, nu), "lx": r(lx, T, nx), "lu": r(lu, T, nu),
            "lxx": r(lxx, T, nx, nx), "lux": r(lux, T, nu, nx), "luu": r(luu, T, nu, nu),
            "lfx": r(lfx, nx), "lfxx": r(lfxx, nx, nx)}


def total_cost(xb, ub, x_traj, immediate_cost, final_cost):
    """Σ_t ℓ(x̄_t − x_traj_t, ū_t) + ℓ_f(x̄_N), summed over t in order (:187-192)."""
    T = ub.shape[1]
    acc = np.zeros(xb.shape[0])
    for t in range(T):
        acc = acc + immediate_cost(xb[:, t] - x_traj[:, t], ub[:, t])
    return acc + final_cost(xb[:, T])


def forward_pass(x, u, x_traj, d, K, prev_cost, dynamicsf, immediate_cost, final_cost,
                 max_trials=64, alpha0=1.0, shrink=0.5):
    """forward_pass.jl:55-93 for every trajectory at once, each with its own α
    → (x̄, ū, cost, trials, accepted)."""
    nb, N, nx = x.shape
    T = N - 1
    xo, uo = x.copy(), u.copy()
    cost = np.full(nb, np.nan)
    trials = np.zeros(nb, dtype=np.int32)
    done = np.zeros(nb, dtype=bool)
    alpha = np.full(nb, float(alpha0))
    with np.errstate(all="ignore"):
        for trial in range(1, max_trials + 1):
            xb = np.empty_like(x)
            ub = np.empty_like(u)
            xb[:, 0] = x[:, 0]                                                        # :65
            for k in range(T):                                                        # :71
                dx = xb[:, k] - x[:, k]                                               # :72
                ub[:, k] = (u[:, k] + alpha[:, None] * d[:, k]) + np.einsum("bij,bj->bi", K[:, k], dx)  # :73
                xb[:, k + 1] = dynamicsf(xb[:, k], ub[:, k])                          # :74
            c = total_cost(xb, ub, x_traj, immediate_cost, final_cost)                # :76
            acc = ~done & ((prev_cost - c) > 0)                                       # :77-80
            trials = np.where(~done, trial, trials)
            cost = np.where(acc | ~done, c, cost)
            xo[acc], uo[acc] = xb[acc], ub[acc]
            done |= acc
            if done.all():
                break
            alpha = np.where(done, alpha, alpha * shrink)                             # :82
    return xo, uo, cost, trials, done


def fit(x_init, u_init, dynamicsf, immediate_cost, final_cost, quad, fquad, x_traj=None,
        max_iter=100, tol=1e-6, max_trials=64, mu=0.01):
    """fit (forward_pass.jl:148-179) for a batch → dict(x, u, cost, iters, status,
    history), status as include/ilqr.h's ilqr_traj_status: 1 converged, 2 max_iter,
    3 line search exhausted, 4 NaN."""
    xi, ui = np.array(x_init, dtype=np.float64), np.array(u_init, dtype=np.float64)
    nb = xi.shape[0]
    xt = np.zeros_like(xi) if x_traj is None else np.asarray(x_traj, dtype=np.float64)
    prev = np.full(nb, np.inf)                                                        # :159
    status = np.zeros(nb, dtype=np.int32)
    iters = np.zeros(nb, dtype=np.int32)
    hist = {"cost": [], "trials": [], "du2": []}
    for it in range(1, max_iter + 1):                                                 # :161
        run = status == 0
        if not run.any():
            break
        tl = derivative_tiles(xi, ui, dynamicsf, quad, fquad)
        d, K, bst = cref.tiles_backward(tl, mu=mu, symmetrize=True)                  # :162
        status = np.where(run & (bst == 4), 4, status)
        run = status == 0
        xn, un, c, ntr, ok = forward_pass(xi, ui, xt, d, K, prev, dynamicsf, immediate_cost,
                                          final_cost, max_trials)                    # :163-166
        iters = np.where(run, it, iters)
        bad = run & ~ok
        status = np.where(bad, np.where(np.isnan(c), 4, 3), status)
        acc = run & ok
        prev = np.where(acc, c, prev)                                                 # :168
        du2 = ((un - ui) ** 2).sum(axis=(1, 2))
        conv = acc & (du2 <= tol)                                                     # :171
        hist["cost"].append(np.where(acc, c, np.nan))
        hist["trials"].append(np.where(run, ntr, 0))
        hist["du2"].append(np.where(run, du2, np.nan))
        status = np.where(conv, 1, status)
        step = acc & ~conv
        xi[step], ui[step] = xn[step], un[step]                                       # :174-175
    status = np.where(status == 0, 2, status)
    return {"x": xi, "u": ui, "cost": prev, "iters": iters, "status": status,
            "history": {k: np.array(v) for k, v in hist.items()}}
