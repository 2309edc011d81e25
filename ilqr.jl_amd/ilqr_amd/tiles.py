"""Derivative tiles for ARBITRARY closures.

The reference differentiates its user callbacks with ForwardDiff
(src/backward_pass.jl:25-40 linearize_dynamics, :81-109
immediate_cost_quadratization, :134-153 final_cost_quadratization). Here the
same derivatives are taken with torch.func, vmapped over every (trajectory, time
step) at once ON THE GPU; the Riccati recursion then runs in the HIP kernel behind
ilqr_backward_tiles. The derivatives are exact like ForwardDiff's, but taken in
REVERSE mode (jacrev): PyTorch 2.10's batching rule for the forward-mode derivative
of linalg.solve / lu_solve under vmap returns wrong values (off by O(1) relative;
tests/test_closures.py keeps the counter-example), and a dynamics closure solving
M v̇ = τ − b — the reference's RBD example, RBD_helper_functions.jl:64 — hits it.

Closures must be written with torch operations on 1-D tensors — the analogue of
the reference's eltype-generic Julia closures:
    dynamicsf(x, u) -> x_next,  immediate_cost(x, u) -> scalar,  final_cost(x) -> scalar

`rollout_forward` is forward_pass (src/forward_pass.jl:55-93) for such closures:
the rollout calls the user's dynamics, so it runs as torch ops on the device
(batched over trajectories, sequential over time), not in a HIP kernel.
"""
from __future__ import annotations

import torch

TILE_NAMES = ("A", "B", "lx", "lu", "lxx", "lux", "luu", "lfx", "lfxx")


def derivative_tiles(x, u, dynamicsf, immediate_cost, final_cost):
    """x (B, T+1, nx), u (B, T, nu) CUDA float64 → dict of ilqr_tiles tensors."""
    from torch.func import jacrev, vmap
    nb, N, nx = x.shape
    T, nu = u.shape[1], u.shape[2]
    try:
        return _tiles(x, u, dynamicsf, immediate_cost, final_cost, jacrev, vmap, nb, nx, T, nu)
    except (TypeError, RuntimeError, ValueError) as e:
        raise NotImplementedError(
            "generic closures must be written with torch operations on 1-D tensors "
            f"(torch.func could not differentiate them: {e})") from e


def _tiles(x, u, dynamicsf, immediate_cost, final_cost, jac, vmap, nb, nx, T, nu):
    xs = x[:, :T].reshape(-1, nx)
    us = u.reshape(-1, nu)
    A, Bm = vmap(jac(dynamicsf, argnums=(0, 1)))(xs, us)                # :32-33
    lx, lu = vmap(jac(immediate_cost, argnums=(0, 1)))(xs, us)          # :95-96,102-103
    lxx = vmap(jac(jac(immediate_cost, argnums=0), argnums=0))(xs, us)  # :97,104
    lux = vmap(jac(jac(immediate_cost, argnums=1), argnums=0))(xs, us)  # :98,105 (m×n)
    luu = vmap(jac(jac(immediate_cost, argnums=1), argnums=1))(xs, us)  # :99,106
    xN = x[:, T]
    lfx = vmap(jac(final_cost))(xN)                                     # :142
    lfxx = vmap(jac(jac(final_cost)))(xN)                               # :143
    out = {"A": A.reshape(nb, T, nx, nx), "B": Bm.reshape(nb, T, nx, nu),
           "lx": lx.reshape(nb, T, nx), "lu": lu.reshape(nb, T, nu),
           "lxx": lxx.reshape(nb, T, nx, nx), "lux": lux.reshape(nb, T, nu, nx),
           "luu": luu.reshape(nb, T, nu, nu), "lfx": lfx.reshape(nb, nx),
           "lfxx": lfxx.reshape(nb, nx, nx)}
    return {k: v.to(torch.float64).contiguous() for k, v in out.items()}


def total_cost(xb, ub, x_traj, immediate_cost, final_cost):
    """total_cost (src/forward_pass.jl:182-196), batched: Σ_t ℓ(x̄_t − x_traj_t, ū_t) + ℓ_f(x̄_N)."""
    from torch.func import vmap
    nb, N, nx = xb.shape
    T = N - 1
    e = xb[:, :T] - (x_traj[:, :T] if x_traj is not None else 0.0)
    c = vmap(vmap(immediate_cost))(e, ub)            # (B, T)
    acc = torch.zeros(nb, dtype=torch.float64, device=xb.device)
    for t in range(T):                                # sequential sum, as :187-190
        acc = acc + c[:, t]
    return acc + vmap(final_cost)(xb[:, T])


def rollout_forward(x, u, x_traj, d, K, prev_cost, dynamicsf, immediate_cost, final_cost,
                    max_trials=64, alpha0=1.0, shrink=0.5):
    """forward_pass (src/forward_pass.jl:55-93) for torch closures, batched over
    trajectories; each trajectory keeps its own α. → (x̄, ū, cost, trials, accepted)."""
    from torch.func import vmap
    f = vmap(dynamicsf)
    nb, N, nx = x.shape
    T = N - 1
    xo, uo = x.clone(), u.clone()
    cost = torch.full((nb,), float("nan"), dtype=torch.float64, device=x.device)
    trials = torch.zeros(nb, dtype=torch.int32, device=x.device)
    done = torch.zeros(nb, dtype=torch.bool, device=x.device)
    alpha = torch.full((nb,), float(alpha0), dtype=torch.float64, device=x.device)
    for trial in range(1, max_trials + 1):
        xb = torch.empty_like(x)
        ub = torch.empty_like(u)
        xb[:, 0] = x[:, 0]                                                      # :65
        for k in range(T):                                                      # :71
            dx = xb[:, k] - x[:, k]                                             # :72
            ub[:, k] = (u[:, k] + alpha[:, None] * d[:, k]) + torch.einsum("bij,bj->bi", K[:, k], dx)  # :73
            xb[:, k + 1] = f(xb[:, k], ub[:, k])                                # :74
        c = total_cost(xb, ub, x_traj, immediate_cost, final_cost)              # :76
        acc = (~done) & ((prev_cost - c) > 0)                                   # :77-80
        sel = acc | ~done
        trials = torch.where(~done, torch.full_like(trials, trial), trials)
        cost = torch.where(sel, c, cost)
        xo = torch.where(acc[:, None, None], xb, xo)
        uo = torch.where(acc[:, None, None], ub, uo)
        done = done | acc
        if bool(done.all()):
            break
        alpha = torch.where(done, alpha, alpha * shrink)                        # :82
    return xo, uo, cost, trials, done
