"""Host-side mirror of the reference API (aabouman/iLQR.jl, module `iLQR`), backed
by the HIP kernels — same names, argument meaning and error behaviour:

  fit(x_init, u_init, dynamicsf, immediate_cost, final_cost; x_traj, max_iter, tol)
        /root/reference/src/forward_pass.jl:148-179
  backward_pass(x, u, dynamicsf, immediate_cost, final_cost) -> (δu, K)
        /root/reference/src/backward_pass.jl:324-357
  forward_pass(x, u, x_traj, δu, K, prev_cost, dynamicsf, immediate_cost, final_cost)
        -> (x̄, ū, new_cost)      /root/reference/src/forward_pass.jl:55-93

Arrays follow the reference's per-trajectory layout (x: (N, nx) rows = time
steps, u: (T, nu), δu: (T, nu), K: (T, nu, nx)); a leading batch dimension
solves many independent problems at once. numpy inputs are copied to the GPU
and results copied back; torch CUDA inputs stay on the device.

Problem families: LinearDynamics/QuadraticCost/QuadraticFinalCost and the 2-link
arm closures run fused device kernels; ANY other closures (written with torch ops
on 1-D tensors) take the generic path — derivative tiles by torch.func on the
device (ForwardDiff's role), the Riccati recursion in the HIP kernel behind
ilqr_backward_tiles, and forward_pass rolling the user's dynamics out with torch.

Errors mirror the reference: AssertionError for N ≠ M+1 (backward_pass.jl:329,
forward_pass.jl:62,156) and for NaNs (backward_pass.jl:353-354,
forward_pass.jl:89-90), TypeError for a non-integer max_iter
(forward_pass.jl:152). The reference's unbounded line search (:70-87) is capped
(`max_trials`); an exhausted search raises `LineSearchExhausted` in
forward_pass and, in fit, stops that trajectory at its current iterate.
"""
from __future__ import annotations

import warnings

import numpy as np
import torch

from . import _lib
from . import cache as _cache
from . import tiles as _tiles
from .chain import ChainSolver, chain_problem_of
from .cost_functions import simple_costs_of
from .problems import (LinearDynamics, QuadraticCost, QuadraticFinalCost, is_two_link,
                       lq_from_closures)
from .solver import Solver


class LineSearchExhausted(RuntimeError):
    pass


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("the iLQR HIP path needs a GPU (no CPU fallback)")
    return torch.cuda.current_device()


def _as_batch(a, name, ndim):
    """→ (device tensor with leading batch dim, was_batched, was_torch)."""
    is_t = isinstance(a, torch.Tensor)
    t = a if is_t else torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.float64)))
    if t.dim() == ndim:
        t, batched = t.unsqueeze(0), False
    elif t.dim() == ndim + 1:
        batched = True
    else:
        raise AssertionError(f"{name}: expected {ndim} or {ndim + 1} dimensions")
    t = t.to(device=_device(), dtype=torch.float64).contiguous()
    return t, batched, is_t


def _out(t, batched, as_torch):
    if not batched:
        t = t[0]
    return t if as_torch else t.cpu().numpy()


def _family(dynamicsf, immediate_cost, final_cost):
    """'two_link', 'lq', 'chain' (recognised problem families with fused device kernels)
    or 'closures' (arbitrary torch closures: derivative tiles + ilqr_backward_tiles)."""
    if is_two_link(dynamicsf, immediate_cost, final_cost):
        return "two_link"
    if chain_problem_of(dynamicsf, immediate_cost, final_cost) is not None:
        return "chain"
    from .floating import floating_problem_of
    if floating_problem_of(dynamicsf, immediate_cost, final_cost) is not None:
        return "floating"
    if (isinstance(dynamicsf, LinearDynamics) and isinstance(immediate_cost, QuadraticCost)
            and isinstance(final_cost, QuadraticFinalCost)):
        return "lq"
    return "closures"


def _eltype(a):
    """The reference is generic in the element type (Julia): Float32 inputs solve in fp32."""
    dt = a.dtype if isinstance(a, (torch.Tensor, np.ndarray)) else None
    return torch.float32 if dt in (torch.float32, np.float32) else torch.float64


def _chain_solver(xb, ub, dynamicsf, immediate_cost, final_cost, dtype):
    nb, N, nx = xb.shape
    _, M, nu = ub.shape
    assert N == M + 1, "size(x)[1] == size(u)[1] + 1"   # backward_pass.jl:329
    p = chain_problem_of(dynamicsf, immediate_cost, final_cost)
    if (p.nx, p.nu) != (nx, nu):
        raise AssertionError(f"problem is ({p.nx}, {p.nu}) but x/u are ({nx}, {nu})")
    s = ChainSolver(p, M, nb, dtype=dtype, device=_device())
    fc = simple_costs_of(p, immediate_cost, final_cost)   # cost_functions.jl's factories
    if fc is not None:
        try:
            s.set_simple_costs(fc.body, fc.point, fc.final_target, fc.weight, fc.euclidean)
        except Exception:
            s.close()
            raise
    return s


def _tiles_solver(xb, ub):
    """The closure path's tiles handle of this shape, cached between calls (cache.py)."""
    nb, N, nx = xb.shape
    _, M, nu = ub.shape
    assert N == M + 1, "size(x)[1] == size(u)[1] + 1"   # backward_pass.jl:329
    dev = _device()
    return _cache.workspace(("tiles", dev, nx, nu, M, nb),
                            lambda: Solver(nx, nu, M, nb, device=dev, kind=_lib.PROBLEM_TILES))


def _floating_solver(xb, ub, dynamicsf, immediate_cost, final_cost):
    """The floating-base family's handle for this model and shape, cached (cache.py)."""
    from .floating import FloatingSolver, floating_problem_of
    nb, N, nx = xb.shape
    _, M, nu = ub.shape
    assert N == M + 1, "size(x)[1] == size(u)[1] + 1"   # backward_pass.jl:329
    p = floating_problem_of(dynamicsf, immediate_cost, final_cost)
    if (p.nx, p.nu) != (nx, nu):
        raise AssertionError(f"problem is ({p.nx}, {p.nu}) but x/u are ({nx}, {nu})")
    dev = _device()
    return _cache.workspace(("floating", dev, bytes(p.struct()), M, nb),
                            lambda: FloatingSolver(p, M, nb, device=dev))


def clear_cache():
    """Close the device workspaces fit / backward_pass / linearize_dynamics keep per shape
    and release the generic closure path's cached rollout graphs (ilqr_amd.tiles)."""
    _cache.clear()
    from . import tiles
    tiles.clear_graphs()


def _solver(xb, ub, dynamicsf, immediate_cost, final_cost):
    nb, N, nx = xb.shape
    _, M, nu = ub.shape
    assert N == M + 1, "size(x)[1] == size(u)[1] + 1"   # backward_pass.jl:329
    assert ub.shape[0] == nb, "batch sizes differ"
    if is_two_link(dynamicsf, immediate_cost, final_cost):
        if (nx, nu) != (4, dynamicsf.nu):
            raise AssertionError(f"the 2-link arm is (4, {dynamicsf.nu}) but x/u are ({nx}, {nu})")
        return Solver(nx, nu, M, nb, device=_device(), kind=_lib.PROBLEM_TWO_LINK)
    lq = lq_from_closures(dynamicsf, immediate_cost, final_cost, nb)
    if (lq.nx, lq.nu) != (nx, nu):
        raise AssertionError(f"problem is ({lq.nx}, {lq.nu}) but x/u are ({nx}, {nu})")
    s = Solver(nx, nu, M, nb, device=_device())
    s.set_problem(lq)
    return s


def backward_pass(x, u, dynamicsf, immediate_cost, final_cost):
    """→ (δu, K) exactly like iLQR.backward_pass (backward_pass.jl:324-357)."""
    xb, batched, is_t = _as_batch(x, "x", 2)
    ub, _, _ = _as_batch(u, "u", 2)
    fam = _family(dynamicsf, immediate_cost, final_cost)
    if fam == "closures":
        with _tiles_solver(xb, ub) as s:
            tl = _tiles.derivative_tiles(xb, ub, dynamicsf, immediate_cost, final_cost)
            d, K, st = s.backward_tiles(tl)
    elif fam == "floating":
        with _floating_solver(xb, ub, dynamicsf, immediate_cost, final_cost) as s:
            d, K, st = s.backward(xb, ub)
    elif fam == "chain":
        dt = _eltype(x)
        xb, ub = xb.to(dt), ub.to(dt)
        s = _chain_solver(xb, ub, dynamicsf, immediate_cost, final_cost, dt)
        d, K, st = s.backward(xb, ub)
        s.close()
    else:
        s = _solver(xb, ub, dynamicsf, immediate_cost, final_cost)
        d, K, st = s.backward(xb, ub)
        s.close()
    if bool((st == _lib.TRAJ_NAN).any()):
        raise AssertionError("!any(isnan, δu/K) failed")   # backward_pass.jl:353-354
    return _out(d, batched, is_t), _out(K, batched, is_t)


def forward_pass(x, u, x_traj, du, K, prev_cost, dynamicsf, immediate_cost, final_cost,
                 max_trials=None):
    """→ (x̄, ū, new_cost) exactly like iLQR.forward_pass (forward_pass.jl:55-93)."""
    xb, batched, is_t = _as_batch(x, "x", 2)
    ub, _, _ = _as_batch(u, "u", 2)
    nb, N, nx = xb.shape
    assert N == ub.shape[1] + 1, "size(x)[1] == size(u)[1] + 1"   # forward_pass.jl:62
    xt, _, _ = _as_batch(x_traj if x_traj is not None else np.zeros((nb, N, nx)) if batched
                         else np.zeros((N, nx)), "x_traj", 2)
    db, _, _ = _as_batch(du, "du", 2)
    Kb, _, _ = _as_batch(K, "K", 3)
    pc = torch.as_tensor(np.broadcast_to(np.asarray(prev_cost, dtype=np.float64), (nb,)).copy()
                         if not isinstance(prev_cost, torch.Tensor) else prev_cost,
                         dtype=torch.float64).reshape(nb).to(xb.device).contiguous()
    fam = _family(dynamicsf, immediate_cost, final_cost)
    if fam == "chain":
        dt = _eltype(x)
        s = _chain_solver(xb, ub, dynamicsf, immediate_cost, final_cost, dt)
        o = _lib.default_options(max_trials=max_trials)
        xn, un, cost, trials, st = s.forward(xb.to(dt), ub.to(dt), db.to(dt), Kb.to(dt),
                                             pc.to(dt), x_traj=xt.to(dt), options=o)
        s.close()
    elif fam == "floating":
        with _floating_solver(xb, ub, dynamicsf, immediate_cost, final_cost) as s:
            o = _lib.default_options(max_trials=max_trials)
            xn, un, cost, trials, st = s.forward(xb, ub, db, Kb, pc, x_traj=xt, options=o)
    elif fam == "closures":
        xn, un, cost, trials, ok = _tiles.rollout_forward(
            xb, ub, xt, db, Kb, pc, dynamicsf, immediate_cost, final_cost,
            max_trials=max_trials or _lib.default_options().max_trials)
        st = torch.where(ok, 0, torch.where(torch.isnan(cost), _lib.TRAJ_NAN,
                                            _lib.TRAJ_LS_EXHAUSTED)).to(torch.int32)
    else:
        s = _solver(xb, ub, dynamicsf, immediate_cost, final_cost)
        xn, un, cost, trials, st = s.forward(xb, ub, db, Kb, pc, x_traj=xt, max_trials=max_trials)
        s.close()
    if bool((st == _lib.TRAJ_NAN).any()):
        raise AssertionError("!any(isnan, ū/x̄) failed")   # forward_pass.jl:89-90
    if bool((st == _lib.TRAJ_LS_EXHAUSTED).any()):
        raise LineSearchExhausted("no cost decrease within max_trials (the reference loops forever)")
    c = cost if is_t else cost.cpu().numpy()
    return _out(xn, batched, is_t), _out(un, batched, is_t), (c if batched else float(c[0]))


def fit(x_init, u_init, dynamicsf, immediate_cost, final_cost, *, x_traj=None,
        max_iter: int = 100, tol: float = 1e-6, return_info: bool = False, verbose: bool = False):
    """→ (x̄, ū) exactly like iLQR.fit (forward_pass.jl:148-179), including its
    quirk of returning the iterate BEFORE the update that met `tol` (:171).
    verbose: print the reference's per-iteration line `Iteration: i  Total Cost: c`
    (:167) — for each trajectory of a batch — from the fit's history (ilqr_fit_ex);
    return_info adds it as info["history"] (arrays (max_iter, batch): cost, trials,
    alpha, du2)."""
    if not isinstance(max_iter, (int, np.integer)) or isinstance(max_iter, bool):
        raise TypeError("max_iter::Int64")   # forward_pass.jl:152
    xb, batched, is_t = _as_batch(x_init, "x_init", 2)
    ub, _, _ = _as_batch(u_init, "u_init", 2)
    nb, N, nx = xb.shape
    assert N == ub.shape[1] + 1, "size(x_init)[2] == size(u_init)[1]"   # forward_pass.jl:156
    xt = None
    if x_traj is not None:
        xt, _, _ = _as_batch(x_traj, "x_traj", 2)
    fam = _family(dynamicsf, immediate_cost, final_cost)
    if fam == "closures":
        r = _fit_closures(xb, ub, xt, dynamicsf, immediate_cost, final_cost, int(max_iter),
                          float(tol), history=verbose or return_info)
    elif fam == "floating":
        with _floating_solver(xb, ub, dynamicsf, immediate_cost, final_cost) as s:
            r = s.fit(xb, ub, x_traj=xt, max_iter=int(max_iter), tol=float(tol),
                      history=verbose or return_info)
    elif fam == "chain":
        dt = _eltype(x_init)
        s = _chain_solver(xb, ub, dynamicsf, immediate_cost, final_cost, dt)
        r = s.fit(xb.to(dt), ub.to(dt), x_traj=None if xt is None else xt.to(dt),
                  max_iter=int(max_iter), tol=float(tol), history=verbose or return_info)
        s.close()
    else:
        s = _solver(xb, ub, dynamicsf, immediate_cost, final_cost)
        r = s.fit(xb, ub, x_traj=xt, max_iter=int(max_iter), tol=float(tol),
                  history=verbose or return_info)
        s.close()
    if verbose and r.history is not None:
        from .solver import print_history
        for b in range(xb.shape[0]):
            print_history(r.history, b)
    st = r.status.cpu().numpy()
    if (st == _lib.TRAJ_NAN).any():
        raise AssertionError("NaN in a trajectory (reference: AssertionError)")
    if (st == _lib.TRAJ_LS_EXHAUSTED).any():
        warnings.warn("line search exhausted for %d trajectories (the reference would loop "
                      "forever); they return their last iterate" % int((st == _lib.TRAJ_LS_EXHAUSTED).sum()))
    out = (_out(r.x, batched, is_t), _out(r.u, batched, is_t))
    if return_info:
        info = {"cost": r.cost.cpu().numpy(), "iters": r.iters.cpu().numpy(), "status": st}
        if r.history is not None:
            info["history"] = {k: v.cpu().numpy() for k, v in r.history.items()}
        return out + (info,)
    return out


def _fit_closures(xb, ub, xt, dynamicsf, immediate_cost, final_cost, max_iter, tol, history=False):
    """fit (forward_pass.jl:148-179) for arbitrary torch closures: per iteration,
    derivative tiles (torch.func on the device) → ilqr_backward_tiles (HIP) →
    forward_pass rollout of the user dynamics (torch on the device). Trajectories
    that converge, exhaust their line search or hit NaN stop; the rest continue."""
    with _tiles_solver(xb, ub) as s:
        return _fit_closures_on(s, xb, ub, xt, dynamicsf, immediate_cost, final_cost, max_iter, tol,
                                history)


def _fit_closures_on(s, xb, ub, xt, dynamicsf, immediate_cost, final_cost, max_iter, tol, history):
    from .solver import FitResult
    nb = xb.shape[0]
    dev = xb.device
    xi, ui = xb.clone(), ub.clone()
    prev = torch.full((nb,), float("inf"), dtype=torch.float64, device=dev)   # :159
    status = torch.zeros(nb, dtype=torch.int32, device=dev)
    iters = torch.zeros(nb, dtype=torch.int32, device=dev)
    opts = _lib.default_options()
    max_trials = opts.max_trials
    hist = None
    if history:
        from .solver import alloc_history
        hist, _ = alloc_history(max_iter, nb, dev)
    for it in range(1, max_iter + 1):                                            # :161
        run = status == _lib.TRAJ_OK
        if not bool(run.any()):
            break
        tl = _tiles.derivative_tiles(xi, ui, dynamicsf, immediate_cost, final_cost)
        d, K, bst = s.backward_tiles(tl)                                          # :162
        status = torch.where(run & (bst == _lib.TRAJ_NAN), _lib.TRAJ_NAN, status).to(torch.int32)
        run = status == _lib.TRAJ_OK
        xn, un, c, ntr, ok = _tiles.rollout_forward(xi, ui, xt, d, K, prev, dynamicsf,
                                                    immediate_cost, final_cost, max_trials)  # :163-166
        iters = torch.where(run, it, iters).to(torch.int32)
        bad = run & ~ok
        status = torch.where(bad, torch.where(torch.isnan(c), _lib.TRAJ_NAN, _lib.TRAJ_LS_EXHAUSTED),
                             status).to(torch.int32)
        acc = run & ok
        prev = torch.where(acc, c, prev)                                          # :168
        du2 = ((un - ui) ** 2).sum(dim=(1, 2))
        conv = acc & (du2 <= tol)                                                 # :171
        if hist is not None:  # ilqr_history's fields for this iteration
            ntr = torch.as_tensor(ntr, device=dev).to(torch.int32)
            hist["trials"][it - 1] = torch.where(run, ntr, 0)
            hist["cost"][it - 1] = torch.where(acc, c, float("nan"))
            alpha = opts.alpha0 * torch.pow(torch.full_like(c, opts.shrink), (ntr - 1).clamp(min=0).double())
            hist["alpha"][it - 1] = torch.where(acc, alpha, float("nan"))
            hist["du2"][it - 1] = torch.where(run, du2, float("nan"))
        status = torch.where(conv, _lib.TRAJ_CONVERGED, status).to(torch.int32)
        step = acc & ~conv
        xi = torch.where(step[:, None, None], xn, xi)                            # :174-175
        ui = torch.where(step[:, None, None], un, ui)
    status = torch.where(status == _lib.TRAJ_OK, _lib.TRAJ_MAX_ITER, status).to(torch.int32)
    return FitResult(xi, ui, prev, iters, status, _lib.OK, hist)


from .helpers import (feedback_parameters, final_cost_quadratization,  # noqa: E402  (the per-step API)
                      immediate_cost_quadratization, linearize_dynamics, optimal_controller_param, step_back)

__all__ = ["fit", "backward_pass", "forward_pass", "LineSearchExhausted", "clear_cache", "linearize_dynamics",
           "immediate_cost_quadratization", "final_cost_quadratization", "optimal_controller_param",
           "feedback_parameters", "step_back"]
