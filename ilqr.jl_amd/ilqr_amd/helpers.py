"""The reference's documented per-step API (docs/src/documentation.md:13-51), re-exposed
with its signatures:

  linearize_dynamics(x, u, dynamicsf) -> (𝐀, 𝐁)                 backward_pass.jl:25-40
  immediate_cost_quadratization(x, u, immediate_cost)
        -> (𝑞, 𝐪, 𝐫, 𝐐, 𝐏, 𝐑)                                    backward_pass.jl:81-109
  final_cost_quadratization(x, final_cost) -> (𝑞ₙ, 𝐪ₙ, 𝐐ₙ)       backward_pass.jl:134-153
  optimal_controller_param(𝐀, 𝐁, 𝐫, 𝐏, 𝐑, 𝐬′, 𝐒′) -> (𝐠, 𝐆, 𝐇)   backward_pass.jl:177-186
  feedback_parameters(𝐠, 𝐆, 𝐇) -> (𝛿𝐮ᶠᶠ, 𝐊)                      backward_pass.jl:207-218
  step_back(𝐀, 𝑞, 𝐪, 𝐐, 𝐠, 𝐆, 𝐇, 𝛿𝐮ᶠᶠ, 𝐊, 𝑠′, 𝐬′, 𝐒′) -> (𝑠, 𝐬, 𝐒) backward_pass.jl:262-273

linearize_dynamics takes the reference's vector form (x::AbstractVector, u) → (A, B), the
trajectory form its own test calls (test/test_linearize_dynamics.jl:10-14: x and u with
one row per step → 𝐀s[i, :, :], 𝐁s[i, :, :]) and a leading batch dimension. It runs on
the device: ilqr_linearize (C ABI) for the LQ family (f linear: A, B exactly) and the
2-link arm (Dual<4+nu> through the RK4 functor — the arithmetic of the fused backward),
ilqr_chain_linearize for URDF chains, torch.func forward-mode AD vmapped over every step
for other torch closures (ForwardDiff's role, as in ilqr_amd.tiles).

The quadratizations use the closed forms of the recognised cost families and torch.func
for torch closures. The three algebra helpers are the step's host algebra, batched over
any leading dimensions, computed with torch on the inputs' device (numpy in → numpy out);
the fused kernels never call them — they exist for callers of the reference's API.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from . import cache as _cache
from .problems import (LinearDynamics, QuadraticCost, QuadraticFinalCost, TwoLinkArm, TwoLinkCost,
                       TwoLinkDynamics, TwoLinkFinalCost)

REG_MU = 0.01  # feedback_parameters' fixed regulariser (backward_pass.jl:214)


def _t(a, device=None):
    """→ float64 tensor (numpy / scalars / tensors)."""
    if isinstance(a, torch.Tensor):
        return a.to(torch.float64) if device is None else a.to(device, torch.float64)
    return torch.as_tensor(np.asarray(a, dtype=np.float64), device=device)


def _ret(as_torch, *ts):
    out = tuple(t if as_torch else (t.item() if t.dim() == 0 else t.cpu().numpy()) for t in ts)
    return out


def _gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("linearize_dynamics runs on the GPU (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


# -- linearize_dynamics (backward_pass.jl:25-40) ------------------------------------------
def linearize_dynamics(x, u, dynamicsf):
    """(𝐀, 𝐁) = (∂f/∂x, ∂f/∂u). x (nx,), u (nu,) → (nx, nx), (nx, nu); x (N, nx),
    u (T, nu) with N ∈ {T, T+1} → 𝐀s (T, nx, nx), 𝐁s (T, nx, nu) at (x[i], u[i]),
    i < T (test_linearize_dynamics.jl:10-14); a leading batch dimension is kept."""
    as_torch = isinstance(x, torch.Tensor)
    dev = _gpu()
    xt, ut = _t(x, dev), _t(u, dev)
    if xt.dim() != ut.dim() or xt.dim() not in (1, 2, 3):
        raise AssertionError("x and u: both vectors, both (steps, n) matrices or both batched")
    point, traj = xt.dim() == 1, xt.dim() == 2
    if point:
        xt, ut = xt[None, None], ut[None, None]
    elif xt.dim() == 2:
        xt, ut = xt[None], ut[None]
    nb, N, nx = xt.shape
    T, nu = ut.shape[1], ut.shape[2]
    if ut.shape[0] != nb or N not in (T, T + 1):
        raise AssertionError(f"x has {N} rows for {T} inputs (expected {T} or {T + 1})")
    if N == T:  # the ABI reads (B, T+1, nx); the extra state is never read
        xt = torch.cat([xt, xt[:, -1:]], dim=1)
    xt, ut = xt.contiguous(), ut.contiguous()
    A, Bm = _linearize(xt, ut, dynamicsf, nb, nx, nu, T)
    if point:
        A, Bm = A[0, 0], Bm[0, 0]
    elif traj:
        A, Bm = A[0], Bm[0]
    return _ret(as_torch, A, Bm)


def _linearize(x, u, dynamicsf, nb, nx, nu, T):
    from .chain import ChainDynamics, ChainSolver
    from .solver import Solver
    dev = x.device.index
    if isinstance(dynamicsf, TwoLinkDynamics) and (nx, nu) == (4, dynamicsf.nu):
        with _cache.workspace(("two_link", dev, nu, T, nb),
                              lambda: Solver(4, nu, T, nb, device=dev, kind=_lib.PROBLEM_TWO_LINK)) as s:
            return _abi_linearize(s, x, u)
    if isinstance(dynamicsf, LinearDynamics) and (dynamicsf.nx, dynamicsf.nu) == (nx, nu) \
            and _lib.load().ilqr_supported(_lib.PROBLEM_LQ, nx, nu):
        from .problems import LQBatch

        def bc(a, shape):
            a = np.asarray(a, dtype=np.float64)
            return np.broadcast_to(a, (nb,) + shape) if a.ndim == 2 else a
        z = np.zeros((nb, nx, nx))
        with _cache.workspace(("lq", dev, nx, nu, T, nb), lambda: Solver(nx, nu, T, nb, device=dev)) as s:
            s.set_problem(LQBatch(bc(dynamicsf.A, (nx, nx)), bc(dynamicsf.B, (nx, nu)), z, np.zeros((nb, nu, nu)), z))
            return _abi_linearize(s, x, u)
    if isinstance(dynamicsf, ChainDynamics) and (dynamicsf.problem.nx, dynamicsf.problem.nu) == (nx, nu):
        s = ChainSolver(dynamicsf.problem, T, nb, dtype=torch.float64, device=dev)
        try:
            A, Bm = s.linearize(x, u)
            torch.cuda.synchronize(x.device)
        finally:
            s.close()
        return A, Bm
    from .floating import FloatingDynamics, FloatingSolver
    if isinstance(dynamicsf, FloatingDynamics) and (dynamicsf.problem.nx, dynamicsf.problem.nu) == (nx, nu):
        key = ("floating", dev, bytes(dynamicsf.problem.struct()), T, nb)
        with _cache.workspace(key, lambda: FloatingSolver(dynamicsf.problem, T, nb, device=dev)) as s:
            return s.linearize(x, u)
    # any other torch closure: ForwardDiff's role, in reverse mode (tiles.py: PyTorch's
    # vmapped forward-mode derivative of linalg.solve is wrong)
    from torch.func import jacrev, vmap
    xs, us = x[:, :T].reshape(-1, nx), u.reshape(-1, nu)
    try:
        A, Bm = vmap(jacrev(dynamicsf, argnums=(0, 1)))(xs, us)   # :32-33
    except (TypeError, RuntimeError, ValueError) as e:
        raise NotImplementedError("closures must be written with torch operations on 1-D tensors "
                                  f"(torch.func could not differentiate them: {e})") from e
    return A.reshape(nb, T, nx, nx).to(torch.float64), Bm.reshape(nb, T, nx, nu).to(torch.float64)


def _abi_linearize(s, x, u):
    """ilqr_linearize on the workspace `s` (the caller owns and keeps it)."""
    from .solver import _ptr
    A = torch.empty((s.batch, s.T, s.nx, s.nx), dtype=torch.float64, device=x.device)
    Bm = torch.empty((s.batch, s.T, s.nx, s.nu), dtype=torch.float64, device=x.device)
    s._bind_stream()
    _lib.check(s.lib.ilqr_linearize(s.h, s._p(), _ptr(x), _ptr(u), _ptr(A), _ptr(Bm)), "ilqr_linearize")
    torch.cuda.current_stream(x.device).synchronize()
    return A, Bm


# -- cost quadratizations (backward_pass.jl:81-109, :134-153) -----------------------------
def _theta_target():
    return torch.as_tensor(TwoLinkArm.inverse_kinematics(), dtype=torch.float64)


def immediate_cost_quadratization(x, u, immediate_cost):
    """(𝑞, 𝐪, 𝐫, 𝐐, 𝐏, 𝐑) = (ℓ, ∇ₓℓ, ∇ᵤℓ, ∇²ₓₓℓ, ∂(∇ᵤℓ)/∂x (nu × nx), ∇²ᵤᵤℓ) at one
    (x, u) — vectors, like the reference."""
    as_torch = isinstance(x, torch.Tensor)
    xt, ut = _t(x), _t(u)
    dev = xt.device
    ut = ut.to(dev)
    nx, nu = xt.shape[0], ut.shape[0]
    P = torch.zeros((nu, nx), dtype=torch.float64, device=dev)
    if isinstance(immediate_cost, QuadraticCost) and immediate_cost.Q.ndim == 2:
        Q, R = _t(immediate_cost.Q, dev), _t(immediate_cost.R, dev)
        q = xt @ (Q @ xt) + ut @ (R @ ut)
        Qs, Rs = Q + Q.T, R + R.T
        return _ret(as_torch, q, Qs @ xt, Rs @ ut, Qs, P, Rs)
    if isinstance(immediate_cost, TwoLinkCost):  # 2_link_helper_functions.jl:82-97
        e = _theta_target().to(dev) - xt[:2]
        q = (e * e).sum() * 1.0 + (ut * ut).sum() * 1.0
        qv = torch.zeros(nx, dtype=torch.float64, device=dev)
        qv[:2] = -2.0 * e
        Q = torch.zeros((nx, nx), dtype=torch.float64, device=dev)
        Q[0, 0] = Q[1, 1] = 2.0
        return _ret(as_torch, q, qv, 2.0 * ut, Q, P, 2.0 * torch.eye(nu, dtype=torch.float64, device=dev))
    from .chain import ChainCost
    from .cost_functions import SimpleImmediateCost
    if isinstance(immediate_cost, ChainCost):
        p = immediate_cost.problem
        n = p.n_joints
        w, rw = _t(p.q_weight, dev), _t(p.r_weight[: p.nu], dev)
        e = _t(p.target, dev) - xt[:n]
        q = (w * e * e).sum() + (rw * ut * ut).sum()
        qv = torch.zeros(nx, dtype=torch.float64, device=dev)
        qv[:n] = -2.0 * w * e
        Q = torch.zeros((nx, nx), dtype=torch.float64, device=dev)
        Q[:n, :n] = torch.diag(2.0 * w)
        return _ret(as_torch, q, qv, 2.0 * rw * ut, Q, P, torch.diag(2.0 * rw))
    if isinstance(immediate_cost, SimpleImmediateCost):  # cost_functions.jl:45-51: Σ uᵢ²
        Z = torch.zeros((nx, nx), dtype=torch.float64, device=dev)
        return _ret(as_torch, (ut * ut).sum(), torch.zeros(nx, dtype=torch.float64, device=dev), 2.0 * ut, Z, P,
                    2.0 * torch.eye(nu, dtype=torch.float64, device=dev))
    from torch.func import hessian, jacfwd
    f = immediate_cost
    try:
        q = f(xt, ut)
        qv = jacfwd(f, argnums=0)(xt, ut)                     # :95, :102
        r = jacfwd(f, argnums=1)(xt, ut)                      # :96, :103
        Q = hessian(f, argnums=0)(xt, ut)                     # :97, :104
        P = jacfwd(jacfwd(f, argnums=1), argnums=0)(xt, ut)   # :98, :105 (nu × nx)
        R = hessian(f, argnums=1)(xt, ut)                     # :99, :106
    except (TypeError, RuntimeError, ValueError) as e:
        raise NotImplementedError(f"immediate_cost must be written with torch operations ({e})") from e
    return _ret(as_torch, *(_t(v) for v in (q, qv, r, Q, P, R)))


def final_cost_quadratization(x, final_cost):
    """(𝑞ₙ, 𝐪ₙ, 𝐐ₙ) = (ℓ_f, ∇ℓ_f, ∇²ℓ_f) at x_N (a vector)."""
    as_torch = isinstance(x, torch.Tensor)
    xt = _t(x)
    dev, nx = xt.device, xt.shape[0]
    if isinstance(final_cost, QuadraticFinalCost) and final_cost.Qf.ndim == 2:
        Qf = _t(final_cost.Qf, dev)
        return _ret(as_torch, xt @ (Qf @ xt), (Qf + Qf.T) @ xt, Qf + Qf.T)
    if isinstance(final_cost, TwoLinkFinalCost):  # 2_link_helper_functions.jl:100-108
        e = _theta_target().to(dev) - xt[:2]
        qv = torch.zeros(nx, dtype=torch.float64, device=dev)
        qv[:2] = -2.0 * e
        Q = torch.zeros((nx, nx), dtype=torch.float64, device=dev)
        Q[0, 0] = Q[1, 1] = 2.0
        return _ret(as_torch, (e * e).sum() * 1.0, qv, Q)
    from .chain import ChainFinalCost
    from .cost_functions import SimpleFinalCost
    if isinstance(final_cost, ChainFinalCost):
        p = final_cost.problem
        n = p.n_joints
        w = _t(p.qf_weight, dev)
        e = _t(p.target, dev) - xt[:n]
        qv = torch.zeros(nx, dtype=torch.float64, device=dev)
        qv[:n] = -2.0 * w * e
        Q = torch.zeros((nx, nx), dtype=torch.float64, device=dev)
        Q[:n, :n] = torch.diag(2.0 * w)
        return _ret(as_torch, (w * e * e).sum(), qv, Q)
    f = final_cost
    if isinstance(final_cost, SimpleFinalCost):
        f = _simple_final_cost_torch(final_cost)
    from torch.func import hessian, jacfwd
    try:
        return _ret(as_torch, _t(f(xt)), _t(jacfwd(f)(xt)), _t(hessian(f)(xt)))   # :141-143
    except (TypeError, RuntimeError, ValueError) as e:
        raise NotImplementedError(f"final_cost must be written with torch operations ({e})") from e


def _simple_final_cost_torch(c):
    """cost_functions.jl:16-24's final cost as torch operations (the kinematics of
    cost_functions.point_position), so torch.func differentiates it."""
    ch = c.chain

    def f(x):
        w = torch.as_tensor(c.point, dtype=x.dtype, device=x.device)
        for i in range(c.body, -1, -1):
            a = torch.as_tensor(ch.axis[i], dtype=x.dtype, device=x.device)
            cq, sq = torch.cos(x[i]), torch.sin(x[i])
            r = cq * w + sq * torch.linalg.cross(a, w) + (1.0 - cq) * (a @ w) * a
            w = torch.as_tensor(ch.p[i], dtype=x.dtype, device=x.device) + \
                torch.as_tensor(ch.R0[i], dtype=x.dtype, device=x.device) @ r
        tg = torch.as_tensor(c.final_target, dtype=x.dtype, device=x.device)
        e = (w if c.euclidean else w[2].expand(3)) - tg
        return c.weight * (e * e).sum()
    return f


# -- the step's algebra (backward_pass.jl:177-186, :207-218, :262-273) --------------------
def _tr(M):
    return M.transpose(-1, -2)


def _mv(M, v):
    return (M @ v.unsqueeze(-1)).squeeze(-1)


def optimal_controller_param(A, B, r, P, R, s, S):
    """(𝐠, 𝐆, 𝐇) = (𝐫 + 𝐁ᵀ𝐬′, 𝐏 + 𝐁ᵀ𝐒′𝐀, 𝐑 + 𝐁ᵀ𝐒′𝐁) (:181-183)."""
    as_torch = isinstance(A, torch.Tensor)
    dev = A.device if as_torch else None
    A, B, r, P, R, s, S = (_t(v, dev) for v in (A, B, r, P, R, s, S))
    BtS = _tr(B) @ S
    return _ret(as_torch, r + _mv(_tr(B), s), P + BtS @ A, R + BtS @ B)


def feedback_parameters(g, G, H, mu=REG_MU):
    """(𝛿𝐮ᶠᶠ, 𝐊) = (−H_reg⁻¹𝐠, −H_reg⁻¹𝐆), H_reg = 𝐇 + 0.01·I (:214-216; the fixed μ).
    Julia's `\\` factorises H_reg (Cholesky or pivoted LU); torch.linalg.solve is pivoted
    LU — equal to rounding."""
    as_torch = isinstance(g, torch.Tensor)
    dev = g.device if as_torch else None
    g, G, H = (_t(v, dev) for v in (g, G, H))
    n = H.shape[-1]
    H_reg = H + mu * torch.eye(n, dtype=H.dtype, device=H.device)
    return _ret(as_torch, -torch.linalg.solve(H_reg, g.unsqueeze(-1)).squeeze(-1), -torch.linalg.solve(H_reg, G))


def step_back(A, q, qv, Q, g, G, H, du, K, s_next, sv_next, S_next):
    """(𝑠, 𝐬, 𝐒) with the UNregularised 𝐇, term for term as :268-270:
    𝑠 = 𝑞 + 𝑠′ + ½𝛿𝐮ᵀ𝐇𝛿𝐮 + 𝛿𝐮ᵀ𝐠, 𝐬 = 𝐪 + 𝐀ᵀ𝐬′ + 𝐊ᵀ𝐇𝛿𝐮 + 𝐊ᵀ𝐠 + 𝐆ᵀ𝛿𝐮,
    𝐒 = 𝐐 + 𝐀ᵀ𝐒′𝐀 + 𝐊ᵀ𝐇𝐊 + 𝐊ᵀ𝐆 + 𝐆ᵀ𝐊."""
    as_torch = isinstance(A, torch.Tensor)
    dev = A.device if as_torch else None
    A, q, qv, Q, g, G, H, du, K, s_next, sv_next, S_next = (
        _t(v, dev) for v in (A, q, qv, Q, g, G, H, du, K, s_next, sv_next, S_next))
    Hdu = _mv(H, du)
    s = q + s_next + 0.5 * (du * Hdu).sum(-1) + (du * g).sum(-1)
    sv = qv + _mv(_tr(A), sv_next) + _mv(_tr(K), Hdu) + _mv(_tr(K), g) + _mv(_tr(G), du)
    S = Q + _tr(A) @ S_next @ A + _tr(K) @ H @ K + _tr(K) @ G + _tr(G) @ K
    return _ret(as_torch, s, sv, S)


__all__ = ["linearize_dynamics", "immediate_cost_quadratization", "final_cost_quadratization",
           "optimal_controller_param", "feedback_parameters", "step_back"]
