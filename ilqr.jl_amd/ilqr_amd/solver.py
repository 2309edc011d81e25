"""Device-resident batched iLQR solver: a thin owner of one ilqr_handle.

All tensors handed to a Solver are torch CUDA (HIP) float64/int32 tensors,
contiguous, laid out as include/ilqr.h documents (trajectory slowest). Calls
are asynchronous on torch's current stream of the solver's device unless the
method says it synchronises.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .problems import LQBatch


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _req(t, dtype, shape, name):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise TypeError(f"{name}: expected a CUDA tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if tuple(t.shape) != tuple(shape):
        raise AssertionError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    return t


@dataclass
class FitResult:
    x: torch.Tensor        # (B, T+1, nx) returned iterate (reference semantics)
    u: torch.Tensor        # (B, T, nu)
    cost: torch.Tensor     # (B,) last accepted forward-pass cost
    iters: torch.Tensor    # (B,) iterations run
    status: torch.Tensor   # (B,) ILQR_TRAJ_* codes
    call_status: int       # ilqr_status of the whole call
    history: dict = None   # fit(history=True): ilqr_history arrays (max_iter, B) — "cost",
                           # "trials", "alpha", "du2" (include/ilqr.h)


def alloc_history(max_iter: int, batch: int, device):
    """Device arrays for ilqr_history, NaN / 0 filled (entries past the last iteration
    stay so), and the struct pointing at them."""
    n = max(max_iter, 1)
    h = {"cost": torch.full((n, batch), float("nan"), dtype=torch.float64, device=device),
         "trials": torch.zeros((n, batch), dtype=torch.int32, device=device),
         "alpha": torch.full((n, batch), float("nan"), dtype=torch.float64, device=device),
         "du2": torch.full((n, batch), float("nan"), dtype=torch.float64, device=device)}
    st = _lib.History(*(h[k].data_ptr() for k in ("cost", "trials", "alpha", "du2")))
    return h, st


def print_history(hist, b: int = 0):
    """The reference's per-iteration line (forward_pass.jl:167) for trajectory b."""
    tr = hist["trials"][:, b].cpu().numpy()
    c = hist["cost"][:, b].cpu().numpy()
    for i in range(len(tr)):
        if tr[i] == 0:
            break
        print(f"Iteration: {i + 1}\t\tTotal Cost: {float(c[i])!r}")  # Julia prints the shortest repr too


class Solver:
    """kind = _lib.PROBLEM_LQ (call set_problem with the per-instance data) or
    _lib.PROBLEM_TWO_LINK (the reference's 2-link arm; nothing to set)."""

    def __init__(self, nx: int, nu: int, T: int, batch: int, device: int = 0,
                 kind: int = _lib.PROBLEM_LQ, lib_path: str = None):
        # lib_path: another build of the library (the tests' variants); default the product's
        self.lib = _lib.load() if lib_path is None else _lib.load(lib_path)
        if not self.lib.ilqr_supported(kind, nx, nu):
            raise NotImplementedError(f"(nx, nu) = ({nx}, {nu}) has no compiled kernel for "
                                      f"problem kind {kind}")
        self.nx, self.nu, self.T, self.batch, self.device = nx, nu, T, batch, device
        self.kind = kind
        self.dev = torch.device("cuda", device)
        h = C.c_void_p()
        _lib.check(self.lib.ilqr_create(C.byref(h), device, nx, nu, T, batch), "ilqr_create")
        self.h = h
        self._problem = None
        self._keep = ()
        if kind == _lib.PROBLEM_TWO_LINK:
            self._problem = _lib.Problem(_lib.PROBLEM_TWO_LINK, 0, None, None, None, None, None)

    # -- setup ---------------------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.ilqr_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _bind_stream(self):
        s = torch.cuda.current_stream(self.dev).cuda_stream
        _lib.check(self.lib.ilqr_set_stream(self.h, C.c_void_p(s)), "ilqr_set_stream")

    def set_schedule(self, pipelined: bool = False, ring_forward: bool = True,
                     backward: str = "auto", fused: bool = True, forward_mfma: bool = False,
                     sequential_search: bool = False):
        """LQ launch schedule (ilqr_set_schedule). pipelined: fit overlaps half of the
        workgroups' forward passes with the other half's backward passes (implies
        backward="wave"); ring_forward: the forward pass streams its inputs HBM → LDS
        ahead of use; backward: "wave" one trajectory per wave (16x16x4 MFMA),
        "block" four per wave (4x4x4 4-block MFMA), "auto" block from 2048
        trajectories up; fused: iterate/fit run backward + forward as one kernel (with the
        "block" backward and the ring forward); forward_mfma: the ring forward's mat-vecs
        on the 4-block f64 MFMA (other rounding); sequential_search: the fused iteration's
        line search trial after trial per wave instead of the cooperative search (same
        bits, include/ilqr.h). Schedules with the same backward kernel and forward form
        return the same bits."""
        bk = {"auto": 0, "wave": _lib.SCHED_BACKWARD_WAVE, "block": _lib.SCHED_BACKWARD_BLOCK}[backward]
        flags = ((_lib.SCHED_PIPELINED if pipelined else 0) | (_lib.SCHED_RING_FORWARD if ring_forward else 0)
                 | bk | (_lib.SCHED_FUSED if fused and not pipelined and backward != "wave" else 0)
                 | (_lib.SCHED_FORWARD_MFMA if forward_mfma else 0)
                 | (_lib.SCHED_SEQUENTIAL_SEARCH if sequential_search else 0))
        _lib.check(self.lib.ilqr_set_schedule(self.h, flags), "ilqr_set_schedule")

    def set_problem(self, lq):
        """lq: LQBatch (host numpy, copied to the device) or a dict of CUDA tensors
        A (B,nx,nx), B (B,nx,nu), Q (B,nx,nx), R (B,nu,nu), Qf (B,nx,nx)."""
        if self.kind != _lib.PROBLEM_LQ:
            raise TypeError("set_problem: only the LQ family has per-instance data")
        nb, nx, nu = self.batch, self.nx, self.nu
        if isinstance(lq, LQBatch):
            t = {k: torch.from_numpy(np.require(getattr(lq, k), np.float64, ("C", "W"))).to(self.dev)
                 for k in ("A", "B", "Q", "R", "Qf")}
        else:
            t = dict(lq)
        shapes = {"A": (nb, nx, nx), "B": (nb, nx, nu), "Q": (nb, nx, nx), "R": (nb, nu, nu),
                  "Qf": (nb, nx, nx)}
        for k, s in shapes.items():
            _req(t[k], torch.float64, s, k)
        self._keep = tuple(t[k] for k in shapes)
        self._problem = _lib.Problem(_lib.PROBLEM_LQ, 0, *(t[k].data_ptr() for k in shapes))

    def _p(self):
        if self._problem is None:
            raise RuntimeError("set_problem() first")
        return C.byref(self._problem)

    def alloc_traj(self, zero=True):
        f = torch.zeros if zero else torch.empty
        return (f((self.batch, self.T + 1, self.nx), dtype=torch.float64, device=self.dev),
                f((self.batch, self.T, self.nu), dtype=torch.float64, device=self.dev))

    # -- passes ----------------------------------------------------------------------
    def backward(self, x, u, mu=None):
        """iLQR.backward_pass for the batch → (d (B,T,nu), K (B,T,nu,nx), status (B,)).
        Synchronises (folds the per-trajectory NaN status)."""
        B, T, nx, nu = self.batch, self.T, self.nx, self.nu
        _req(x, torch.float64, (B, T + 1, nx), "x")
        _req(u, torch.float64, (B, T, nu), "u")
        d = torch.empty((B, T, nu), dtype=torch.float64, device=self.dev)
        K = torch.empty((B, T, nu, nx), dtype=torch.float64, device=self.dev)
        st = torch.empty((B,), dtype=torch.int32, device=self.dev)
        self._bind_stream()
        o = _lib.default_options(mu=mu)
        rc = self.lib.ilqr_backward(self.h, self._p(), C.byref(o), _ptr(x), _ptr(u), _ptr(d),
                                    _ptr(K), _ptr(st))
        _lib.check(rc, "ilqr_backward", allow=(_lib.ERR_NAN,))
        return d, K, st

    def backward_tiles(self, tiles, mu=None):
        """iLQR.backward_pass on caller-supplied derivative tiles (ilqr_backward_tiles):
        `tiles` maps ilqr_tiles' field names to CUDA float64 tensors (lux may be None)
        → (d, K, status). Synchronises."""
        B, T, nx, nu = self.batch, self.T, self.nx, self.nu
        shapes = {"A": (B, T, nx, nx), "B": (B, T, nx, nu), "lx": (B, T, nx), "lu": (B, T, nu),
                  "lxx": (B, T, nx, nx), "lux": (B, T, nu, nx), "luu": (B, T, nu, nu),
                  "lfx": (B, nx), "lfxx": (B, nx, nx)}
        for k, shp in shapes.items():
            if k == "lux" and tiles.get(k) is None:
                continue
            _req(tiles[k], torch.float64, shp, k)
        tl = _lib.Tiles(*(None if tiles.get(k) is None else tiles[k].data_ptr() for k in shapes))
        d = torch.empty((B, T, nu), dtype=torch.float64, device=self.dev)
        K = torch.empty((B, T, nu, nx), dtype=torch.float64, device=self.dev)
        st = torch.empty((B,), dtype=torch.int32, device=self.dev)
        self._bind_stream()
        o = _lib.default_options(mu=mu)
        rc = self.lib.ilqr_backward_tiles(self.h, C.byref(tl), C.byref(o), _ptr(d), _ptr(K), _ptr(st))
        _lib.check(rc, "ilqr_backward_tiles", allow=(_lib.ERR_NAN,))
        return d, K, st

    def forward(self, x, u, d, K, prev_cost, x_traj=None, alpha0=None, shrink=None,
                max_trials=None):
        """iLQR.forward_pass for the batch → (x_new, u_new, new_cost, trials, status).
        Synchronises."""
        B, T, nx, nu = self.batch, self.T, self.nx, self.nu
        _req(x, torch.float64, (B, T + 1, nx), "x")
        _req(u, torch.float64, (B, T, nu), "u")
        _req(d, torch.float64, (B, T, nu), "d")
        _req(K, torch.float64, (B, T, nu, nx), "K")
        _req(prev_cost, torch.float64, (B,), "prev_cost")
        if x_traj is not None:
            _req(x_traj, torch.float64, (B, T + 1, nx), "x_traj")
        xn, un = self.alloc_traj(zero=False)
        cost = torch.empty((B,), dtype=torch.float64, device=self.dev)
        trials = torch.empty((B,), dtype=torch.int32, device=self.dev)
        st = torch.empty((B,), dtype=torch.int32, device=self.dev)
        self._bind_stream()
        o = _lib.default_options(alpha0=alpha0, shrink=shrink, max_trials=max_trials)
        rc = self.lib.ilqr_forward(self.h, self._p(), C.byref(o), _ptr(x), _ptr(u), _ptr(x_traj),
                                   _ptr(d), _ptr(K), _ptr(prev_cost), _ptr(xn), _ptr(un),
                                   _ptr(cost), _ptr(trials), _ptr(st))
        _lib.check(rc, "ilqr_forward", allow=(_lib.ERR_NAN, _lib.ERR_LS_EXHAUSTED))
        return xn, un, cost, trials, st

    def rollout(self, x0, u):
        """Open-loop rollout x[t+1] = dynamicsf(x[t], u[t]) from x0 (B, nx) —
        animate_2_link.jl:11-16's x_init — as forward_pass with δu = K = 0 (its
        first trial at prev_cost = Inf is exactly that rollout). Synchronises."""
        B, T, nx, nu = self.batch, self.T, self.nx, self.nu
        _req(x0, torch.float64, (B, nx), "x0")
        _req(u, torch.float64, (B, T, nu), "u")
        x = torch.zeros((B, T + 1, nx), dtype=torch.float64, device=self.dev)
        x[:, 0] = x0
        d = torch.zeros((B, T, nu), dtype=torch.float64, device=self.dev)
        K = torch.zeros((B, T, nu, nx), dtype=torch.float64, device=self.dev)
        pc = torch.full((B,), float("inf"), dtype=torch.float64, device=self.dev)
        xn, _, _, _, _ = self.forward(x, u, d, K, pc)
        return xn

    def iterate(self, x, u, x_new, u_new, prev_cost, status, du2=None, trials=None,
                x_traj=None, options=None, new_cost=None):
        """One fit iteration (backward + forward + convergence test), asynchronous.
        prev_cost None = +Inf (cold start); new_cost defaults to prev_cost (in
        place, fit semantics). No shape checks beyond the ABI's: the bench's hot loop."""
        o = options if options is not None else _lib.default_options()
        nc = new_cost if new_cost is not None else prev_cost
        rc = self.lib.ilqr_iterate(self.h, self._p(), C.byref(o), _ptr(x), _ptr(u), _ptr(x_traj),
                                   _ptr(x_new), _ptr(u_new), _ptr(prev_cost), _ptr(nc),
                                   _ptr(du2), _ptr(trials), _ptr(status))
        _lib.check(rc, "ilqr_iterate")

    def fit(self, x_init, u_init, x_traj=None, max_iter=100, tol=1e-6, mu=None,
            max_trials=None, history: bool = False) -> FitResult:
        """iLQR.fit for the batch (synchronises). history: also return the per-iteration
        record (ilqr_fit_ex; FitResult.history)."""
        if not isinstance(max_iter, int):
            raise TypeError("max_iter::Int64")  # forward_pass.jl:152
        B, T, nx, nu = self.batch, self.T, self.nx, self.nu
        _req(x_init, torch.float64, (B, T + 1, nx), "x_init")
        _req(u_init, torch.float64, (B, T, nu), "u_init")
        if x_traj is not None:
            _req(x_traj, torch.float64, (B, T + 1, nx), "x_traj")
        xo, uo = self.alloc_traj(zero=False)
        cost = torch.empty((B,), dtype=torch.float64, device=self.dev)
        iters = torch.empty((B,), dtype=torch.int32, device=self.dev)
        st = torch.empty((B,), dtype=torch.int32, device=self.dev)
        self._bind_stream()
        o = _lib.default_options(max_iter=max_iter, tol=float(tol), mu=mu, max_trials=max_trials)
        hist, hst = alloc_history(max_iter, B, self.dev) if history else (None, None)
        rc = self.lib.ilqr_fit_ex(self.h, self._p(), C.byref(o), _ptr(x_init), _ptr(u_init),
                                  _ptr(x_traj), _ptr(xo), _ptr(uo), _ptr(cost), _ptr(iters), _ptr(st),
                                  C.byref(hst) if hst is not None else None)
        _lib.check(rc, "ilqr_fit", allow=(_lib.ERR_NAN, _lib.ERR_LS_EXHAUSTED))
        return FitResult(xo, uo, cost, iters, st, rc, hist)


def selftest(device: int = 0) -> int:
    lib = _lib.load()
    f = C.c_int32(-1)
    _lib.check(lib.ilqr_selftest(device, C.byref(f)), "ilqr_selftest")
    return f.value
