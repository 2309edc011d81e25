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
(batched over trajectories, sequential over time), not in a HIP kernel. One step of it
(control law :72-73 + dynamics :74) is captured once per (closure, shape) in a HIP
graph and replayed T times per line-search trial: a closure of a few hundred small ops
(the reference's RBD caller) then costs one graph launch per step instead of a few
hundred dispatches (tools/archive/r05/rollout_probe.py: 4.0 → 0.73 ms per step at nx = 16, B = 1).
The capture is checked against an eager step bit for bit before it is used, and again
at the start of EVERY later forward_pass on the cached graph: a replay freezes what the
closure read from Python when it was captured (a rebound global or attribute, a changed
target or Δt), where the reference calls dynamicsf afresh at every step, so a replay
that no longer equals the eager step is captured again (and the closure runs eagerly if
that fails). Closures that cannot be captured (a host synchronisation inside them) run
eagerly. The graphs' static buffers are bounded (MAX_GRAPH_BYTES in all, oldest evicted)
and released by ilqr_amd.api.clear_cache(). ILQR_ROLLOUT_GRAPH=0 turns the graphs off.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref

import torch
from torch.overrides import TorchFunctionMode

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


ROLLOUT_GRAPHS = os.environ.get("ILQR_ROLLOUT_GRAPH", "1") != "0"
MAX_GRAPHS_PER_CLOSURE = 4
MAX_GRAPH_BYTES = int(os.environ.get("ILQR_ROLLOUT_GRAPH_BYTES", str(2 << 30)))  # all graphs' buffers
_GRAPHS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()  # dynamicsf → {shape: graph}
_GRAPHS_LOCK = threading.Lock()
_CAPTURE_LOCK = threading.Lock()


class _CapturableLinalg(TorchFunctionMode):
    """torch.linalg.solve / inv check their LAPACK info on the host, which a capture
    forbids; inside the capture they run as solve_ex / inv_ex (the same kernels without
    the check: a singular system then gives non-finite states, reported as a NaN
    trajectory, where the eager call raises). A torch-function mode is per thread: other
    threads' calls are untouched."""

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = dict(kwargs or {})
        if func is torch.linalg.solve and "out" not in kwargs:
            return torch.linalg.solve_ex(*args, **kwargs)[0]
        if func is torch.linalg.inv and "out" not in kwargs:
            return torch.linalg.inv_ex(*args, **kwargs)[0]
        return func(*args, **kwargs)


def _capturable_linalg():
    return _CapturableLinalg()


class _RolloutGraph:
    """forward_pass's step (:72-74) on static buffers, the step index on the device:
    XB[:, k+1] = f(XB[:, k], U[:, k] + α·D[:, k] + K[:, k]·(XB[:, k] − X[:, k]))."""

    def __init__(self, x, u):
        dev = x.device
        nb, N, nx = x.shape
        nu = u.shape[2]
        self.X, self.U = torch.empty_like(x), torch.empty_like(u)
        self.D = torch.empty_like(u)
        self.K = torch.empty((nb, N - 1, nu, nx), dtype=x.dtype, device=dev)
        self.alpha = torch.empty(nb, dtype=torch.float64, device=dev)
        self.XB, self.UB = torch.empty_like(x), torch.empty_like(u)
        self.k = torch.zeros(1, dtype=torch.long, device=dev)
        self.graph = None
        self.lock = threading.Lock()
        self.seq = 0  # last use (eviction order)
        self.nbytes = sum(t.numel() * t.element_size() for t in (self.X, self.U, self.D, self.K, self.XB, self.UB))

    def step(self, f):
        k = self.k
        k1 = k + 1
        xk = self.XB.index_select(1, k).squeeze(1)
        dx = xk - self.X.index_select(1, k).squeeze(1)                              # :72
        uk = (self.U.index_select(1, k).squeeze(1) + self.alpha[:, None] * self.D.index_select(1, k).squeeze(1)) \
            + torch.einsum("bij,bj->bi", self.K.index_select(1, k).squeeze(1), dx)  # :73
        xn = f(xk, uk)                                                              # :74
        self.UB.index_copy_(1, k, uk.unsqueeze(1))
        self.XB.index_copy_(1, k1, xn.unsqueeze(1))
        self.k.add_(1)

    def load(self, x, u, d, K):
        for dst, src in ((self.X, x), (self.U, u), (self.D, d), (self.K, K)):
            dst.copy_(src)

    def start(self, alpha):
        self.alpha.copy_(alpha)
        self.XB[:, 0] = self.X[:, 0]                                                # :65
        self.k.zero_()

    def capture(self, f):
        """Warm up on a side stream, capture, then replay step 0 and compare it with an
        eager step 0 bit for bit. → True when the graph can be used."""
        self.start(torch.ones_like(self.alpha))
        side = torch.cuda.Stream(device=self.X.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                self.k.zero_()
                self.step(f)
        torch.cuda.current_stream().wait_stream(side)
        self.start(torch.ones_like(self.alpha))
        self.step(f)                                                                # the eager reference
        want_x, want_u = self.XB[:, 1].clone(), self.UB[:, 0].clone()
        g = torch.cuda.CUDAGraph()
        self.start(torch.ones_like(self.alpha))
        torch.cuda.synchronize()
        # begin/end by hand rather than torch.cuda.graph: a failed capture must still end
        # it and restore this thread's stream (the context manager skips both when
        # capture_end raises), then clear the runtime's last error before eager work
        with _CAPTURE_LOCK, _capturable_linalg(), torch.cuda.stream(side):
            g.capture_begin(capture_error_mode="thread_local")
            try:
                self.step(f)
            finally:
                try:
                    g.capture_end()
                except Exception:
                    _clear_hip_error()
                    raise
        torch.cuda.synchronize()
        self.start(torch.ones_like(self.alpha))
        g.replay()
        ok = bool(torch.equal(self.XB[:, 1], want_x)) and bool(torch.equal(self.UB[:, 0], want_u)) \
            and int(self.k.item()) == 1
        self.graph = g if ok else None
        return ok

    def still_valid(self, f):
        """Replay step 0 and an eager step 0 on the loaded inputs (α = 1): equal bit for bit
        when the closure still computes what was captured."""
        self.start(torch.ones_like(self.alpha))
        self.step(f)
        want_x, want_u = self.XB[:, 1].clone(), self.UB[:, 0].clone()
        self.start(torch.ones_like(self.alpha))
        self.graph.replay()
        return bool(torch.equal(self.XB[:, 1], want_x)) and bool(torch.equal(self.UB[:, 0], want_u))


def _clear_hip_error():
    """Reset the HIP runtime's per-thread last error that an invalidated capture leaves
    (torch reports it at the next kernel launch otherwise)."""
    try:
        hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch already loaded (same soname)
        hip.hipGetLastError()
    except OSError:
        pass


def _graph_bytes():
    return sum(g.nbytes for per in list(_GRAPHS.values()) for g in per.values() if g)


def _evict_for(nbytes):
    """Drop the oldest cached graphs (any closure) until nbytes more fit under
    MAX_GRAPH_BYTES. Caller holds _GRAPHS_LOCK."""
    while _graph_bytes() + nbytes > MAX_GRAPH_BYTES:
        victim = None
        for per in list(_GRAPHS.values()):
            for key, g in per.items():
                if g and not g.lock.locked() and (victim is None or g.seq < victim[2].seq):
                    victim = (per, key, g)
        if victim is None:
            return False
        del victim[0][victim[1]]
    return True


_SEQ = [0]


def clear_graphs():
    """Release every cached rollout graph and its static buffers (ilqr_amd.api.clear_cache)."""
    with _GRAPHS_LOCK:
        _GRAPHS.clear()


def _rollout_graph(dynamicsf, x, u):
    """The cached captured step for (dynamicsf, shape), capturing on first use; None
    when graphs are off, the closure cannot be cached or captured, or its buffers would
    not fit under MAX_GRAPH_BYTES."""
    if not (ROLLOUT_GRAPHS and x.is_cuda):
        return None
    key = (tuple(x.shape), tuple(u.shape), x.dtype, x.device.index)
    nb, N, nx = x.shape
    need = 8 * (2 * nb * N * nx + 3 * nb * (N - 1) * u.shape[2] + nb * (N - 1) * u.shape[2] * nx)
    try:
        with _GRAPHS_LOCK:
            per = _GRAPHS.setdefault(dynamicsf, {})
            g = per.get(key)
            if g is None:
                if len(per) >= MAX_GRAPHS_PER_CLOSURE:
                    per.pop(next(iter(per)))
                if not _evict_for(need):
                    return None
                g = per[key] = _RolloutGraph(x, u)  # holds no reference to the closure
            if g:
                _SEQ[0] += 1
                g.seq = _SEQ[0]
    except TypeError:  # not weak-referenceable
        return None
    return g or None  # False: this closure failed to capture at this shape


def _mark_uncapturable(dynamicsf, x, u):
    key = (tuple(x.shape), tuple(u.shape), x.dtype, x.device.index)
    with _GRAPHS_LOCK:
        _GRAPHS.setdefault(dynamicsf, {})[key] = False


def _rollout_eager(f, x, u, d, K, alpha):
    xb = torch.empty_like(x)
    ub = torch.empty_like(u)
    xb[:, 0] = x[:, 0]                                                          # :65
    for k in range(x.shape[1] - 1):                                             # :71
        dx = xb[:, k] - x[:, k]                                                 # :72
        ub[:, k] = (u[:, k] + alpha[:, None] * d[:, k]) + torch.einsum("bij,bj->bi", K[:, k], dx)  # :73
        xb[:, k + 1] = f(xb[:, k], ub[:, k])                                    # :74
    return xb, ub


def rollout_forward(x, u, x_traj, d, K, prev_cost, dynamicsf, immediate_cost, final_cost,
                    max_trials=64, alpha0=1.0, shrink=0.5):
    """forward_pass (src/forward_pass.jl:55-93) for torch closures, batched over
    trajectories; each trajectory keeps its own α. → (x̄, ū, cost, trials, accepted)."""
    from torch.func import vmap
    f = vmap(dynamicsf)
    nb, N, nx = x.shape
    T = N - 1
    g = _rollout_graph(dynamicsf, x, u)
    if g is None:
        return _line_search(x, u, x_traj, prev_cost, immediate_cost, final_cost, max_trials, alpha0, shrink,
                            lambda alpha: _rollout_eager(f, x, u, d, K, alpha))
    with g.lock:
        g.load(x, u, d, K)
        if g.graph is not None and not g.still_valid(f):
            g.graph = None        # the closure changed since the capture: capture again
        if g.graph is None:
            try:
                g.capture(f)
            except Exception:  # a host synchronisation (or another capture error) in the closure
                g.graph = None
                _clear_hip_error()
                torch.cuda.synchronize()
            if g.graph is None:
                _mark_uncapturable(dynamicsf, x, u)
                return _line_search(x, u, x_traj, prev_cost, immediate_cost, final_cost, max_trials, alpha0,
                                    shrink, lambda alpha: _rollout_eager(f, x, u, d, K, alpha))

        def graphed(alpha):
            g.start(alpha)
            for _ in range(T):
                g.graph.replay()
            return g.XB.clone(), g.UB.clone()
        return _line_search(x, u, x_traj, prev_cost, immediate_cost, final_cost, max_trials, alpha0, shrink,
                            graphed)


def _line_search(x, u, x_traj, prev_cost, immediate_cost, final_cost, max_trials, alpha0, shrink, rollout):
    nb = x.shape[0]
    xo, uo = x.clone(), u.clone()
    cost = torch.full((nb,), float("nan"), dtype=torch.float64, device=x.device)
    trials = torch.zeros(nb, dtype=torch.int32, device=x.device)
    done = torch.zeros(nb, dtype=torch.bool, device=x.device)
    alpha = torch.full((nb,), float(alpha0), dtype=torch.float64, device=x.device)
    for trial in range(1, max_trials + 1):
        xb, ub = rollout(alpha)                                                 # :65-75
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
