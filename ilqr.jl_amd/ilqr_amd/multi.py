"""Single-process multi-GPU fit (ilqr_multi_* in include/ilqr.h):
the batch is sharded in contiguous blocks over the given devices, each shard runs
ilqr_fit concurrently on its own device (one host thread per device inside the
library). `fit`: host numpy in, host numpy out — what a single-process host (the Julia
shim's solve!) hands over, every array crossing PCIe on every call. The resident calls
(`set_problem`, `load`, `fit_resident`, `gather`) keep problem and trajectories on the
devices between calls (an MPC loop). The one-process-per-GPU path with
torch.distributed is ilqr_amd.dist."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .problems import LQBatch


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _host(a, dtype=np.float64):
    return np.require(a, dtype, ("C", "W"))


class MultiSolver:
    def __init__(self, devices, nx: int, nu: int, T: int, batch: int):
        self.lib = _lib.load()
        self.nx, self.nu, self.T, self.batch = nx, nu, T, batch
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        _lib.check(self.lib.ilqr_multi_create(C.byref(h), devs, len(devices), nx, nu, T, batch),
                   "ilqr_multi_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.ilqr_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_schedule(self, pipelined: bool = False, ring_forward: bool = True, backward: str = "auto",
                     fused: bool = True, forward_mfma: bool = False,
                     sequential_search: bool = False):
        """As Solver.set_schedule, on every device's handle."""
        bk = {"auto": 0, "wave": _lib.SCHED_BACKWARD_WAVE, "block": _lib.SCHED_BACKWARD_BLOCK}[backward]
        flags = ((_lib.SCHED_PIPELINED if pipelined else 0) | (_lib.SCHED_RING_FORWARD if ring_forward else 0)
                 | bk | (_lib.SCHED_FUSED if fused and not pipelined and backward != "wave" else 0)
                 | (_lib.SCHED_FORWARD_MFMA if forward_mfma else 0)
                 | (_lib.SCHED_SEQUENTIAL_SEARCH if sequential_search else 0))
        _lib.check(self.lib.ilqr_multi_set_schedule(self.h, flags), "ilqr_multi_set_schedule")

    def fit(self, lq: LQBatch, x_init, u_init, x_traj=None, max_iter=100, tol=1e-6, mu=None,
            max_trials=None):
        """→ (x, u, cost, iters, status, call_status), numpy, whole batch."""
        if not isinstance(max_iter, int):
            raise TypeError("max_iter::Int64")  # forward_pass.jl:152
        B, T, nx, nu = self.batch, self.T, self.nx, self.nu
        x_init, u_init = _host(x_init), _host(u_init)
        if x_init.shape != (B, T + 1, nx) or u_init.shape != (B, T, nu):
            raise AssertionError("size(x_init)[2] == size(u_init)[1] + 1")  # forward_pass.jl:156
        arrs = {k: _host(getattr(lq, k)) for k in ("A", "B", "Q", "R", "Qf")}
        prob = _lib.Problem(_lib.PROBLEM_LQ, 0, *(arrs[k].ctypes.data for k in ("A", "B", "Q", "R", "Qf")))
        xt = None if x_traj is None else _host(x_traj)
        xo, uo = np.empty_like(x_init), np.empty_like(u_init)
        cost = np.empty(B)
        iters = np.empty(B, dtype=np.int32)
        st = np.empty(B, dtype=np.int32)
        o = _lib.default_options(max_iter=max_iter, tol=float(tol), mu=mu, max_trials=max_trials)
        rc = self.lib.ilqr_multi_fit(self.h, C.byref(prob), C.byref(o), _ptr(x_init), _ptr(u_init),
                                     _ptr(xt), _ptr(xo), _ptr(uo), _ptr(cost), _ptr(iters), _ptr(st))
        _lib.check(rc, "ilqr_multi_fit", allow=(_lib.ERR_NAN, _lib.ERR_LS_EXHAUSTED))
        return xo, uo, cost, iters, st, rc

    # -- device-resident calls -------------------------------------------------------
    def set_problem(self, lq: LQBatch = None, kind: int = _lib.PROBLEM_LQ):
        """Upload the per-instance problem once (ilqr_multi_set_problem)."""
        if kind == _lib.PROBLEM_LQ:
            self._arrs = {k: _host(getattr(lq, k)) for k in ("A", "B", "Q", "R", "Qf")}
            prob = _lib.Problem(kind, 0, *(self._arrs[k].ctypes.data for k in ("A", "B", "Q", "R", "Qf")))
        else:
            prob = _lib.Problem(kind, 0, None, None, None, None, None)
        _lib.check(self.lib.ilqr_multi_set_problem(self.h, C.byref(prob)), "ilqr_multi_set_problem")

    def load(self, x=None, u=None, x_traj=None):
        """Upload trajectories (host numpy; None keeps what the devices hold)."""
        B, T, nx, nu = self.batch, self.T, self.nx, self.nu
        a = [None if v is None else _host(v) for v in (x, u, x_traj)]
        for v, shp in zip(a, ((B, T + 1, nx), (B, T, nu), (B, T + 1, nx))):
            if v is not None and v.shape != shp:
                raise AssertionError(f"expected {shp}, got {v.shape}")
        _lib.check(self.lib.ilqr_multi_load(self.h, *(_ptr(v) for v in a)), "ilqr_multi_load")

    def fit_resident(self, max_iter=100, tol=1e-6, warm_start=False, use_x_traj=False, history=None):
        """Fit from the resident trajectories (or the previous result) into resident
        results; nothing crosses PCIe. history: a solver.alloc_history struct (device
        arrays (max_iter, batch)) or None. → call status."""
        if not isinstance(max_iter, int):
            raise TypeError("max_iter::Int64")
        o = _lib.default_options(max_iter=max_iter, tol=float(tol))
        flags = (_lib.MULTI_WARM_START if warm_start else 0) | (_lib.MULTI_USE_X_TRAJ if use_x_traj else 0)
        rc = self.lib.ilqr_multi_fit_resident(self.h, C.byref(o), flags,
                                              C.byref(history) if history is not None else None)
        return _lib.check(rc, "ilqr_multi_fit_resident", allow=(_lib.ERR_NAN, _lib.ERR_LS_EXHAUSTED))

    def gather(self, x=True, u=True, cost=True, iters=True, status=True, out=None):
        """Copy the last fit's results to host (only the fields asked for). `out`: a dict
        of preallocated (pinned, see HostBuffers) arrays to fill instead of new ones."""
        B, T, nx, nu = self.batch, self.T, self.nx, self.nu
        shapes = {"x": ((B, T + 1, nx), np.float64), "u": ((B, T, nu), np.float64), "cost": ((B,), np.float64),
                  "iters": ((B,), np.int32), "status": ((B,), np.int32)}
        want = {"x": x, "u": u, "cost": cost, "iters": iters, "status": status}
        res = {}
        for k, (shp, dt) in shapes.items():
            if want[k]:
                res[k] = out[k] if out is not None and k in out else np.empty(shp, dtype=dt)
        _lib.check(self.lib.ilqr_multi_gather(self.h, *(_ptr(res.get(k)) for k in shapes)), "ilqr_multi_gather")
        return res


class HostBuffers:
    """Pinned host arrays (ilqr_host_alloc) for MultiSolver.gather / load: PCIe at
    full rate instead of the driver's pageable staging."""

    def __init__(self, **shapes):
        self.lib = _lib.load()
        self._ptrs, self.arrays = [], {}
        for k, (shape, dtype) in shapes.items():
            n = int(np.prod(shape)) * np.dtype(dtype).itemsize
            p = C.c_void_p()
            _lib.check(self.lib.ilqr_host_alloc(n, C.byref(p)), "ilqr_host_alloc")
            self._ptrs.append(p)
            buf = (C.c_char * n).from_address(p.value)
            self.arrays[k] = np.frombuffer(buf, dtype=dtype).reshape(shape)

    def close(self):
        self.arrays = {}
        for p in self._ptrs:
            self.lib.ilqr_host_free(p)
        self._ptrs = []
