"""The Julia shim's resident single-device Solver (ilqr.jl_amd/julia/iLQRHIP.jl: Solver,
set_problem!, fit!, backward!, forward!, close; the functional fit / backward_pass /
forward_pass run on a cached one) replayed without Julia: the same C calls in the same
order on the column-major memory of the Julia arrays (tests/julia_layout.py), through a
library proxy that counts ilqr_create / ilqr_malloc / ilqr_free / ilqr_destroy.

Checks the include/ilqr.h promise "hot calls never allocate" for the MPC loop of
forward_pass.jl:148-179: 100 fits on one Solver keep the create and malloc counts
constant (the verbose history scratch is allocated once, on the first verbose call),
close() frees every buffer, and every fit is bit-equal to the per-call path
(tests/test_gpu_julia_layout.py::shim_fit, a fresh handle and buffers per call).
"""
import ctypes as C
import os

import numpy as np
import pytest

import julia_layout as J
from ilqr_amd import _lib

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


class CountingLib:
    """The loaded library with a call counter on the allocation entry points."""
    COUNTED = ("ilqr_create", "ilqr_destroy", "ilqr_malloc", "ilqr_free")

    def __init__(self):
        self.lib = _lib.load()
        self.n = dict.fromkeys(self.COUNTED, 0)

    def __getattr__(self, name):
        fn = getattr(self.lib, name)
        if name not in self.COUNTED:
            return fn

        def counted(*a):
            self.n[name] += 1
            return fn(*a)
        return counted


class ShimHandle:
    """iLQRHIP.Handle on the counting library: alloc / upload / upload! / download! /
    release! / close, in the shim's terms."""

    def __init__(self, lib, nx, nu, T, batch):
        self.lib = lib
        h = C.c_void_p()
        _lib.check(lib.ilqr_create(C.byref(h), 0, nx, nu, T, batch), "ilqr_create")
        self.h, self.bufs = h, []

    def alloc(self, dtype, n):
        p = C.c_void_p()
        _lib.check(self.lib.ilqr_malloc(self.h, max(n, 1) * np.dtype(dtype).itemsize, C.byref(p)), "ilqr_malloc")
        self.bufs.append(p.value)
        return p

    def upload_into(self, p, a, dtype=np.float64):          # upload!(h, p, a)
        buf = np.ascontiguousarray(J.memory(a).astype(dtype))
        _lib.check(self.lib.ilqr_memcpy_h2d(self.h, p, buf.ctypes.data_as(C.c_void_p), buf.nbytes), "h2d")

    def download(self, shape, p, dtype=np.float64):
        buf = np.empty(int(np.prod(shape)), dtype=dtype)
        _lib.check(self.lib.ilqr_memcpy_d2h(self.h, buf.ctypes.data_as(C.c_void_p), p, buf.nbytes), "d2h")
        return J.from_memory(buf, shape)

    def release(self, p):                                      # release!(h, p)
        self.bufs.remove(p.value)
        self.lib.ilqr_free(self.h, p)

    def close(self):                                           # Base.close(h::Handle)
        if self.h is None:
            return
        for p in self.bufs:
            self.lib.ilqr_free(self.h, C.c_void_p(p))
        self.bufs = []
        self.lib.ilqr_destroy(self.h)
        self.h = None


class ShimSolver:
    """iLQRHIP.Solver: the 17 resident buffers in the constructor's order, then
    set_problem! (LQ, one instance), fit! and close."""

    def __init__(self, lib, nx, nu, T, batch=1):
        self.hd = h = ShimHandle(lib, nx, nu, T, batch)
        self.nx, self.nu, self.M, self.nb = nx, nu, T, batch
        N = T + 1
        f = lambda n: h.alloc(np.float64, batch * n)  # noqa: E731
        i = lambda n: h.alloc(np.int32, batch * n)  # noqa: E731
        (self.A, self.B, self.Q, self.R, self.Qf) = (f(nx * nx), f(nx * nu), f(nx * nx), f(nu * nu), f(nx * nx))
        (self.x, self.u, self.xt, self.xo, self.uo) = (f(N * nx), f(T * nu), f(N * nx), f(N * nx), f(T * nu))
        (self.d, self.K, self.pc, self.cost) = (f(T * nu), f(T * nu * nx), f(1), f(1))
        (self.iters, self.status, self.trials) = (i(1), i(1), i(1))
        self.hc = self.ht = None
        self.hcap = 0

    def set_problem_lq(self, A, B, Q, R, Qf):
        for p, M in ((self.A, A), (self.B, B), (self.Q, Q), (self.R, R), (self.Qf, Qf)):
            self.hd.upload_into(p, J.rowmajor(M))
        self.prob = _lib.Problem(_lib.PROBLEM_LQ, 0, self.A.value, self.B.value, self.Q.value, self.R.value,
                                 self.Qf.value)

    def ensure_history(self, n):
        if self.hcap < n:
            if self.hc is not None:
                self.hd.release(self.hc)
                self.hd.release(self.ht)
            self.hc, self.ht = self.hd.alloc(np.float64, n * self.nb), self.hd.alloc(np.int32, n * self.nb)
            self.hcap = n
        self.hd.upload_into(self.ht, J.jl(np.zeros(n * self.nb)), dtype=np.int32)
        return _lib.History(self.hc.value, self.ht.value, None, None)

    def fit(self, x_init, u_init, x_traj, max_iter, tol, verbose=False):
        h = self.hd
        h.upload_into(self.x, J.to_abi(x_init))
        h.upload_into(self.u, J.to_abi(u_init))
        h.upload_into(self.xt, J.to_abi(x_traj))
        o = _lib.default_options(max_iter=max_iter, tol=tol)
        n = max(max_iter, 1)
        hist = self.ensure_history(n) if verbose else _lib.History(None, None, None, None)
        rc = h.lib.ilqr_fit_ex(h.h, C.byref(self.prob), C.byref(o), self.x, self.u, self.xt, self.xo, self.uo,
                               self.cost, self.iters, self.status, C.byref(hist))
        assert rc in (_lib.OK, _lib.ERR_LS_EXHAUSTED)
        out = (J.from_abi(h.download((self.nx, self.M + 1), self.xo)),
               J.from_abi(h.download((self.nu, self.M), self.uo)))
        if verbose:
            out = out + (h.download((self.nb, n), self.hc), h.download((self.nb, n), self.ht, dtype=np.int32))
        return out

    def close(self):
        self.hd.close()


def test_resident_solver_100_fits_allocate_nothing(gpu):
    from test_gpu_julia_layout import lq_problem, shim_fit
    z = np.load(os.path.join(GOLD, "dense_xtraj.npz"), allow_pickle=False)
    b = 1
    A, B, Q, R, Qf = (z[k][b] for k in ("A", "B", "Q", "R", "Qf"))
    x0, u0, xt = z["x"][b], z["u"][b], z["xtraj"][b]
    N, nx = x0.shape
    M, nu = u0.shape
    lib = CountingLib()
    s = ShimSolver(lib, nx, nu, M)
    s.set_problem_lq(A, B, Q, R, Qf)
    after_create = dict(lib.n)
    assert after_create == {"ilqr_create": 1, "ilqr_destroy": 0, "ilqr_malloc": 17, "ilqr_free": 0}
    rng = np.random.default_rng(0)
    counts = []
    for call in range(100):
        xi = x0 + 0.01 * rng.standard_normal(x0.shape)    # an MPC loop: a new start every call
        verbose = call % 10 == 3
        out = s.fit(xi, u0, xt, 30, 1e-6, verbose=verbose)
        counts.append(dict(lib.n))
        if call % 25 == 0 or verbose:
            ref = shim_fit(lambda h: lq_problem(h, A, B, Q, R, Qf), xi, u0, xt, 30, 1e-6, with_history=True)
            assert np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]), call
            if verbose:
                n = int((ref[3] > 0).sum())
                assert np.array_equal(out[3][0], ref[3])
                assert np.array_equal(out[2][0, :n], ref[2][:n], equal_nan=True)  # NaN: a failed search
    # the per-call replays above went to their own handles, not the counting proxy
    assert counts[0] == after_create
    assert all(c == counts[3] for c in counts[3:])                   # the history scratch once, at call 3
    assert counts[3]["ilqr_create"] == 1 and counts[3]["ilqr_malloc"] == 19 and counts[3]["ilqr_free"] == 0
    s.close()
    assert lib.n["ilqr_free"] == lib.n["ilqr_malloc"] == 19 and lib.n["ilqr_destroy"] == 1
    s.close()                                                        # idempotent
    assert lib.n["ilqr_destroy"] == 1
