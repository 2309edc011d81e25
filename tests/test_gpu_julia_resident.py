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
    COUNTED = ("ilqr_create", "ilqr_destroy", "ilqr_malloc", "ilqr_free", "ilqr_floating_create",
               "ilqr_floating_destroy")

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
    assert after_create == {"ilqr_create": 1, "ilqr_destroy": 0, "ilqr_malloc": 17, "ilqr_free": 0,
                            "ilqr_floating_create": 0, "ilqr_floating_destroy": 0}
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


# -- the arbitrary-closure path: iLQRHIP.fit → fit_tiles → backward_tiles_device ---------
class ShimTilesSolver:
    """iLQRHIP.TilesSolver: one handle and the 12 resident buffers in the constructor's
    order (A B lx lu lxx lux luu lfx lfxx, then δu K status)."""

    def __init__(self, lib, nx, nu, T):
        self.hd = h = ShimHandle(lib, nx, nu, T, 1)
        self.nx, self.nu, self.M = nx, nu, T
        f = lambda n: h.alloc(np.float64, n)  # noqa: E731
        self.tl = [f(T * nx * nx), f(T * nx * nu), f(T * nx), f(T * nu), f(T * nx * nx),
                   f(T * nu * nx), f(T * nu * nu), f(nx), f(nx * nx)]
        self.d, self.K, self.status = f(T * nu), f(T * nu * nx), h.alloc(np.int32, 1)

    def close(self):
        self.hd.close()


def julia_tiles(x, u, fj, quad, fquad):
    """iLQRHIP.derivative_tiles' Julia arrays — A (nx, nx, M) with A[:, :, i] =
    permutedims(jacobian), lx (nx, M), … — from the oracle's forward-mode Jacobians and
    the exact cost quadratizations (ForwardDiff's values; Julia's own call per step)."""
    from oracle import jet
    M = u.shape[0]
    A, B = jet.jacobians(fj, x[:M], u)
    lx, lu, lxx, lux, luu = quad(x[:M], u)
    lfx, lfxx = fquad(x[M:M + 1])
    stepT = lambda a: J.jl(np.transpose(a, (2, 1, 0)))   # (M, r, c) → Julia (c, r, M)  # noqa: E731
    return [stepT(A), stepT(B), J.jl(lx.T), J.jl(lu.T), stepT(lxx), stepT(lux), stepT(luu),
            J.jl(lfx[0]), J.jl(lfxx[0].T)]


def shim_backward_tiles(cache, lib, x, u, fj, quad, fquad):
    """iLQRHIP.backward_tiles_device: the host tiles into the cached TilesSolver's buffers
    (with_cached(TILES_CACHE, …)), ilqr_backward_tiles, download."""
    M, nu = u.shape
    nx = x.shape[1]
    t = julia_tiles(x, u, fj, quad, fquad)
    s = cache.get((nx, nu, M))
    if s is None:
        s = cache[(nx, nu, M)] = ShimTilesSolver(lib, nx, nu, M)
    for p, a in zip(s.tl, t):
        s.hd.upload_into(p, a)
    tl = _lib.Tiles(*(p.value for p in s.tl))
    o = _lib.default_options()
    rc = lib.ilqr_backward_tiles(s.hd.h, C.byref(tl), C.byref(o), s.d, s.K, s.status)
    _lib.check(rc, "ilqr_backward_tiles")
    return (J.from_abi(s.hd.download((nu, M), s.d)), J.gains_from_abi(s.hd.download((nx, nu, M), s.K)))


def shim_fit_tiles(cache, lib, x_init, u_init, fj, lj, lfj, quad, fquad, max_iter, tol, max_trials=64):
    """iLQRHIP.fit_tiles with forward_host: the host rollout of the user's closure."""
    xi, ui = np.array(x_init), np.array(u_init)
    xt = np.zeros_like(xi)
    prev = np.inf
    iters = 0
    for it in range(1, max_iter + 1):
        iters = it
        du, K = shim_backward_tiles(cache, lib, xi, ui, fj, quad, fquad)           # :162
        N, M = xi.shape[0], ui.shape[0]
        alpha, xb, ub, exhausted = 1.0, np.zeros_like(xi), np.zeros_like(ui), False
        for trial in range(1, max_trials + 1):
            xb[0] = xi[0]
            for k in range(M):
                ub[k] = ui[k] + alpha * du[k] + K[k] @ (xb[k] - xi[k])
                xb[k + 1] = fj(xb[k][None], ub[k][None])[0]
            c = sum(float(lj((xb[k] - xt[k])[None], ub[k][None])[0]) for k in range(M)) + float(lfj(xb[M][None])[0])
            if prev - c > 0:
                break
            if trial == max_trials:
                exhausted = True
            alpha /= 2
        if exhausted:
            break
        prev = c
        if float(((ub - ui) ** 2).sum()) <= tol:                                   # :171
            break
        xi, ui = xb.copy(), ub.copy()
    return xi, ui, iters


def test_tiles_path_20_fits_allocate_nothing_rbd_shape(gpu):
    """iLQRHIP.fit with the reference RBD example's closures (nx = 16, nu = 8, T = 1000):
    the tiles workspace is created once (1 handle, 12 buffers) and reused by every
    iteration of 20 MPC-style fits; results agree with the batched closure oracle."""
    from closures import jet_ns, rbd_cost_quads, rbd_floating_arm, rbd_initial_state
    from oracle import closure_fit as CF
    fj, lj, lfj = rbd_floating_arm(jet_ns())
    quad, fquad = rbd_cost_quads()
    T = 1000
    lib = CountingLib()
    cache = {}
    rng = np.random.default_rng(11)
    u0 = np.zeros((T, 8))
    counts = []
    for call in range(20):
        x0 = rbd_initial_state()
        x0[8:] = 0.02 * rng.standard_normal(8)
        x = np.zeros((T + 1, 16))
        x[0] = x0
        for t in range(T):
            x[t + 1] = fj(x[t][None], u0[t][None])[0]
        max_iter = 3 if call == 19 else 1
        xo, uo, iters = shim_fit_tiles(cache, lib, x, u0, fj, lj, lfj, quad, fquad, max_iter, 1e-6)
        counts.append(dict(lib.n))
        if call in (0, 19):
            r = CF.fit(x[None], u0[None], fj, lj, lfj, quad, fquad, max_iter=max_iter, tol=1e-6)
            assert iters == int(r["iters"][0])
            assert rel(xo, r["x"][0]) < 1e-8 and rel(uo, r["u"][0]) < 1e-8
    assert counts[0] == {"ilqr_create": 1, "ilqr_destroy": 0, "ilqr_malloc": 12, "ilqr_free": 0,
                         "ilqr_floating_create": 0, "ilqr_floating_destroy": 0}
    assert all(c == counts[0] for c in counts)
    for s in cache.values():
        s.close()
    assert lib.n["ilqr_free"] == 12 and lib.n["ilqr_destroy"] == 1


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


# -- the floating-base family: iLQRHIP.fit with FloatingDynamics / FloatingCost /
# FloatingFinalCost → floating_fit1 on the cached FloatingSolver (floating_cached) --------
class ShimFloatingSolver:
    """iLQRHIP.FloatingSolver: ilqr_floating_create, then the helper Handle and its 12
    buffers in the constructor's order (x u x_traj x̄ ū, δu K prev_cost cost, iters status
    trials); close = ilqr_floating_destroy + the Handle's close (destroy!)."""

    def __init__(self, lib, model, T, nb):
        self.lib = lib
        fh = C.c_void_p()
        _lib.check(lib.ilqr_floating_create(C.byref(fh), 0, C.byref(model), T, nb), "ilqr_floating_create")
        self.fh = fh
        nu = 6 + model.n_joints
        nx = 2 * nu
        self.nx, self.nu, self.M, self.nb = nx, nu, T, nb
        self.hd = h = ShimHandle(lib, nx, nu, T, 1)
        N = T + 1
        f = lambda n: h.alloc(np.float64, nb * n)  # noqa: E731
        i = lambda n: h.alloc(np.int32, nb * n)  # noqa: E731
        (self.x, self.u, self.xt, self.xo, self.uo) = (f(N * nx), f(T * nu), f(N * nx), f(N * nx), f(T * nu))
        (self.d, self.K, self.pc, self.cost) = (f(T * nu), f(T * nu * nx), f(1), f(1))
        (self.iters, self.status, self.trials) = (i(1), i(1), i(1))

    def fit1(self, x_init, u_init, x_traj, max_iter, tol):
        """iLQRHIP.floating_fit1 (verbose = false): the reference-layout trajectory in, fit."""
        h = self.hd
        h.upload_into(self.x, J.to_abi(x_init))
        h.upload_into(self.u, J.to_abi(u_init))
        h.upload_into(self.xt, J.to_abi(x_traj))
        o = _lib.default_options(max_iter=max_iter, tol=tol)
        rc = self.lib.ilqr_floating_fit_ex(self.fh, C.byref(o), self.x, self.u, self.xt, self.xo, self.uo,
                                           self.cost, self.iters, self.status,
                                           C.byref(_lib.History(None, None, None, None)))
        assert rc in (_lib.OK, _lib.ERR_LS_EXHAUSTED)
        return (J.from_abi(h.download((self.nx, self.M + 1), self.xo)),
                J.from_abi(h.download((self.nu, self.M), self.uo)))

    def close(self):
        if self.fh is not None:
            self.lib.ilqr_floating_destroy(self.fh)
            self.fh = None
        self.hd.close()


def test_floating_callables_20_fits_allocate_nothing_rbd_script(gpu):
    """animate_RBD_2_link.jl:31-32 through the shim: iLQRHIP.fit(state_traj, input_traj,
    FloatingDynamics(m), FloatingCost(m), FloatingFinalCost(m); …) is family :floating and
    runs floating_fit1 on the cached FloatingSolver of (model, T = 1000, batch 1). Twenty
    MPC-style calls create one floating handle and 12 buffers once, and every result is
    bit-equal to the Python mirror's FloatingSolver.fit (same kernels) on the same start."""
    import torch
    from closures import jet_ns, rbd_floating_arm, rbd_initial_state
    from ilqr_amd.floating import FloatingSolver, rbd_example_problem
    fj, _, _ = rbd_floating_arm(jet_ns())
    T = 1000
    model = J.rbd_2dof_arm_floating()
    lib = CountingLib()
    cache = {}
    ref = FloatingSolver(rbd_example_problem(), T, 1)
    rng = np.random.default_rng(12)
    u0 = np.zeros((T, 8))
    counts = []
    try:
        for call in range(20):
            x0 = rbd_initial_state()
            x0[8:] = 0.02 * rng.standard_normal(8)
            x = np.zeros((T + 1, 16))
            x[0] = x0
            for t in range(T):
                x[t + 1] = fj(x[t][None], u0[t][None])[0]
            key = (bytes(model), T, 1)                       # floating_cached(m, M, 1)
            s = cache.get(key)
            if s is None:
                s = cache[key] = ShimFloatingSolver(lib, model, T, 1)
            max_iter = 3 if call in (0, 19) else 1
            xo, uo = s.fit1(x, u0, np.zeros_like(x), max_iter, 1e-6)
            counts.append(dict(lib.n))
            r = ref.fit(torch.from_numpy(x[None]).cuda(), torch.from_numpy(u0[None]).cuda(), max_iter=max_iter,
                        tol=1e-6)
            assert np.array_equal(xo, r.x[0].cpu().numpy()) and np.array_equal(uo, r.u[0].cpu().numpy()), call
    finally:
        ref.close()
    assert counts[0] == {"ilqr_create": 1, "ilqr_destroy": 0, "ilqr_malloc": 12, "ilqr_free": 0,
                         "ilqr_floating_create": 1, "ilqr_floating_destroy": 0}
    assert all(c == counts[0] for c in counts)
    for s in cache.values():
        s.close()
    assert lib.n["ilqr_free"] == 12 and lib.n["ilqr_destroy"] == 1 and lib.n["ilqr_floating_destroy"] == 1
