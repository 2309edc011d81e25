"""The Julia shim's boundary, exercised without Julia: every entry point of
ilqr.jl_amd/julia/iLQRHIP.jl replayed through the same C symbols with the same
buffers — the column-major memory of the Julia arrays the shim builds (its
permutedims conventions restated in tests/julia_layout.py), uploaded with the ABI's
own ilqr_malloc / ilqr_memcpy_h2d and read back with ilqr_memcpy_d2h, exactly as the
shim does — and compared with the oracle in the reference's layout (x::(N×nx),
δu::(T×nu), 𝐊s::(T×nu×nx)).

Covers: backward_pass / forward_pass / fit on the LQ family (per-trajectory
`to_abi`, `gains_to_abi`/`gains_from_abi`), the 2-link structs (nu = 2 and the nu = 1
variant) dispatched to ILQR_PROBLEM_TWO_LINK, the TILES fallback for arbitrary closures
(host derivative tiles → ilqr_backward_tiles), and batched solve! ((2,1,3) per-instance
matrices, (nx, N, B) trajectories), and the RBD families' chain_fit (f64 and f32) and
floating_fit with the shim's own rbd_2dof_arm_floating() model.
"""
import ctypes as C
import os

import numpy as np
import pytest

import julia_layout as J
from ilqr_amd import _lib
from oracle import ilqr_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


class Handle:
    """iLQRHIP.Handle: ilqr_create + buffers from ilqr_malloc, freed with it."""

    def __init__(self, nx, nu, T, batch):
        self.lib = _lib.load()
        h = C.c_void_p()
        _lib.check(self.lib.ilqr_create(C.byref(h), 0, nx, nu, T, batch), "ilqr_create")
        self.h, self.bufs = h, []

    def alloc(self, dtype, n):
        p = C.c_void_p()
        _lib.check(self.lib.ilqr_malloc(self.h, max(n, 1) * np.dtype(dtype).itemsize, C.byref(p)), "ilqr_malloc")
        self.bufs.append(p)
        return p

    def upload(self, a, dtype=np.float64):
        buf = np.ascontiguousarray(J.memory(a).astype(dtype))
        p = self.alloc(dtype, buf.size)
        _lib.check(self.lib.ilqr_memcpy_h2d(self.h, p, buf.ctypes.data_as(C.c_void_p), buf.nbytes), "h2d")
        return p

    def download(self, shape, p, dtype=np.float64):
        buf = np.empty(int(np.prod(shape)), dtype=dtype)
        _lib.check(self.lib.ilqr_memcpy_d2h(self.h, buf.ctypes.data_as(C.c_void_p), p, buf.nbytes), "d2h")
        return J.from_memory(buf, shape)

    def close(self):
        for p in self.bufs:
            self.lib.ilqr_free(self.h, p)
        self.lib.ilqr_destroy(self.h)


def lq_problem(h, A, B, Q, R, Qf):
    """iLQRHIP.problem(h, ::LinearDynamics, ::QuadraticCost, ::QuadraticFinalCost)."""
    return _lib.Problem(_lib.PROBLEM_LQ, 0, *(h.upload(J.rowmajor(M)).value for M in (A, B, Q, R, Qf)))


def tl_problem():
    return _lib.Problem(_lib.PROBLEM_TWO_LINK, 0, None, None, None, None, None)


def shim_backward(prob_fn, x, u):
    """iLQRHIP.backward_pass for a device family."""
    N, nx = x.shape
    M, nu = u.shape
    h = Handle(nx, nu, M, 1)
    p = prob_fn(h)
    xd, ud = h.upload(J.to_abi(x)), h.upload(J.to_abi(u))
    dd, Kd, st = h.alloc(np.float64, M * nu), h.alloc(np.float64, M * nu * nx), h.alloc(np.int32, 1)
    _lib.check(h.lib.ilqr_backward(h.h, C.byref(p), C.byref(_lib.default_options()), xd, ud, dd, Kd, st),
               "ilqr_backward")
    du = J.from_abi(h.download((nu, M), dd))
    K = J.gains_from_abi(h.download((nx, nu, M), Kd))
    h.close()
    return du, K


def shim_forward(prob_fn, x, u, x_traj, du, K, prev_cost):
    N, nx = x.shape
    M, nu = u.shape
    h = Handle(nx, nu, M, 1)
    p = prob_fn(h)
    xd, ud, xt = h.upload(J.to_abi(x)), h.upload(J.to_abi(u)), h.upload(J.to_abi(x_traj))
    dd, Kd = h.upload(J.to_abi(du)), h.upload(J.gains_to_abi(K))
    pc = h.upload(J.jl([prev_cost]))
    xo, uo, co = h.alloc(np.float64, N * nx), h.alloc(np.float64, M * nu), h.alloc(np.float64, 1)
    st = h.alloc(np.int32, 1)
    _lib.check(h.lib.ilqr_forward(h.h, C.byref(p), C.byref(_lib.default_options()), xd, ud, xt, dd, Kd, pc,
                                  xo, uo, co, None, st), "ilqr_forward")
    out = (J.from_abi(h.download((nx, N), xo)), J.from_abi(h.download((nu, M), uo)),
           float(h.download((1,), co)[0]))
    h.close()
    return out


def shim_fit(prob_fn, x_init, u_init, x_traj, max_iter, tol, with_history=False):
    """iLQRHIP.fit: ilqr_fit_ex with the (cost, trials) history the verbose print reads."""
    N, nx = x_init.shape
    M, nu = u_init.shape
    h = Handle(nx, nu, M, 1)
    p = prob_fn(h)
    o = _lib.default_options(max_iter=max_iter, tol=tol)
    xi, ui, xt = h.upload(J.to_abi(x_init)), h.upload(J.to_abi(u_init)), h.upload(J.to_abi(x_traj))
    xo, uo = h.alloc(np.float64, N * nx), h.alloc(np.float64, M * nu)
    hc = h.alloc(np.float64, max_iter)
    ht = h.upload(J.jl(np.zeros(max(max_iter, 1))), dtype=np.int32)
    hist = _lib.History(hc.value, ht.value, None, None)
    rc = h.lib.ilqr_fit_ex(h.h, C.byref(p), C.byref(o), xi, ui, xt, xo, uo, None, None, None, C.byref(hist))
    assert rc in (_lib.OK, _lib.ERR_LS_EXHAUSTED)
    out = J.from_abi(h.download((nx, N), xo)), J.from_abi(h.download((nu, M), uo))
    if with_history:  # print_history's inputs: download!(h, zeros(max_iter), hc), … Int32 …
        out = out + (h.download((max_iter,), hc), h.download((max(max_iter, 1),), ht, dtype=np.int32))
    h.close()
    return out


@pytest.fixture(scope="module")
def quad():
    return load("dense_xtraj")


@pytest.mark.gpu
def test_shim_lq_backward_pass(gpu, quad):
    g = quad
    b = 1
    du, K = shim_backward(lambda h: lq_problem(h, g["A"][b], g["B"][b], g["Q"][b], g["R"][b], g["Qf"][b]),
                          g["x"][b], g["u"][b])
    assert du.shape == g["d"][b].shape and K.shape == g["K"][b].shape    # (T × nu), (T × nu × nx)
    assert rel(du, g["d"][b]) < 1e-8 and rel(K, g["K"][b]) < 1e-8


@pytest.mark.gpu
def test_shim_lq_forward_pass_with_x_traj(gpu, quad):
    g = quad
    b = 0
    x̄, ū, c = shim_forward(lambda h: lq_problem(h, g["A"][b], g["B"][b], g["Q"][b], g["R"][b], g["Qf"][b]),
                            g["x"][b], g["u"][b], g["xtraj"][b], g["d"][b], g["K"][b], np.inf)
    assert rel(x̄, g["fw_x"][b]) < 1e-10 and rel(ū, g["fw_u"][b]) < 1e-10
    assert abs(c - g["fw_cost"][b]) / g["fw_cost"][b] < 1e-11


@pytest.mark.gpu
def test_shim_lq_fit(gpu, quad):
    g = quad
    b = 1
    x, u, hc, ht = shim_fit(lambda h: lq_problem(h, g["A"][b], g["B"][b], g["Q"][b], g["R"][b], g["Qf"][b]),
                            g["x"][b], g["u"][b], g["xtraj"][b], 30, 1e-6, with_history=True)
    assert rel(x, g["fit_x"][b]) < 1e-8 and rel(u, g["fit_u"][b]) < 1e-8
    # fit(...; verbose=true) prints one line per iteration with trials > 0: the oracle's costs
    n = int(g["fit_iters"][b])
    assert (ht[:n] > 0).all() and (ht[n:] == 0).all()
    assert rel(hc[:n], g["fit_cost"][b, :n]) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("nu,name", [(2, "twolink_t50"), (1, "twolink_nu1_t50")])
def test_shim_two_link_structs(gpu, nu, name):
    """TwoLinkDynamics{NU}/TwoLinkCost/TwoLinkFinalCost → ILQR_PROBLEM_TWO_LINK."""
    g = load(name)
    b = 2
    du, K = shim_backward(lambda h: tl_problem(), g["x"][b], g["u"][b])
    assert rel(du, g["d"][b]) < 1e-10 and rel(K, g["K"][b]) < 1e-10
    x̄, ū, c = shim_forward(lambda h: tl_problem(), g["x"][b], g["u"][b], np.zeros_like(g["x"][b]),
                            g["d"][b], g["K"][b], np.inf)
    assert rel(x̄, g["fw_x"][b]) < 1e-11 and abs(c - g["fw_cost"][b]) / g["fw_cost"][b] < 1e-12
    x, u = shim_fit(lambda h: tl_problem(), g["x"][b], g["u"][b], np.zeros_like(g["x"][b]), 40, 1e-6)
    assert rel(u, g["fit_u"][b]) < 1e-9


@pytest.mark.gpu
def test_shim_tiles_fallback_arbitrary_closures(gpu):
    """Arbitrary closures (here the oracle's plain 2-link functions, not the recognised
    structs): derivative tiles on the host (iLQRHIP.derivative_tiles; oracle.dual
    standing in for ForwardDiff) → ilqr_backward_tiles on the device; the gains equal
    the reference restatement's backward_pass."""
    g = load("twolink_t50")
    b = 1
    x, u = g["x"][b], g["u"][b]
    TL = O.TwoLink
    t = J.derivative_tiles(x, u, TL.dynamicsf, TL.immediate_cost, TL.final_cost)
    N, nx = x.shape
    M, nu = u.shape
    h = Handle(nx, nu, M, 1)
    tl = _lib.Tiles(*(h.upload(t[k]).value for k in ("A", "B", "lx", "lu", "lxx", "lux", "luu", "lfx", "lfxx")))
    dd, Kd, st = h.alloc(np.float64, M * nu), h.alloc(np.float64, M * nu * nx), h.alloc(np.int32, 1)
    _lib.check(h.lib.ilqr_backward_tiles(h.h, C.byref(tl), C.byref(_lib.default_options()), dd, Kd, st),
               "ilqr_backward_tiles")
    du, K = J.from_abi(h.download((nu, M), dd)), J.gains_from_abi(h.download((nx, nu, M), Kd))
    h.close()
    assert rel(du, g["d"][b]) < 1e-10 and rel(K, g["K"][b]) < 1e-10


def test_shim_tiles_layout_is_row_major_per_step():
    """The tiles' Julia arrays hold each step's matrices transposed, i.e. their memory is
    the ABI's row-major (T, r, c) blocks (a layout-only property: no GPU)."""
    rng = np.random.default_rng(1)
    A = rng.standard_normal((3, 4, 4))                 # three steps' A_t
    Aj = J.jl(np.zeros((4, 4, 3)))
    for i in range(3):
        Aj[:, :, i] = A[i].T
    assert np.array_equal(J.memory(Aj), A.reshape(-1))


@pytest.mark.gpu
def test_shim_solve_batched(gpu):
    """solve!(::iLQRProblem): Julia (nx, nx, B) per-instance matrices permuted (2,1,3),
    trajectories (nx, N, B) passed as they are."""
    g = load("dense_t16")
    nb = g["A"].shape[0]
    T = g["u"].shape[1]
    nx, nu = g["A"].shape[1], g["B"].shape[2]
    jA, jB, jQ, jR, jQf = (J.jl(np.moveaxis(g[k], 0, -1)) for k in ("A", "B", "Q", "R", "Qf"))  # A[:, :, b]
    jx = J.jl(np.transpose(g["x"], (2, 1, 0)))        # x[:, t, b]
    ju = J.jl(np.transpose(g["u"], (2, 1, 0)))
    h = Handle(nx, nu, T, nb)
    p = _lib.Problem(_lib.PROBLEM_LQ, 0, *(h.upload(J.rowmajor3(a)).value for a in (jA, jB, jQ, jR, jQf)))
    o = _lib.default_options(max_iter=30, tol=1e-6)
    xi, ui = h.upload(jx), h.upload(ju)
    xo, uo = h.alloc(np.float64, jx.size), h.alloc(np.float64, ju.size)
    n = 30  # solve!(prob; history=true): (max_iter, batch) row-major = Julia (batch, max_iter)
    hd = (h.alloc(np.float64, n * nb), h.upload(J.jl(np.zeros(n * nb)), dtype=np.int32),
          h.alloc(np.float64, n * nb), h.alloc(np.float64, n * nb))
    hist = _lib.History(*(q.value for q in hd))
    assert h.lib.ilqr_fit_ex(h.h, C.byref(p), C.byref(o), xi, ui, None, xo, uo, None, None, None,
                             C.byref(hist)) == _lib.OK
    x, u = h.download(jx.shape, xo), h.download(ju.shape, uo)
    cost = h.download((nb, n), hd[0])
    trials = h.download((nb, n), hd[1], dtype=np.int32)
    h.close()
    for b in range(nb):
        assert rel(x[:, :, b].T, g["fit_x"][b]) < 1e-8 and rel(u[:, :, b].T, g["fit_u"][b]) < 1e-8
        k = int(g["fit_iters"][b])
        assert (trials[b, :k] > 0).all() and (trials[b, k:] == 0).all()
        assert rel(cost[b, :k], g["fit_cost"][b, :k]) < 1e-9


@pytest.mark.gpu
def test_shim_multisolver_resident(gpu):
    """MultiSolver(prob, devices) + solve!(ms, prob; warm_start): ilqr_multi_set_problem
    with the (2,1,3)-permuted per-instance matrices (host arrays, once), ilqr_multi_load of
    the (nx, N, B) trajectories as they are, ilqr_multi_fit_resident, ilqr_multi_gather into
    the same Julia arrays — two shards on the test box's GPU; equal to the batched fit
    (solve!) above, and a warm-started second call equals a fit from the first's result."""
    g = load("dense_t16")
    nb = g["A"].shape[0]
    T = g["u"].shape[1]
    nx, nu = g["A"].shape[1], g["B"].shape[2]
    mats = [np.ascontiguousarray(J.memory(J.rowmajor3(J.jl(np.moveaxis(g[k], 0, -1)))))
            for k in ("A", "B", "Q", "R", "Qf")]
    jx = J.jl(np.transpose(g["x"], (2, 1, 0)))
    ju = J.jl(np.transpose(g["u"], (2, 1, 0)))
    lib = _lib.load()
    m = C.c_void_p()
    devs = (C.c_int * 2)(0, 0)
    _lib.check(lib.ilqr_multi_create(C.byref(m), devs, 2, nx, nu, T, nb), "ilqr_multi_create")
    try:
        p = _lib.Problem(_lib.PROBLEM_LQ, 0, *(a.ctypes.data for a in mats))
        _lib.check(lib.ilqr_multi_set_problem(m, C.byref(p)), "ilqr_multi_set_problem")
        xm = np.ascontiguousarray(J.memory(jx))
        um = np.ascontiguousarray(J.memory(ju))
        _lib.check(lib.ilqr_multi_load(m, xm.ctypes.data_as(C.c_void_p), um.ctypes.data_as(C.c_void_p), None),
                   "ilqr_multi_load")

        def fit_gather(flags, max_iter):
            o = _lib.default_options(max_iter=max_iter, tol=1e-6)
            assert lib.ilqr_multi_fit_resident(m, C.byref(o), flags, None) in (_lib.OK, _lib.ERR_LS_EXHAUSTED)
            xo, uo = np.empty_like(xm), np.empty_like(um)
            _lib.check(lib.ilqr_multi_gather(m, xo.ctypes.data_as(C.c_void_p), uo.ctypes.data_as(C.c_void_p),
                                             None, None, None), "ilqr_multi_gather")
            return J.from_memory(xo, jx.shape), J.from_memory(uo, ju.shape)

        x, u = fit_gather(0, 30)
        for b in range(nb):
            assert rel(x[:, :, b].T, g["fit_x"][b]) < 1e-8 and rel(u[:, :, b].T, g["fit_u"][b]) < 1e-8
        # warm start: 2 more iterations from the resident result = a fit from it
        xw, uw = fit_gather(1, 2)
        for b in range(nb):
            A, B, Q, R, Qf = (g[k][b] for k in ("A", "B", "Q", "R", "Qf"))
            xr, ur = O.fit(x[:, :, b].T, u[:, :, b].T, *O.lq_closures(A, B, Q, R, Qf), max_iter=2, tol=1e-6,
                           symmetrize=True)[:2]
            assert rel(xw[:, :, b].T, xr) < 1e-8 and rel(uw[:, :, b].T, ur) < 1e-8
    finally:
        lib.ilqr_multi_destroy(m)


def shim_family_fit(create, fit, destroy, x_init, u_init, max_iter, tol, dtype):
    """The tail shared by iLQRHIP.chain_fit / floating_fit: a memory-helper Handle,
    upload(h, x_init) of the (nx, N, batch) Julia arrays as they are, the family's fit
    with x_traj / cost / iterations left C_NULL, download! into similar(x_init), the
    family handle destroyed and the helper closed."""
    nx, N, nb = x_init.shape
    nu, M = u_init.shape[0], u_init.shape[1]
    r = create(M, nb)
    h = Handle(nx, nu, M, 1)
    try:
        xi, ui = h.upload(x_init, dtype=dtype), h.upload(u_init, dtype=dtype)
        xo, uo, sd = h.alloc(dtype, x_init.size), h.alloc(dtype, u_init.size), h.alloc(np.int32, nb)
        o = _lib.default_options(max_iter=max_iter, tol=tol)
        st = fit(r, C.byref(o), xi, ui, None, xo, uo, None, None, sd)
        assert st in (_lib.OK, _lib.ERR_LS_EXHAUSTED)
        return (h.download(x_init.shape, xo, dtype=dtype), h.download(u_init.shape, uo, dtype=dtype),
                h.download((nb,), sd, dtype=np.int32))
    finally:
        destroy(r)
        h.close()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_shim_chain_fit(gpu, dtype):
    """iLQRHIP.chain_fit(::Chain, x_init::Array{E,3}, u_init): Ref{Chain} to
    ilqr_chain_create with the element type's precision, set_dynamics(AUTO), the helper
    Handle's buffers — the same trajectories, bit for bit, as ChainSolver.fit on
    (batch, N, nx) tensors (whose results the chain tests pin to the oracle)."""
    import torch
    from ilqr_amd.chain import ChainSolver, rbd_2dof_problem, rbd_initial_states
    p = rbd_2dof_problem()
    nb, T, iters = 4, 60, 8
    x0 = rbd_initial_states(nb)
    u0 = np.zeros((nb, T, p.nu))
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    s = ChainSolver(p, T, nb, dtype=tdt)
    try:
        xs = s.rollout(torch.as_tensor(x0, dtype=tdt, device="cuda"), torch.as_tensor(u0, dtype=tdt, device="cuda"))
        x_init = xs.cpu().numpy().astype(np.float64)
        ref = s.fit(xs, torch.as_tensor(u0, dtype=tdt, device="cuda"), max_iter=iters, tol=1e-6)
        rx, ru, rs = ref.x.cpu().numpy(), ref.u.cpu().numpy(), ref.status.cpu().numpy()
    finally:
        s.close()
    lib = _lib.load()
    st = p.struct()

    def create(M, b):
        r = C.c_void_p()
        _lib.check(lib.ilqr_chain_create(C.byref(r), 0, C.byref(st), M, b,
                                         _lib.F64 if dtype == np.float64 else _lib.F32, _lib.LINEARIZE_DUAL),
                   "ilqr_chain_create")
        _lib.check(lib.ilqr_chain_set_dynamics(r, _lib.CHAIN_DYN_AUTO), "ilqr_chain_set_dynamics")
        return r

    jx = J.jl(np.transpose(x_init, (2, 1, 0)))          # x_init[:, t, b]
    ju = J.jl(np.transpose(u0, (2, 1, 0)))
    x, u, status = shim_family_fit(create, lib.ilqr_chain_fit, lib.ilqr_chain_destroy, jx, ju, iters, 1e-6, dtype)
    assert np.array_equal(np.transpose(x, (2, 1, 0)), rx) and np.array_equal(np.transpose(u, (2, 1, 0)), ru)
    assert np.array_equal(status, rs)


@pytest.mark.gpu
def test_shim_floating_fit(gpu):
    """iLQRHIP.floating_fit(rbd_2dof_arm_floating(), x_init, u_init): the shim's model
    by Ref to ilqr_floating_create and (16, N, batch) / (8, T, batch) arrays through the
    helper Handle — the same fit, bit for bit, as FloatingSolver.fit on the example
    problem (pinned to the oracle by tests/test_gpu_floating.py)."""
    import torch
    from ilqr_amd.floating import FloatingSolver, rbd_example_problem, rbd_initial_state
    nb, T, iters = 3, 80, 3
    x0 = np.tile(rbd_initial_state(), (nb, 1))
    x0[1:, 8:] = 0.05 * np.random.default_rng(3).standard_normal((nb - 1, 8))
    u0 = np.zeros((nb, T, 8))
    s = FloatingSolver(rbd_example_problem(), T, nb)
    try:
        xs = s.rollout(torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda())
        x_init = xs.cpu().numpy()
        ref = s.fit(xs, torch.from_numpy(u0).cuda(), max_iter=iters, tol=1e-6)
        rx, ru, rs = ref.x.cpu().numpy(), ref.u.cpu().numpy(), ref.status.cpu().numpy()
    finally:
        s.close()
    lib = _lib.load()
    m = J.rbd_2dof_arm_floating()

    def create(M, b):
        r = C.c_void_p()
        _lib.check(lib.ilqr_floating_create(C.byref(r), 0, C.byref(m), M, b), "ilqr_floating_create")
        return r

    jx = J.jl(np.transpose(x_init, (2, 1, 0)))
    ju = J.jl(np.transpose(u0, (2, 1, 0)))
    x, u, status = shim_family_fit(create, lib.ilqr_floating_fit, lib.ilqr_floating_destroy, jx, ju, iters,
                                   1e-6, np.float64)
    assert np.array_equal(np.transpose(x, (2, 1, 0)), rx) and np.array_equal(np.transpose(u, (2, 1, 0)), ru)
    assert np.array_equal(status, rs)
