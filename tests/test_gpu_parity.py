"""GPU parity tests: the HIP path (through the C ABI) against the oracle.

Tolerances (fp64): the device evaluates the reference's formulas in a different
order and with the exact algebraic rewrite step_back(:268-270) ≡
[Qxx | lx+Aᵀs] − K_augᵀ(H+2μI)K_aug, so results agree to rounding amplified by
the Riccati recursion: K, d within rel 1e-8 of max|·| over a fixture; forward
rollouts within rel 1e-10 given identical gains; costs rel 1e-11; line-search
trial counts and fit iteration counts exactly. Full-size (B=4096, T=100)
checks compare with the C restatement on a sample and use size-independent
properties (KKT fixed point, monotone cost, idempotence).
"""
import json
import os

import numpy as np
import pytest
import torch

from ilqr_amd import _lib
from ilqr_amd.problems import LQBatch, quadrotor_batch, random_lq_batch
from ilqr_amd.solver import Solver, selftest
from oracle import cref
from oracle import ilqr_oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
LQ_FIXTURES = ["quad_t16", "quad_t100_sym", "dense_t16", "dense_t64_sym", "dense_xtraj"]

TOL_GAIN = 1e-8       # vs the LITERAL oracle: bounded by the literal recursion's own drift (< 1e-9 on these fixtures)
TOL_GAIN_SYM = 1e-11  # vs the symmetrised oracle (identity in exact arithmetic)
TOL_ROLL = 1e-10
TOL_COST = 1e-11


def tol_gain(g):
    return TOL_GAIN_SYM if json.loads(str(g["meta"]))["symmetrize"] else TOL_GAIN


def rel(a, b):
    a = a.cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = b.cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def dev(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a)).to("cuda", dtype).contiguous()


def load(name):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def solver_for(g):
    lq = LQBatch(g["A"], g["B"], g["Q"], g["R"], g["Qf"])
    T = g["u"].shape[1]
    s = Solver(lq.nx, lq.nu, T, lq.batch)
    s.set_problem(lq)
    return s, lq


def test_selftest_lane_maps(gpu):
    assert selftest(0) == 0


@pytest.mark.parametrize("backward", ["auto", "block"])
@pytest.mark.parametrize("name", LQ_FIXTURES)
def test_backward_matches_golden(gpu, name, backward):
    """Golden gains through the default backward kernel (one trajectory per wave at
    these batch sizes) and the four-trajectories-per-wave one."""
    g = load(name)
    s, _ = solver_for(g)
    s.set_schedule(backward=backward)
    d, K, st = s.backward(dev(g["x"]), dev(g["u"]))
    assert (st.cpu().numpy() == 0).all()
    assert rel(K, g["K"]) < tol_gain(g), rel(K, g["K"])
    assert rel(d, g["d"]) < tol_gain(g), rel(d, g["d"])


@pytest.mark.parametrize("name", LQ_FIXTURES)
def test_forward_matches_golden(gpu, name):
    g = load(name)
    s, _ = solver_for(g)
    nb = g["A"].shape[0]
    xt = dev(g["xtraj"]) if "xtraj" in g else None
    pc = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
    xn, un, c, tr, st = s.forward(dev(g["x"]), dev(g["u"]), dev(g["d"]), dev(g["K"]), pc, x_traj=xt)
    assert (st.cpu().numpy() == 0).all()
    assert rel(xn, g["fw_x"]) < TOL_ROLL and rel(un, g["fw_u"]) < TOL_ROLL
    assert rel(c, g["fw_cost"]) < TOL_COST
    assert np.array_equal(tr.cpu().numpy(), g["fw_trials"])


@pytest.mark.parametrize("backward", ["auto", "block"])
@pytest.mark.parametrize("name", LQ_FIXTURES)
def test_fit_matches_golden(gpu, name, backward):
    g = load(name)
    meta = json.loads(str(g["meta"]))
    s, _ = solver_for(g)
    s.set_schedule(backward=backward)
    xt = dev(g["xtraj"]) if "xtraj" in g else None
    r = s.fit(dev(g["x"]), dev(g["u"]), x_traj=xt, max_iter=meta["fit_max_iter"], tol=meta["tol"])
    assert r.call_status == 0
    assert np.array_equal(r.iters.cpu().numpy(), g["fit_iters"])
    assert (r.status.cpu().numpy() == _lib.TRAJ_CONVERGED).all()
    assert rel(r.u, g["fit_u"]) < 1e-8 and rel(r.x, g["fit_x"]) < 1e-8
    last = np.array([g["fit_cost"][b, g["fit_iters"][b] - 1] for b in range(len(g["fit_iters"]))])
    assert rel(r.cost, last) < 1e-9


# -- reference API mirror ------------------------------------------------------------
def test_reference_api_single_trajectory_numpy(gpu):
    import ilqr_amd
    g = load("quad_t16")
    b = 1
    f = ilqr_amd.LinearDynamics(g["A"][b], g["B"][b])
    l = ilqr_amd.QuadraticCost(g["Q"][b], g["R"][b])
    lf = ilqr_amd.QuadraticFinalCost(g["Qf"][b])
    du, K = ilqr_amd.backward_pass(g["x"][b], g["u"][b], f, l, lf)
    assert du.shape == (16, 4) and K.shape == (16, 4, 12)
    assert rel(K, g["K"][b]) < TOL_GAIN
    xb, ub, c = ilqr_amd.forward_pass(g["x"][b], g["u"][b], np.zeros_like(g["x"][b]), du, K, np.inf, f, l, lf)
    assert isinstance(c, float) and rel(ub, g["fw_u"][b]) < 1e-9
    xf, uf = ilqr_amd.fit(g["x"][b], g["u"][b], f, l, lf, max_iter=30, tol=1e-6)
    assert rel(uf, g["fit_u"][b]) < 1e-8
    # the closures are real callables (same objects a CPU reference would call)
    assert np.allclose(f(g["x"][b, 0], g["u"][b, 0]), g["x"][b, 1])


def test_reference_api_errors(gpu):
    import ilqr_amd
    g = load("quad_t16")
    f = ilqr_amd.LinearDynamics(g["A"][0], g["B"][0])
    l = ilqr_amd.QuadraticCost(g["Q"][0], g["R"][0])
    lf = ilqr_amd.QuadraticFinalCost(g["Qf"][0])
    with pytest.raises(AssertionError):                       # backward_pass.jl:329
        ilqr_amd.backward_pass(g["x"][0][:-1], g["u"][0], f, l, lf)
    with pytest.raises(TypeError):                            # forward_pass.jl:152
        ilqr_amd.fit(g["x"][0], g["u"][0], f, l, lf, max_iter=1e5)
    with pytest.raises(NotImplementedError):                  # closures torch.func cannot differentiate
        ilqr_amd.backward_pass(g["x"][0], g["u"][0], lambda x, u: np.asarray(x), l, lf)
    # a mixed triple (non-family dynamics, family costs) takes the generic tiles path
    d, K = ilqr_amd.backward_pass(g["x"][0], g["u"][0], lambda x, u: f(x, u), l, lf)
    dr, Kr = ilqr_amd.backward_pass(g["x"][0], g["u"][0], f, l, lf)
    assert rel(d, dr) < 1e-12 and rel(K, Kr) < 1e-12
    with pytest.raises(AssertionError):                       # NaN → AssertionError (:353)
        xbad = g["x"][0].copy()
        xbad[5, 3] = np.nan
        ilqr_amd.backward_pass(xbad, g["u"][0], f, l, lf)


# -- edge cases -----------------------------------------------------------------------
@pytest.mark.parametrize("nb,T", [(1, 1), (1, 2), (5, 3), (7, 17), (6, 40)])
def test_ragged_batches_and_short_horizons(gpu, nb, T):
    lq, x, u = random_lq_batch(nb, 12, 4, T, seed=nb * 100 + T)
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    d, K, st = s.backward(dev(x), dev(u))
    dc, Kc, _ = cref.lq_backward(lq, x, u, symmetrize=True)
    assert rel(K, Kc) < TOL_GAIN_SYM and rel(d, dc) < TOL_GAIN_SYM
    pc = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
    xn, un, c, tr, st = s.forward(dev(x), dev(u), d, K, pc)
    xo, uo, co, tro = cref.lq_forward(lq, x, u, None, d.cpu().numpy(), K.cpu().numpy(), np.inf)
    assert rel(xn, xo) < TOL_ROLL and rel(c, co) < TOL_COST and np.array_equal(tr.cpu().numpy(), tro)


def test_line_search_exhaustion_returns_inputs(gpu):
    """prev_cost = -Inf can never be beaten: the reference would loop forever
    (forward_pass.jl:70-87); the device stops at max_trials and returns x, u."""
    lq, x, u = random_lq_batch(4, 12, 4, 10, seed=3)
    s = Solver(12, 4, 10, 4)
    s.set_problem(lq)
    d, K, _ = s.backward(dev(x), dev(u))
    pc = torch.full((4,), -float("inf"), dtype=torch.float64, device="cuda")
    xn, un, c, tr, st = s.forward(dev(x), dev(u), d, K, pc, max_trials=7)
    assert (st.cpu().numpy() == _lib.TRAJ_LS_EXHAUSTED).all()
    assert (tr.cpu().numpy() == 7).all()
    assert torch.equal(xn.cpu(), torch.from_numpy(x)) and torch.equal(un.cpu(), torch.from_numpy(u))


def test_nan_is_reported_per_trajectory(gpu):
    lq, x, u = random_lq_batch(8, 12, 4, 12, seed=4)
    x[3, 6, 2] = np.nan
    s = Solver(12, 4, 12, 8)
    s.set_problem(lq)
    d, K, st = s.backward(dev(x), dev(u))
    st = st.cpu().numpy()
    assert st[3] == _lib.TRAJ_NAN and (np.delete(st, 3) == 0).all()
    r = s.fit(dev(x), dev(u), max_iter=20, tol=1e-6)
    st = r.status.cpu().numpy()
    assert r.call_status == _lib.ERR_NAN and st[3] == _lib.TRAJ_NAN
    assert (np.delete(st, 3) == _lib.TRAJ_CONVERGED).all()


def test_x_traj_none_equals_zeros(gpu):
    lq, x, u = random_lq_batch(4, 12, 4, 20, seed=8)
    s = Solver(12, 4, 20, 4)
    s.set_problem(lq)
    a = s.fit(dev(x), dev(u), max_iter=10)
    b = s.fit(dev(x), dev(u), x_traj=torch.zeros_like(dev(x)), max_iter=10)
    assert torch.equal(a.x, b.x) and torch.equal(a.u, b.u)


# -- headline size (B = 4096, T = 100) --------------------------------------------------
@pytest.fixture(scope="module")
def headline():
    lq, x, u = quadrotor_batch(4096, T=100, seed0=0)
    s = Solver(12, 4, 100, 4096)
    s.set_problem(lq)
    return s, lq, x, u


def test_headline_backward_vs_c_oracle(gpu, headline):
    s, lq, x, u = headline
    d, K, st = s.backward(dev(x), dev(u))
    assert (st.cpu().numpy() == 0).all()
    idx = np.random.default_rng(0).choice(4096, 256, replace=False)
    sub = lq.slice(0, 4096)
    sub = LQBatch(lq.A[idx], lq.B[idx], lq.Q[idx], lq.R[idx], lq.Qf[idx])
    dc, Kc, stc = cref.lq_backward(sub, x[idx], u[idx], symmetrize=True)
    assert rel(K.cpu().numpy()[idx], Kc) < TOL_GAIN_SYM and rel(d.cpu().numpy()[idx], dc) < TOL_GAIN_SYM


def test_backward_kernels_agree_headline(gpu, headline):
    """The two backward kernels (4 trajectories / wave on the 4-block MFMA, the
    default; 1 trajectory / wave on the 16x16x4 tile, ILQR_SCHED_BACKWARD_WAVE) agree
    to rounding: both sit within 2e-13 of the symmetrised oracle on these fixtures."""
    s, lq, x, u = headline
    d4_, K4_, st4 = s.backward(dev(x), dev(u))
    s.set_schedule(backward="wave")
    try:
        dw, Kw, stw = s.backward(dev(x), dev(u))
    finally:
        s.set_schedule()
    assert (st4.cpu().numpy() == 0).all() and (stw.cpu().numpy() == 0).all()
    assert rel(K4_, Kw) < 1e-12 and rel(d4_, dw) < 1e-12


@pytest.mark.parametrize("nb", [1, 3, 5, 17, 1030])
def test_backward4_ragged_batch_and_nan_slot(gpu, nb):
    """Batches that leave a wave's last slots empty, and a NaN trajectory sharing its
    wave with clean ones: the clean slots' gains match the oracle, the NaN slot alone
    is flagged."""
    T = 13
    lq, x, u = random_lq_batch(nb, 12, 4, T, seed=nb + 101)
    bad = nb // 2
    x[bad, 4, 2] = np.nan
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    s.set_schedule(backward="block")  # small batches default to one trajectory per wave
    d, K, st = s.backward(dev(x), dev(u))
    st = st.cpu().numpy()
    assert st[bad] == _lib.TRAJ_NAN and (np.delete(st, bad) == 0).all()
    ok = np.arange(nb) != bad
    dc, Kc, _ = cref.lq_backward(LQBatch(lq.A[ok], lq.B[ok], lq.Q[ok], lq.R[ok], lq.Qf[ok]), x[ok], u[ok],
                                 symmetrize=True)
    if ok.any():
        assert rel(K.cpu().numpy()[ok], Kc) < TOL_GAIN_SYM and rel(d.cpu().numpy()[ok], dc) < TOL_GAIN_SYM


@pytest.mark.parametrize("T", [1, 2, 3, 6, 14, 19])
def test_backward4_horizon_remainders(gpu, T):
    """The four-trajectories-per-wave backward runs its step loop four steps at a time
    (static L z column per step) plus a remainder of T mod 4 steps: every remainder,
    and horizons shorter than one block, against the oracle (backward and fit)."""
    nb = 7
    lq, x, u = random_lq_batch(nb, 12, 4, T, seed=300 + T)
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    s.set_schedule(backward="block")
    d, K, st = s.backward(dev(x), dev(u))
    assert (st.cpu().numpy() == 0).all()
    dc, Kc, _ = cref.lq_backward(lq, x, u, symmetrize=True)
    assert rel(K, Kc) < TOL_GAIN_SYM and rel(d, dc) < TOL_GAIN_SYM
    r = s.fit(dev(x), dev(u), max_iter=6, tol=1e-9)
    xo, uo, co, it, sto = cref.lq_fit(lq, x, u, max_iter=6, tol=1e-9, symmetrize=True)
    assert np.array_equal(r.iters.cpu().numpy(), it)
    assert rel(r.u.cpu().numpy(), uo) < 1e-8


def test_headline_fit_reaches_kkt_and_cost_is_monotone(gpu, headline):
    s, lq, x, u = headline
    # three iterations with tol disabled: every trajectory improves (α = 1 from cold,
    # then strictly decreasing costs — the @assert(prev_cost > new_cost) of :168)
    xi, ui = dev(x), dev(u)
    xn, un = torch.empty_like(xi), torch.empty_like(ui)
    pc = torch.full((4096,), float("inf"), dtype=torch.float64, device="cuda")
    st = torch.zeros((4096,), dtype=torch.int32, device="cuda")
    costs = []
    o = _lib.default_options(tol=-1.0)
    for _ in range(3):
        s.iterate(xi, ui, xn, un, pc, st, options=o)
        costs.append(pc.clone())
        xi, xn, ui, un = xn, xi, un, ui
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    c = torch.stack(costs).cpu().numpy()
    assert (np.diff(c, axis=0) < 0).all()
    # fit to the fixed point: iLQR's fixed point is the exact LQ minimiser (KKT). Once
    # no step can lower the cost the reference's line search would spin forever; the
    # device stops that trajectory (LS_EXHAUSTED) at its fixed point.
    r = s.fit(dev(x), dev(u), max_iter=30, tol=1e-14)
    stf = r.status.cpu().numpy()
    assert np.isin(stf, [_lib.TRAJ_CONVERGED, _lib.TRAJ_LS_EXHAUSTED, _lib.TRAJ_MAX_ITER]).all()
    for b in (0, 1234, 4095):
        X, U = O.lq_kkt_solution(lq.A[b], lq.B[b], lq.Q[b], lq.R[b], lq.Qf[b], x[b, 0], 100)
        assert rel(r.u[b], U) < 1e-6, rel(r.u[b], U)


def test_headline_iterate_matches_backward_plus_forward(gpu, headline):
    """The fused iteration entry point equals backward_pass + forward_pass."""
    s, lq, x, u = headline
    xi, ui = dev(x), dev(u)
    d, K, _ = s.backward(xi, ui)
    pc = torch.full((4096,), float("inf"), dtype=torch.float64, device="cuda")
    xf, uf, cf, _, _ = s.forward(xi, ui, d, K, pc)
    xn, un = torch.empty_like(xi), torch.empty_like(ui)
    st = torch.zeros((4096,), dtype=torch.int32, device="cuda")
    s.iterate(xi, ui, xn, un, pc, st, options=_lib.default_options(tol=-1.0))
    torch.cuda.synchronize()
    assert torch.equal(xn, xf) and torch.equal(un, uf) and torch.equal(pc, cf)


# -- launch schedules (ilqr_set_schedule) ----------------------------------------------
def _fit_both(s, x, u, **kw):
    s.set_schedule(pipelined=False, backward="wave")  # the pipelined kernel's backward
    a = s.fit(x, u, **kw)
    s.set_schedule(pipelined=True)
    b = s.fit(x, u, **kw)
    torch.cuda.synchronize()
    s.set_schedule()
    return a, b


def _same(a, b):
    assert a.call_status == b.call_status
    for f in ("x", "u", "cost", "iters", "status"):  # bitwise, NaN == NaN
        torch.testing.assert_close(getattr(a, f), getattr(b, f), rtol=0, atol=0, equal_nan=True,
                                   msg=f)


def test_pipelined_fit_equals_sequential_headline(gpu, headline):
    """Role A/B workgroups run forward(i−1) ∥ backward(i): same results, bit for bit,
    through convergence (tol), max_iter and the final gather."""
    s, lq, x, u = headline
    for kw in (dict(max_iter=1, tol=-1.0), dict(max_iter=5, tol=-1.0), dict(max_iter=40, tol=1e-9)):
        a, b = _fit_both(s, dev(x), dev(u), **kw)
        _same(a, b)


@pytest.mark.parametrize("nb,T", [(1, 5), (5, 3), (37, 17), (1029, 9)])
def test_pipelined_fit_ragged(gpu, nb, T):
    lq, x, u = random_lq_batch(nb, 12, 4, T, seed=nb + 7 * T)
    x[nb // 2, 1, 0] = np.nan  # one NaN trajectory leaves the batch in iteration 1
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    a, b = _fit_both(s, dev(x), dev(u), max_iter=12, tol=1e-8)
    _same(a, b)
    st = b.status.cpu().numpy()
    assert st[nb // 2] == _lib.TRAJ_NAN
    xo, uo, co, it, sto = cref.lq_fit(LQBatch(lq.A, lq.B, lq.Q, lq.R, lq.Qf), x, u, max_iter=12,
                                      tol=1e-8, symmetrize=True)
    ok = np.arange(nb) != nb // 2
    if ok.any():
        assert np.array_equal(b.iters.cpu().numpy()[ok], it[ok])
        assert rel(b.u.cpu().numpy()[ok], uo[ok]) < 1e-8


@pytest.mark.parametrize("nb,T", [(5, 3), (37, 17), (1029, 9)])
def test_fit_block_backward_ragged_vs_oracle(gpu, nb, T):
    """fit through the four-trajectories-per-wave backward on ragged batches with a
    NaN trajectory that leaves in iteration 1 (its wave's other slots keep going)."""
    lq, x, u = random_lq_batch(nb, 12, 4, T, seed=nb + 7 * T)
    x[nb // 2, 1, 0] = np.nan
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    s.set_schedule(backward="block")
    r = s.fit(dev(x), dev(u), max_iter=12, tol=1e-8)
    st = r.status.cpu().numpy()
    assert st[nb // 2] == _lib.TRAJ_NAN
    xo, uo, co, it, sto = cref.lq_fit(LQBatch(lq.A, lq.B, lq.Q, lq.R, lq.Qf), x, u, max_iter=12,
                                      tol=1e-8, symmetrize=True)
    ok = np.arange(nb) != nb // 2
    assert np.array_equal(r.iters.cpu().numpy()[ok], it[ok])
    assert rel(r.x.cpu().numpy()[ok], xo[ok]) < 1e-8 and rel(r.u.cpu().numpy()[ok], uo[ok]) < 1e-8


@pytest.mark.parametrize("nb,T", [(4096, 100), (37, 17), (5, 3)])
def test_ring_forward_iterate_equals_standard(gpu, nb, T):
    """The LDS-ring forward kernel (ILQR_SCHED_RING_FORWARD) returns the register-ring
    forward's bits, line-search trials included."""
    lq, x, u = (quadrotor_batch(nb, T=T, seed0=0) if nb == 4096
                else random_lq_batch(nb, 12, 4, T, seed=nb * 3 + T))
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    xi, ui = dev(x), dev(u)
    outs = []
    for ring in (False, True):
        s.set_schedule(ring_forward=ring)
        xn, un = torch.empty_like(xi), torch.empty_like(ui)
        pc = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
        st = torch.zeros((nb,), dtype=torch.int32, device="cuda")
        tr = torch.zeros((nb,), dtype=torch.int32, device="cuda")
        xa, ua = xi.clone(), ui.clone()
        for _ in range(3):  # cold start, then line searches against finite costs
            s.iterate(xa, ua, xn, un, pc, st, trials=tr, options=_lib.default_options(tol=-1.0))
            xa, xn, ua, un = xn, xa, un, ua
        torch.cuda.synchronize()
        outs.append((xa, ua, pc, st, tr))
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, rtol=0, atol=0, equal_nan=True)


@pytest.mark.parametrize("pipelined", [False, True])
def test_fit_zero_iterations_returns_inputs(gpu, pipelined):
    """for iter = 1:0 runs nothing (forward_pass.jl:161): fit returns x_init, u_init
    (the fit driver reads the caller's buffers in place; the gather copies them out)."""
    lq, x, u = random_lq_batch(6, 12, 4, 9, seed=11)
    s = Solver(12, 4, 9, 6)
    s.set_problem(lq)
    s.set_schedule(pipelined=pipelined)
    xi, ui = dev(x), dev(u)
    r = s.fit(xi, ui, max_iter=0)
    assert torch.equal(r.x, xi) and torch.equal(r.u, ui)
    assert (r.iters.cpu().numpy() == 0).all()
    assert (r.status.cpu().numpy() == _lib.TRAJ_MAX_ITER).all()
    assert torch.isinf(r.cost).all()
    # the inputs are never written (ownership rule, backward_pass.jl:332-333)
    r = s.fit(xi, ui, max_iter=5)
    assert torch.equal(xi.cpu(), torch.from_numpy(x)) and torch.equal(ui.cpu(), torch.from_numpy(u))


# -- LQ problems of other shapes: zero-padded onto the (12, 4) kernels ---------------
PAD_SHAPES = [(1, 1), (3, 2), (4, 1), (4, 2), (6, 2), (8, 3), (10, 4), (12, 1), (12, 3)]


@pytest.mark.parametrize("backward", ["auto", "block"])
@pytest.mark.parametrize("nx,nu", PAD_SHAPES)
def test_lq_padded_shapes_vs_oracle(gpu, nx, nu, backward):
    """Any nx ≤ 12, nu ≤ 4 runs on the (12, 4) kernels with zero rows/columns
    (exactly decoupled): backward, forward, iterate and fit against the C oracle,
    with the default backward kernel (one trajectory per wave at this batch) and the
    four-trajectories-per-wave one."""
    nb, T = 9, 25
    lq, x, u = random_lq_batch(nb, nx, nu, T, seed=17 * nx + nu)
    assert _lib.load().ilqr_supported(_lib.PROBLEM_LQ, nx, nu) == 1
    s = Solver(nx, nu, T, nb)
    s.set_problem(lq)
    s.set_schedule(backward=backward)
    xi, ui = dev(x), dev(u)
    d, K, st = s.backward(xi, ui)
    assert d.shape == (nb, T, nu) and K.shape == (nb, T, nu, nx)
    dc, Kc, _ = cref.lq_backward(lq, x, u, symmetrize=True)
    assert (st.cpu().numpy() == 0).all()
    assert rel(K, Kc) < TOL_GAIN_SYM and rel(d, dc) < TOL_GAIN_SYM
    pc = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
    xn, un, c, tr, st = s.forward(xi, ui, d, K, pc)
    xo, uo, co, tro = cref.lq_forward(lq, x, u, None, d.cpu().numpy(), K.cpu().numpy(), np.inf)
    assert rel(xn, xo) < TOL_ROLL and rel(un, uo) < TOL_ROLL and rel(c, co) < TOL_COST
    assert np.array_equal(tr.cpu().numpy(), tro)
    # iterate = backward + forward, bit for bit
    xn2, un2 = torch.empty_like(xi), torch.empty_like(ui)
    pc2 = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
    st2 = torch.zeros((nb,), dtype=torch.int32, device="cuda")
    s.iterate(xi, ui, xn2, un2, pc2, st2, options=_lib.default_options(tol=-1.0))
    torch.cuda.synchronize()
    assert torch.equal(xn2, xn) and torch.equal(un2, un) and torch.equal(pc2, c)
    r = s.fit(xi, ui, max_iter=15, tol=1e-8)
    xf, uf, cf, itf, stf = cref.lq_fit(lq, x, u, max_iter=15, tol=1e-8, symmetrize=True)
    assert r.x.shape == (nb, T + 1, nx) and r.u.shape == (nb, T, nu)
    assert np.array_equal(r.iters.cpu().numpy(), itf)
    assert rel(r.u, uf) < 1e-8 and rel(r.x, xf) < 1e-8


def test_lq_unsupported_shapes_raise(gpu):
    lib = _lib.load()
    for nx, nu in ((13, 1), (12, 5), (16, 4)):
        assert lib.ilqr_supported(_lib.PROBLEM_LQ, nx, nu) == 0
        with pytest.raises(NotImplementedError):
            Solver(nx, nu, 10, 4)


# -- single-process multi-GPU fit (ilqr_multi_*) --------------------------------------
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_fit_equals_single_handle(gpu, devices):
    """Shards (here several on one GPU: each shard has its own handle and stream,
    one host thread each) return exactly the single-handle fit, ragged splits too."""
    from ilqr_amd.multi import MultiSolver
    nb, T = 37, 20
    lq, x, u = random_lq_batch(nb, 12, 4, T, seed=5)
    x[7, 3, 1] = np.nan  # one NaN trajectory: reported, the others unaffected
    ms = MultiSolver(devices, 12, 4, T, nb)
    xo, uo, co, it, st, rc = ms.fit(lq, x, u, max_iter=12, tol=1e-8)
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    r = s.fit(dev(x), dev(u), max_iter=12, tol=1e-8)
    assert rc == r.call_status == _lib.ERR_NAN
    np.testing.assert_array_equal(xo, r.x.cpu().numpy())
    np.testing.assert_array_equal(uo, r.u.cpu().numpy())
    np.testing.assert_array_equal(co, r.cost.cpu().numpy())
    np.testing.assert_array_equal(it, r.iters.cpu().numpy())
    np.testing.assert_array_equal(st, r.status.cpu().numpy())
    ms.close()


def test_multi_fit_padded_shape(gpu):
    from ilqr_amd.multi import MultiSolver
    nb, T = 10, 15
    lq, x, u = random_lq_batch(nb, 6, 2, T, seed=6)
    xo, uo, co, it, st, rc = MultiSolver([0, 0], 6, 2, T, nb).fit(lq, x, u, max_iter=10, tol=1e-8)
    xf, uf, cf, itf, stf = cref.lq_fit(lq, x, u, max_iter=10, tol=1e-8, symmetrize=True)
    assert np.array_equal(it, itf) and rel(uo, uf) < 1e-8 and rel(xo, xf) < 1e-8


@pytest.mark.parametrize("nb,T", [(4096, 100), (13, 9)])
def test_ring_forward_pass_api_equals_register_ring(gpu, nb, T):
    """ilqr_forward (forward_pass) through either forward kernel: same bits, including
    exhausted line searches (prev_cost = -Inf → inputs returned, max_trials trials)."""
    lq, x, u = (quadrotor_batch(nb, T=T, seed0=1) if nb == 4096
                else random_lq_batch(nb, 12, 4, T, seed=nb + T))
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    xi, ui = dev(x), dev(u)
    d, K, _ = s.backward(xi, ui)
    pcs = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
    pcs[::3] = -float("inf")
    outs = []
    for ring in (False, True):
        s.set_schedule(ring_forward=ring)
        outs.append(s.forward(xi, ui, d, K, pcs, max_trials=5))
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, rtol=0, atol=0, equal_nan=True)
    assert (outs[1][4][::3].cpu().numpy() == _lib.TRAJ_LS_EXHAUSTED).all()


@pytest.mark.parametrize("max_iter,tol", [(1, -1.0), (3, -1.0), (6, 1e-8), (40, 1e-9)])
def test_fit_output_aliasing_input(gpu, max_iter, tol):
    """fit's last iteration writes the caller's x_out/u_out directly unless they
    overlap an input; in-place (x_out = x_init) calls take the gather path and return
    the same bits. Covers trajectories that converge before and at the last iteration."""
    import ctypes as C
    nb, T = 37, 20
    lq, x, u = random_lq_batch(nb, 12, 4, T, seed=21)
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    ref = s.fit(dev(x), dev(u), max_iter=max_iter, tol=tol)
    xi, ui = dev(x), dev(u)
    cost = torch.empty((nb,), dtype=torch.float64, device="cuda")
    it = torch.empty((nb,), dtype=torch.int32, device="cuda")
    st = torch.empty((nb,), dtype=torch.int32, device="cuda")
    s._bind_stream()
    o = _lib.default_options(max_iter=max_iter, tol=tol)
    p = C.c_void_p
    rc = s.lib.ilqr_fit(s.h, s._p(), C.byref(o), p(xi.data_ptr()), p(ui.data_ptr()), None,
                        p(xi.data_ptr()), p(ui.data_ptr()), p(cost.data_ptr()), p(it.data_ptr()),
                        p(st.data_ptr()))
    assert rc == ref.call_status
    assert torch.equal(xi, ref.x) and torch.equal(ui, ref.u) and torch.equal(it, ref.iters)
    assert torch.equal(st, ref.status) and torch.equal(cost, ref.cost)


@pytest.mark.parametrize("max_iter,tol", [(1, -1.0), (3, -1.0), (6, 1e-8)])
def test_fit_output_aliasing_x_traj(gpu, max_iter, tol):
    """x_out = x_traj (a tracking target the caller overwrites with the result): every
    iteration reads x_traj, so the last one must not write x_out directly — the gather
    does, after the iterations. Same bits as the call with separate buffers."""
    import ctypes as C
    nb, T = 37, 20
    lq, x, u = random_lq_batch(nb, 12, 4, T, seed=23)
    xt_np = np.ascontiguousarray(x[:, ::-1]) * 0.5
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    ref = s.fit(dev(x), dev(u), x_traj=dev(xt_np), max_iter=max_iter, tol=tol)
    xi, ui, xt = dev(x), dev(u), dev(xt_np)
    uo = torch.empty_like(ui)
    cost = torch.empty((nb,), dtype=torch.float64, device="cuda")
    it = torch.empty((nb,), dtype=torch.int32, device="cuda")
    st = torch.empty((nb,), dtype=torch.int32, device="cuda")
    s._bind_stream()
    o = _lib.default_options(max_iter=max_iter, tol=tol)
    p = C.c_void_p
    rc = s.lib.ilqr_fit(s.h, s._p(), C.byref(o), p(xi.data_ptr()), p(ui.data_ptr()), p(xt.data_ptr()),
                        p(xt.data_ptr()), p(uo.data_ptr()), p(cost.data_ptr()), p(it.data_ptr()),
                        p(st.data_ptr()))
    assert rc == ref.call_status
    assert torch.equal(xt, ref.x) and torch.equal(uo, ref.u) and torch.equal(it, ref.iters)
    assert torch.equal(st, ref.status) and torch.equal(cost, ref.cost)


@pytest.mark.parametrize("nb,T", [(4096, 100), (37, 17), (5, 3), (2051, 9)])
def test_fused_iteration_equals_two_launches(gpu, nb, T):
    """ILQR_SCHED_FUSED (one kernel: the block backward then the ring forward per wave)
    returns the bits of the two-launch iteration, through iterate and fit, with a NaN
    trajectory sharing a wave with clean ones."""
    lq, x, u = (quadrotor_batch(nb, T=T, seed0=0) if nb == 4096
                else random_lq_batch(nb, 12, 4, T, seed=nb * 5 + T))
    if nb != 4096:
        x[nb // 2, 1, 3] = np.nan
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    outs = []
    for fused in (False, True):
        s.set_schedule(backward="block", fused=fused)
        xi, ui = dev(x), dev(u)
        xn, un = torch.zeros_like(xi), torch.zeros_like(ui)  # a skipped (NaN) trajectory is never written
        pc = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
        st = torch.zeros((nb,), dtype=torch.int32, device="cuda")
        tr = torch.zeros((nb,), dtype=torch.int32, device="cuda")
        for _ in range(3):
            s.iterate(xi, ui, xn, un, pc, st, trials=tr, options=_lib.default_options(tol=-1.0))
            xi, xn, ui, un = xn, xi, un, ui
        r = s.fit(dev(x), dev(u), max_iter=6, tol=1e-8)
        torch.cuda.synchronize()
        outs.append((xi, ui, pc, st, tr, r.x, r.u, r.cost, r.iters, r.status))
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, rtol=0, atol=0, equal_nan=True)


# -- the forward pass on the 4-block MFMA (ILQR_SCHED_FORWARD_MFMA) ---------------------------
@pytest.mark.parametrize("name", LQ_FIXTURES)
def test_forward_mfma_matches_golden(gpu, name):
    """The MFMA form of the ring forward (ilqr_fwd_ring.h: lq_forward_wave_mfma) against
    the oracle's forward_pass fixtures: the same tolerances as the DPP form."""
    g = load(name)
    s, _ = solver_for(g)
    s.set_schedule(forward_mfma=True)
    nb = g["A"].shape[0]
    xt = dev(g["xtraj"]) if "xtraj" in g else None
    pc = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
    xn, un, c, tr, st = s.forward(dev(g["x"]), dev(g["u"]), dev(g["d"]), dev(g["K"]), pc, x_traj=xt)
    assert (st.cpu().numpy() == 0).all()
    assert rel(xn, g["fw_x"]) < TOL_ROLL and rel(un, g["fw_u"]) < TOL_ROLL
    assert rel(c, g["fw_cost"]) < TOL_COST
    assert np.array_equal(tr.cpu().numpy(), g["fw_trials"])


@pytest.mark.parametrize("name", LQ_FIXTURES)
def test_fit_mfma_matches_golden(gpu, name):
    g = load(name)
    meta = json.loads(str(g["meta"]))
    s, _ = solver_for(g)
    s.set_schedule(forward_mfma=True)
    xt = dev(g["xtraj"]) if "xtraj" in g else None
    r = s.fit(dev(g["x"]), dev(g["u"]), x_traj=xt, max_iter=meta["fit_max_iter"], tol=meta["tol"])
    assert r.call_status == 0
    assert np.array_equal(r.iters.cpu().numpy(), g["fit_iters"])
    assert rel(r.u, g["fit_u"]) < 1e-8 and rel(r.x, g["fit_x"]) < 1e-8


@pytest.mark.parametrize("nb,T", [(4096, 100), (37, 23)])
def test_fused_mfma_equals_split_mfma(gpu, nb, T):
    """With the MFMA forward, the fused iteration returns the split schedule's bits
    (iterate and fit, a NaN trajectory sharing a wave with clean ones), and it agrees
    with the DPP forward to rounding."""
    lq, x, u = (quadrotor_batch(nb, T=T, seed0=0) if nb == 4096
                else random_lq_batch(nb, 12, 4, T, seed=nb * 7 + T))
    if nb != 4096:
        x[nb // 2, 1, 3] = np.nan
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    outs = []
    for fused, mfma in ((False, True), (True, True), (True, False)):
        s.set_schedule(backward="block", fused=fused, forward_mfma=mfma)
        xi, ui = dev(x), dev(u)
        xn, un = torch.zeros_like(xi), torch.zeros_like(ui)
        pc = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
        st = torch.zeros((nb,), dtype=torch.int32, device="cuda")
        tr = torch.zeros((nb,), dtype=torch.int32, device="cuda")
        for _ in range(3):
            s.iterate(xi, ui, xn, un, pc, st, trials=tr, options=_lib.default_options(tol=-1.0))
            xi, xn, ui, un = xn, xi, un, ui
        r = s.fit(dev(x), dev(u), max_iter=6, tol=1e-8)
        torch.cuda.synchronize()
        outs.append((xi, ui, pc, st, tr, r.x, r.u, r.cost, r.iters, r.status))
    for a, b in zip(outs[0], outs[1]):
        torch.testing.assert_close(a, b, rtol=0, atol=0, equal_nan=True)
    ok = outs[1][3].cpu().numpy() == outs[2][3].cpu().numpy()
    assert ok.all()
    for a, b in zip(outs[1][:3], outs[2][:3]):  # x̄, ū, cost after three iterations
        a, b = a.cpu().numpy(), b.cpu().numpy()
        fin = np.isfinite(b)
        assert np.array_equal(np.isfinite(a), fin)
        assert np.abs(a[fin] - b[fin]).max() <= 1e-10 * max(np.abs(b[fin]).max(), 1e-300)


@pytest.mark.parametrize("nb,T,max_iter,tol,max_trials,nan,inplace", [
    (37, 17, 1, -1.0, None, False, False),
    (37, 17, 3, -1.0, None, True, False),
    (2051, 9, 2, -1.0, None, True, True),
    (37, 17, 6, 1e-8, None, False, False),
    (41, 20, 40, 1e-9, None, True, False),
    (37, 17, 5, -1.0, 1, False, False),
    (37, 17, 5, -1.0, 1, True, True),
    (5, 3, 4, 1e-3, None, False, True),
])
def test_fit_in_kernel_init(gpu, nb, T, max_iter, tol, max_trials, nan, inplace):
    """The fused path's fit initialises its per-trajectory state in the first
    iteration's kernel (no fit_init launch); the split schedule launches fit_init.
    Same bits and call status (the gather's host-mapped flags), over early stops
    (converged, exhausted line searches, NaN), fits whose poll ends before max_iter,
    in-place calls (x_out = x_init: the gather's copy path) and ragged batches."""
    import ctypes as C
    lq, x, u = random_lq_batch(nb, 12, 4, T, seed=nb + 7 * T + max_iter)
    if nan:
        x[nb // 3, 1, 2] = np.nan
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    outs = []
    for fused in (False, True):
        s.set_schedule(backward="block", fused=fused)
        xi, ui = dev(x), dev(u)
        if inplace:
            cost = torch.empty((nb,), dtype=torch.float64, device="cuda")
            it = torch.empty((nb,), dtype=torch.int32, device="cuda")
            st = torch.empty((nb,), dtype=torch.int32, device="cuda")
            s._bind_stream()
            o = _lib.default_options(max_iter=max_iter, tol=tol, max_trials=max_trials)
            p = C.c_void_p
            rc = s.lib.ilqr_fit(s.h, s._p(), C.byref(o), p(xi.data_ptr()), p(ui.data_ptr()), None,
                                p(xi.data_ptr()), p(ui.data_ptr()), p(cost.data_ptr()),
                                p(it.data_ptr()), p(st.data_ptr()))
            outs.append((rc, xi, ui, cost, it, st))
        else:
            r = s.fit(xi, ui, max_iter=max_iter, tol=tol, max_trials=max_trials)
            outs.append((r.call_status, r.x, r.u, r.cost, r.iters, r.status))
    assert outs[0][0] == outs[1][0]
    for a, b in zip(outs[0][1:], outs[1][1:]):
        torch.testing.assert_close(a, b, rtol=0, atol=0, equal_nan=True)
    if nan:
        assert outs[1][5][nb // 3].item() == _lib.TRAJ_NAN
