"""CPU tests: pin the oracle (CPU restatement of the reference) with known-answer
tests derived from the reference's own tests and algebra, and check the
committed golden vectors and the C restatement against it."""
import json
import os

import numpy as np
import pytest

from ilqr_amd.problems import quadrotor_batch, random_lq_batch
from oracle import cref, dual
from oracle import ilqr_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(b).max(), 1e-300))


# -- AD restatement (ForwardDiff) --------------------------------------------------
def test_dual_ad_matches_analytic_lq_derivatives():
    """ForwardDiff on linear/quadratic closures is exact; so must the restatement be
    (linearize_dynamics :25-40, immediate_cost_quadratization :81-109,
    final_cost_quadratization :134-153)."""
    rng = np.random.default_rng(3)
    n, m = 12, 4
    A, B = rng.standard_normal((n, n)), rng.standard_normal((n, m))
    Q, R, Qf = rng.standard_normal((n, n)), rng.standard_normal((m, m)), rng.standard_normal((n, n))
    f, l, lf = O.lq_closures(A, B, Q, R, Qf)
    x, u = rng.standard_normal(n), rng.standard_normal(m)
    Aad = dual.jacobian(lambda z: f(z, u), x)
    Bad = dual.jacobian(lambda z: f(x, z), u)
    assert np.array_equal(Aad, A) and np.array_equal(Bad, B)
    # strip the analytic shortcut to force the generic AD path
    plain_l = lambda xx, uu: xx @ (Q @ xx) + uu @ (R @ uu)  # noqa: E731
    plain_lf = lambda xx: xx @ (Qf @ xx)  # noqa: E731
    ad = O.immediate_cost_quadratization(x, u, plain_l)
    an = l.quad(x, u)
    for a, b in zip(ad[1:], an[1:]):
        assert rel(a, b) < 1e-14 if np.abs(b).max() > 0 else np.abs(a).max() == 0
    fad = O.final_cost_quadratization(x, plain_lf)
    fan = lf.fquad(x)
    assert rel(fad[1], fan[1]) < 1e-14 and rel(fad[2], fan[2]) < 1e-14


def test_linearisation_of_linear_dynamics_is_exact():
    """Repaired test/test_linearize_dynamics.jl:24-25: for linear f the linearised
    one-step prediction A x + B u equals f(x, u) (the test's 1e-10 bound)."""
    lq, x, u = random_lq_batch(1, 12, 4, 10, seed=5)
    f = lambda xx, uu: lq.A[0] @ xx + lq.B[0] @ uu  # noqa: E731  (no analytic shortcut)
    for t in range(10):
        A, B = O.linearize_dynamics(x[0, t], u[0, t], f)
        pred = A @ x[0, t] + B @ u[0, t]
        assert np.abs(pred - x[0, t + 1]).max() < 1e-10


def test_twolink_constants_and_ik():
    """test/2_link_example/2_link_helper_functions.jl:5-26 constants; values quoted
    in SURVEY.md §8a12 (θ* = (-1.6804522359448377, 1.9714279194962687))."""
    k = json.load(open(os.path.join(GOLD, "twolink_constants.json")))
    assert O.TwoLink.alpha == 0.8333333333333335
    assert O.TwoLink.beta == 0.25000000000000006
    assert abs(O.TwoLink.delta - 1 / 6) < 1e-15
    th = O.TwoLink.inverse_kinematics(O.TwoLink.target_tool_loc)
    assert th[0] == -1.6804522359448377 and th[1] == 1.9714279194962687
    assert th.tolist() == k["theta_star"]
    # forward kinematics of θ* reaches the target tool location
    l1, l2 = O.TwoLink.l1, O.TwoLink.l2
    tip = (l1 * np.cos(th[0]) + l2 * np.cos(th[0] + th[1]), l1 * np.sin(th[0]) + l2 * np.sin(th[0] + th[1]))
    assert np.allclose(tip, O.TwoLink.target_tool_loc, atol=1e-12)


def test_twolink_ad_matches_central_differences():
    TL = O.TwoLink
    rng = np.random.default_rng(1)
    for _ in range(3):
        x, u = rng.random(4), rng.standard_normal(2)
        A, B = O.linearize_dynamics(x, u, TL.dynamicsf)
        e = 1e-6
        Afd = np.stack([(TL.dynamicsf(x + e * np.eye(4)[i], u) - TL.dynamicsf(x - e * np.eye(4)[i], u)) / (2 * e)
                        for i in range(4)], 1)
        Bfd = np.stack([(TL.dynamicsf(x, u + e * np.eye(2)[i]) - TL.dynamicsf(x, u - e * np.eye(2)[i])) / (2 * e)
                        for i in range(2)], 1)
        assert np.abs(A - Afd).max() < 1e-8 and np.abs(B - Bfd).max() < 1e-8


def test_twolink_coriolis_quirk():
    """`for k in length(θ)` (2_link_helper_functions.jl:43) iterates k = 2 only:
    C = ½ θ̇₂ ∂M/∂θ₂ transposed — NOT the physical Coriolis matrix."""
    th, thd = np.array([0.3, 0.7]), np.array([0.5, -1.1])
    C = np.asarray(O.TwoLink.coriolis_matrix(th, thd), dtype=float)
    b, s2 = O.TwoLink.beta, np.sin(0.7)
    exp = np.array([[-b * s2 * thd[1], -0.5 * b * s2 * thd[1]], [-0.5 * b * s2 * thd[1], 0.0]])
    assert np.allclose(C, exp, rtol=0, atol=1e-15)


def test_twolink_fit_decreases_cost_to_a_stationary_point():
    """Repaired test/test_iLQR.jl (broken as written: Float64 max_iter, 1×404
    state matrix): fit from a seeded x₀ with u₀ = 0 terminates by the tol test
    with a monotonically decreasing cost (the @assert at forward_pass.jl:168).
    The test's `final_cost(x̄[end]) < 0.01` does not hold for this oracle at
    T = 100…300 (the running cost dominates); see DESIGN.md §Oracle."""
    TL = O.TwoLink
    T = 100
    x0 = np.random.default_rng(42).random(4)
    x = O.rollout(x0, np.zeros((T, 2)), TL.dynamicsf)
    hist = []
    xf, uf = O.fit(x, np.zeros((T, 2)), TL.dynamicsf, TL.immediate_cost, TL.final_cost,
                   max_iter=200, tol=1e-6, max_trials=60, history=hist)
    c = [h["cost"] for h in hist]
    assert all(b < a for a, b in zip(c, c[1:]))
    assert hist[-1]["du2"] <= 1e-6 and len(hist) < 200
    assert TL.final_cost(xf[-1]) < TL.final_cost(x[-1])


# -- LQ known answers --------------------------------------------------------------
@pytest.mark.parametrize("seed", [0, 1])
def test_lq_fit_converges_to_kkt_solution(seed):
    """iLQR's fixed point has δu ≡ 0, i.e. ∇_u J = 0, so fit converges to the exact
    minimiser of the LQ problem independent of μ."""
    lq, x, u = quadrotor_batch(1, T=20, seed0=seed)
    f, l, lf = O.lq_closures(lq.A[0], lq.B[0], lq.Q[0], lq.R[0], lq.Qf[0])
    xf, uf = O.fit(x[0], u[0], f, l, lf, max_iter=50, tol=1e-14, max_trials=60)
    X, U = O.lq_kkt_solution(lq.A[0], lq.B[0], lq.Q[0], lq.R[0], lq.Qf[0], x[0, 0], 20)
    assert rel(uf, U) < 1e-6 and rel(xf, X) < 1e-6


def test_literal_step_back_amplifies_asymmetry():
    """Documents the reference-numerics finding: the literal
    update (backward_pass.jl:270) diverges on the headline instances at T = 100,
    while the symmetrised recursion (identity in exact arithmetic) does not."""
    lq, x, u = quadrotor_batch(1, T=100, seed0=0)
    f, l, lf = O.lq_closures(lq.A[0], lq.B[0], lq.Q[0], lq.R[0], lq.Qf[0])
    d, K = O.backward_pass(x[0], u[0], f, l, lf, symmetrize=True)
    assert np.isfinite(K).all() and np.abs(K).max() < 1e3
    try:
        with np.errstate(all="ignore"):
            dl, Kl = O.backward_pass(x[0], u[0], f, l, lf)
        diverged = not np.isfinite(Kl).all() or rel(Kl, K) > 1e-3
    except (np.linalg.LinAlgError, AssertionError):
        diverged = True
    assert diverged
    # on a short horizon the two agree to rounding
    d20, K20 = O.backward_pass(x[0, :21], u[0, :20], f, l, lf)
    d20s, K20s = O.backward_pass(x[0, :21], u[0, :20], f, l, lf, symmetrize=True)
    assert rel(K20, K20s) < 1e-9


def test_fit_returns_previous_iterate_and_rejects_float_max_iter():
    """forward_pass.jl:171-178: on convergence fit returns the iterate BEFORE the
    update; forward_pass.jl:152: max_iter::Int64 (test_iLQR.jl:4's 1e5 is a TypeError)."""
    lq, x, u = quadrotor_batch(1, T=10, seed0=3)
    f, l, lf = O.lq_closures(lq.A[0], lq.B[0], lq.Q[0], lq.R[0], lq.Qf[0])
    with pytest.raises(TypeError):
        O.fit(x[0], u[0], f, l, lf, max_iter=1e5)
    hist = []
    xf, uf = O.fit(x[0], u[0], f, l, lf, max_iter=50, tol=1e-6, max_trials=60, history=hist)
    # replay: the returned iterate is the input of the last (converging) iteration
    xi, ui, pc = x[0], u[0], np.inf
    for h in hist[:-1]:
        d, K = O.backward_pass(xi, ui, f, l, lf)
        xi, ui, pc = O.forward_pass(xi, ui, np.zeros_like(xi), d, K, pc, f, l, lf)
    assert np.array_equal(xf, xi) and np.array_equal(uf, ui)
    assert hist[-1]["du2"] <= 1e-6 and all(h["du2"] > 1e-6 for h in hist[:-1])


def test_shape_assertions():
    lq, x, u = quadrotor_batch(1, T=5, seed0=0)
    f, l, lf = O.lq_closures(lq.A[0], lq.B[0], lq.Q[0], lq.R[0], lq.Qf[0])
    with pytest.raises(AssertionError):
        O.backward_pass(x[0, :-1], u[0], f, l, lf)   # backward_pass.jl:329


# -- golden vectors and the C restatement --------------------------------------------
def _load(name):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name", ["quad_t16", "quad_t100_sym", "dense_t16", "dense_t64_sym", "dense_xtraj"])
def test_golden_reproduces_and_c_oracle_agrees(name):
    g = _load(name)
    meta = json.loads(str(g["meta"]))
    from ilqr_amd.problems import LQBatch
    lq = LQBatch(g["A"], g["B"], g["Q"], g["R"], g["Qf"])
    sym = meta["symmetrize"]
    xt = g.get("xtraj")
    # numpy oracle reproduces the committed vectors (first trajectory)
    f, l, lf = O.lq_closures(lq.A[0], lq.B[0], lq.Q[0], lq.R[0], lq.Qf[0])
    d, K = O.backward_pass(g["x"][0], g["u"][0], f, l, lf, symmetrize=sym)
    assert rel(K, g["K"][0]) < 1e-12 and rel(d, g["d"][0]) < 1e-12
    # C restatement agrees with the fixtures for the whole batch
    dc, Kc, st = cref.lq_backward(lq, g["x"], g["u"], symmetrize=sym)
    assert (st == 0).all()
    assert rel(Kc, g["K"]) < 1e-9 and rel(dc, g["d"]) < 1e-9
    xn, un, c, tr = cref.lq_forward(lq, g["x"], g["u"], xt, g["d"], g["K"], np.inf)
    assert rel(xn, g["fw_x"]) < 1e-10 and rel(un, g["fw_u"]) < 1e-10
    assert rel(c, g["fw_cost"]) < 1e-11 and np.array_equal(tr, g["fw_trials"])
    xo, uo, co, it, st = cref.lq_fit(lq, g["x"], g["u"], x_traj=xt, max_iter=meta["fit_max_iter"],
                                     tol=meta["tol"], symmetrize=sym)
    assert np.array_equal(it, g["fit_iters"])
    assert rel(uo, g["fit_u"]) < 1e-8 and rel(xo, g["fit_x"]) < 1e-8


def test_golden_twolink_reproduces():
    g = _load("twolink_t50")
    TL = O.TwoLink
    d, K = O.backward_pass(g["x"][0], g["u"][0], TL.dynamicsf, TL.immediate_cost, TL.final_cost)
    assert rel(K, g["K"][0]) < 1e-12 and rel(d, g["d"][0]) < 1e-12


def test_c_oracle_twolink_agrees_with_golden():
    """The C restatement's 2-link path (dual-number AD, oracle/ilqr_ref.c) against
    the Python oracle's frozen fixture: backward, forward and fit."""
    g = _load("twolink_t50")
    d, K, st = cref.tl_backward(g["x"], g["u"])
    assert (st == 0).all() and rel(d, g["d"]) < 1e-12 and rel(K, g["K"]) < 1e-12
    xn, un, c, tr = cref.tl_forward(g["x"], g["u"], None, g["d"], g["K"], np.inf)
    assert (tr == 1).all() and rel(xn, g["fw_x"]) < 1e-13 and rel(un, g["fw_u"]) < 1e-13
    assert rel(c, g["fw_cost"]) < 1e-14
    xo, uo, co, it, st = cref.tl_fit(g["x"], g["u"], max_iter=40)
    assert np.array_equal(it, g["fit_iters"]) and (st == 1).all()
    assert rel(xo, g["fit_x"]) < 1e-12 and rel(uo, g["fit_u"]) < 1e-12


def test_c_oracle_twolink_nu1_agrees_with_golden():
    """The C restatement's nu = 1 variant (f(x, [u₁, 0])) against the Python oracle's
    twolink_nu1_t50 fixture (TwoLink.dynamicsf_nu1): backward, forward and fit."""
    g = _load("twolink_nu1_t50")
    d, K, st = cref.tl_backward(g["x"], g["u"])
    assert d.shape[-1] == 1 and K.shape[-2:] == (1, 4)
    assert (st == 0).all() and rel(d, g["d"]) < 1e-12 and rel(K, g["K"]) < 1e-12
    xn, un, c, tr = cref.tl_forward(g["x"], g["u"], None, g["d"], g["K"], np.inf)
    assert (tr == 1).all() and rel(xn, g["fw_x"]) < 1e-13 and rel(un, g["fw_u"]) < 1e-13
    assert rel(c, g["fw_cost"]) < 1e-14
    xo, uo, co, it, st = cref.tl_fit(g["x"], g["u"], max_iter=40)
    assert np.array_equal(it, g["fit_iters"]) and (st == 1).all()
    assert rel(xo, g["fit_x"]) < 1e-12 and rel(uo, g["fit_u"]) < 1e-12
