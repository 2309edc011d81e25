"""GPU parity of the floating-base RBD family (include/ilqr.h ilqr_floating_*): the
reference's RBD script (test/RBD_2_link_example/, 2Dof_arm.urdf floating, zero gravity,
nx = 16, nu = 8, T = 1000) fitted natively, against the restatement the generic closure
path is checked with (tests/closures.py rbd_floating_arm on numpy / oracle.jet; parity
against RigidBodyDynamics.jl itself is unpinned: it is not runnable here).

Tolerances (fp64): one RK4 step rel 1e-12 (the same algorithms in another operation
order); the dual-number Jacobians rel 1e-10 against oracle.jet's forward mode; fit
iterates and costs rel 1e-8 with exact iteration counts and statuses, as the closure
path's test_rbd_caller_fit_t1000."""
import numpy as np
import pytest
import torch

from closures import jet_ns, rbd_cost_quads, rbd_floating_arm
from ilqr_amd import _lib, api
from ilqr_amd.floating import (FloatingSolver, floating_closures, rbd_example_problem,
                               rbd_initial_state)
from oracle import closure_fit as CF
from oracle import jet

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a, float)
    b = b.cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b, float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def random_states(n, seed=3):
    rng = np.random.default_rng(seed)
    x = np.zeros((n, 16))
    x[:, 0:3] = 0.4 * rng.standard_normal((n, 3))       # MRP
    x[:, 3:6] = rng.standard_normal((n, 3))
    x[:, 6:8] = rng.uniform(-3.0, 3.0, (n, 2))
    x[:, 8:16] = rng.standard_normal((n, 8))
    u = 5.0 * rng.standard_normal((n, 8))
    return x, u


def script_batch(nb, T, seed=7):
    """The script's start (rest state, zero inputs, x_init = rollout: animate_RBD_2_link.jl:19-25)
    plus perturbed copies, rolled out by the restatement."""
    fj, _, _ = rbd_floating_arm(jet_ns())
    x = np.zeros((nb, T + 1, 16))
    x[:, 0] = rbd_initial_state()
    x[1:, 0, 8:] = 0.05 * np.random.default_rng(seed).standard_normal((nb - 1, 8))
    u = np.zeros((nb, T, 8))
    for t in range(T):
        x[:, t + 1] = fj(x[:, t], u[:, t])
    return x, u


def test_floating_dynamics_vs_restatement(gpu):
    fj, _, _ = rbd_floating_arm(jet_ns())
    x, u = random_states(257)
    s = FloatingSolver(rbd_example_problem(), 1, 1)
    try:
        y = s.dynamics(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda())
    finally:
        s.close()
    assert rel(y, fj(x, u)) < 1e-12


def test_floating_linearize_vs_forward_mode(gpu):
    fj, _, _ = rbd_floating_arm(jet_ns())
    nb, T = 3, 5
    xs, us = random_states(nb * (T + 1), seed=11)
    x = xs.reshape(nb, T + 1, 16)
    u = us[: nb * T].reshape(nb, T, 8)
    s = FloatingSolver(rbd_example_problem(), T, nb)
    try:
        A, Bm = s.linearize(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda())
    finally:
        s.close()
    Aj, Bj = jet.jacobians(fj, x[:, :T].reshape(-1, 16), u.reshape(-1, 8))
    assert rel(A.reshape(-1, 16, 16), Aj) < 1e-10
    assert rel(Bm.reshape(-1, 16, 8), Bj) < 1e-10


def test_floating_fit_script_shape_vs_closure_oracle(gpu):
    """The script's fit (T = 1000) natively against the batched closure oracle (ForwardDiff's
    algorithm for A, B; the closed-form cost tiles; the C restatement's recursion)."""
    nb, T, iters = 2, 1000, 4
    x, u = script_batch(nb, T)
    s = FloatingSolver(rbd_example_problem(), T, nb)
    try:
        r = s.fit(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda(), max_iter=iters, tol=1e-6,
                  history=True)
    finally:
        s.close()
    fj, lj, lfj = rbd_floating_arm(jet_ns())
    o = CF.fit(x, u, fj, lj, lfj, *rbd_cost_quads(), max_iter=iters, tol=1e-6)
    assert r.iters.tolist() == o["iters"].tolist()
    # the per-iteration record (ilqr_floating_fit_ex): trials and costs as the oracle's
    assert r.history["trials"][:iters].cpu().tolist() == o["history"]["trials"].tolist()
    assert rel(r.history["cost"][:iters], o["history"]["cost"]) < 1e-8
    assert r.status.tolist() == o["status"].tolist()
    assert rel(r.cost, o["cost"]) < 1e-8
    assert rel(r.x, o["x"]) < 1e-8 and rel(r.u, o["u"]) < 1e-8


def test_floating_fit_batch_converges_like_the_oracle(gpu):
    """A batch of 33 perturbed starts at T = 60 until convergence (tol 1e-6): statuses,
    iteration counts, iterates."""
    nb, T = 33, 60
    x, u = script_batch(nb, T, seed=5)
    s = FloatingSolver(rbd_example_problem(), T, nb)
    try:
        r = s.fit(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda(), max_iter=30, tol=1e-6)
    finally:
        s.close()
    fj, lj, lfj = rbd_floating_arm(jet_ns())
    o = CF.fit(x, u, fj, lj, lfj, *rbd_cost_quads(), max_iter=30, tol=1e-6)
    assert r.status.tolist() == o["status"].tolist()
    assert r.iters.tolist() == o["iters"].tolist()
    assert rel(r.x, o["x"]) < 1e-8 and rel(r.u, o["u"]) < 1e-8 and rel(r.cost, o["cost"]) < 1e-8


def test_api_fit_dispatches_the_recognised_closures(gpu):
    """ilqr_amd.fit with the family's reference-API callables runs the native fit (same
    bits as FloatingSolver.fit) and keeps one cached handle."""
    from ilqr_amd import cache
    api.clear_cache()
    p = rbd_example_problem()
    nb, T = 2, 40
    x, u = script_batch(nb, T, seed=9)
    xt, ut = torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda()
    xf, uf = api.fit(xt, ut, *floating_closures(p), max_iter=6)
    xf2, uf2 = api.fit(xt, ut, *floating_closures(p), max_iter=6)
    assert cache.size() == 1
    s = FloatingSolver(p, T, nb)
    try:
        r = s.fit(xt, ut, max_iter=6, tol=1e-6)
    finally:
        s.close()
    assert torch.equal(xf, r.x) and torch.equal(uf, r.u) and torch.equal(xf2, r.x)
    # the callables evaluate the same functions one point at a time
    dyn, cost, fcost = floating_closures(p)
    fj, lj, lfj = rbd_floating_arm(jet_ns())
    assert rel(dyn(x[0, 0], u[0, 0]), fj(x[:1, 0], u[:1, 0])[0]) < 1e-12
    assert abs(cost(x[0, 3], u[0, 3]) - float(lj(x[:1, 3], u[:1, 3])[0])) <= 1e-12 * abs(cost(x[0, 3], u[0, 3]))
    assert abs(fcost(x[0, T]) - float(lfj(x[:1, T])[0])) <= 1e-12 * abs(fcost(x[0, T]))
    # the script builds state_traj with 1000 dynamicsf calls: one cached handle serves them,
    # and a device tensor stays on its device
    n0 = cache.size()
    ys = [dyn(xt[0, t], ut[0, t]) for t in range(20)]
    assert cache.size() == n0 and isinstance(ys[0], torch.Tensor) and ys[0].is_cuda
    assert rel(ys[3], fj(x[:1, 3], u[:1, 3])[0]) < 1e-12
    api.clear_cache()


def test_floating_nan_state_is_reported(gpu):
    """A NaN in one trajectory's start stops that trajectory with status NAN; the other
    one fits as alone (the reference asserts on NaN: forward_pass.jl:89-90)."""
    nb, T = 2, 30
    x, u = script_batch(nb, T, seed=13)
    x[1, 0, 9] = np.nan
    x[1, 1:] = np.nan
    s = FloatingSolver(rbd_example_problem(), T, nb)
    s1 = FloatingSolver(rbd_example_problem(), T, 1)
    try:
        r = s.fit(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda(), max_iter=5)
        r1 = s1.fit(torch.from_numpy(x[:1].copy()).cuda(), torch.from_numpy(u[:1].copy()).cuda(), max_iter=5)
    finally:
        s.close()
        s1.close()
    assert r.call_status == _lib.ERR_NAN
    assert int(r.status[1]) == _lib.TRAJ_NAN
    assert torch.equal(r.x[0], r1.x[0]) and torch.equal(r.u[0], r1.u[0])


def test_floating_backward_forward_vs_closure_oracle(gpu):
    """backward_pass / forward_pass one at a time (ilqr_floating_backward / _forward, and
    ilqr_amd.backward_pass / forward_pass with the family's callables) against the closure
    oracle's tiles recursion and rollout, including a forward that must halve α."""
    from oracle import cref
    nb, T = 3, 80
    x, u = script_batch(nb, T, seed=17)
    p = rbd_example_problem()
    fj, lj, lfj = rbd_floating_arm(jet_ns())
    tl = CF.derivative_tiles(x, u, fj, *rbd_cost_quads())
    d_o, K_o, _ = cref.tiles_backward(tl, mu=0.01, symmetrize=True)
    xt, ut = torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda()
    d, K = api.backward_pass(xt, ut, *floating_closures(p))
    assert rel(d, d_o) < 1e-9 and rel(K, K_o) < 1e-9
    # prev_cost: Inf (accept trial 1), the oracle's trial-1 cost minus a bit on trajectory 0
    # (trial 1 rejected there, a later α accepted)
    _, _, c1, _, _ = CF.forward_pass(x, u, np.zeros_like(x), d_o, K_o, np.full(nb, np.inf), fj, lj, lfj)
    prev = np.full(nb, np.inf)
    prev[0] = c1[0] * (1.0 - 1e-9)
    xo, uo, co, tro, ok = CF.forward_pass(x, u, np.zeros_like(x), d_o, K_o, prev, fj, lj, lfj)
    s = FloatingSolver(p, T, nb)
    try:
        xn, un, cost, trials, st = s.forward(xt, ut, torch.from_numpy(d_o).cuda(), torch.from_numpy(K_o).cuda(),
                                             torch.from_numpy(prev).cuda())
    finally:
        s.close()
    assert trials.tolist() == tro.tolist() and st.tolist() == [0 if a else 3 for a in ok]
    assert rel(cost, co) < 1e-10 and rel(xn, xo) < 1e-10 and rel(un, uo) < 1e-10
    assert int(trials[0]) > 1


@pytest.mark.parametrize("nb,shrink,alpha0,cand", [(17, 0.5, 1.0, 16), (4, 0.7, 0.9, 64), (70, 0.5, 1.0, 4)])
def test_floating_forward_slots_rounds_and_partial_workgroups(gpu, nb, shrink, alpha0, cand, monkeypatch):
    """The line search across rounds of trials: prev_cost set per trajectory so that the
    accepted trial falls anywhere in 1..6 or the search exhausts at max_trials = 6 —
    trials > 1 come from their lanes' slots, an exhausted search returns the inputs;
    every trajectory as the closure oracle's forward_pass, the lanes a trajectory pinned
    (ILQR_FB_CAND; by default such batches run 64). B = 17 runs 16 lanes a
    trajectory (17 · 16 lanes: the last workgroup partly empty), B = 4 runs 64 (one round
    covers every trial) with a non-dyadic shrink (trial j's α = α₀ multiplied by shrink
    j − 1 times, as the reference's `α *= shrink`), B = 70 runs 4 (trials 5-6 in a second
    round)."""
    from oracle import cref
    T, mt = 30, 6
    x, u = script_batch(nb, T, seed=29)
    u = u + 0.5 * np.random.default_rng(31).standard_normal(u.shape)
    fj, lj, lfj = rbd_floating_arm(jet_ns())
    # the iterate a rollout of u (the forward's inputs must be a consistent trajectory)
    for t in range(T):
        x[:, t + 1] = fj(x[:, t], u[:, t])
    tl = CF.derivative_tiles(x, u, fj, *rbd_cost_quads())
    d, K, _ = cref.tiles_backward(tl, mu=0.01, symmetrize=True)
    d = 32.0 * d  # large early steps: the cost falls over the first trials
    zt = np.zeros_like(x)
    alphas = [alpha0]
    for _ in range(7):
        alphas.append(alphas[-1] * shrink)
    # the cost of trial j alone, j = 1..8
    c = np.stack([CF.forward_pass(x, u, zt, d, K, np.full(nb, np.inf), fj, lj, lfj, max_trials=1,
                                  alpha0=a)[2] for a in alphas], axis=1)
    prev = np.full(nb, np.inf)
    for b in range(nb):
        k = 1 + b % 7  # aim at trial k: prev just under the smallest cost of trials 1..k−1
        if k > 1:       # (a tie would be decided by rounding: GPU and oracle differ at 1e-12)
            prev[b] = c[b, :k - 1].min() * (1.0 - 1e-9)
    xo, uo, co, tro, ok = CF.forward_pass(x, u, zt, d, K, prev, fj, lj, lfj, max_trials=mt, alpha0=alpha0,
                                          shrink=shrink)
    assert len(set(tro[ok].tolist())) >= 3 and ((~ok).any() or nb <= 4)
    o = _lib.default_options(max_trials=mt, alpha0=alpha0, shrink=shrink)
    monkeypatch.setenv("ILQR_FB_CAND", str(cand))  # the lanes a trajectory, read at creation
    s = FloatingSolver(rbd_example_problem(), T, nb)
    try:
        xn, un, cost, trials, st = s.forward(*(torch.from_numpy(a).cuda() for a in (x, u, d, K, prev)),
                                             options=o)
    finally:
        s.close()
    assert trials.tolist() == tro.tolist()
    assert st.tolist() == [_lib.TRAJ_OK if a else _lib.TRAJ_LS_EXHAUSTED for a in ok]
    assert rel(cost, co) < 1e-10 and rel(xn, xo) < 1e-10 and rel(un, uo) < 1e-10
    ex = ~ok
    assert np.array_equal(xn.cpu().numpy()[ex], x[ex]) and np.array_equal(un.cpu().numpy()[ex], u[ex])


def test_floating_fit_x_traj_and_edges(gpu):
    """x_traj enters the line search's cost (forward_pass.jl:187-190) as in the oracle;
    max_iter = 0 returns the inputs (status MAX_ITER); two fits on one handle are
    bit-identical."""
    nb, T = 2, 40
    x, u = script_batch(nb, T, seed=21)
    xtraj = 0.1 * np.random.default_rng(3).standard_normal(x.shape)
    xt, ut, xtr = (torch.from_numpy(a).cuda() for a in (x, u, xtraj))
    s = FloatingSolver(rbd_example_problem(), T, nb)
    try:
        r = s.fit(xt, ut, max_iter=5, tol=1e-6, x_traj=xtr)
        r2 = s.fit(xt, ut, max_iter=5, tol=1e-6, x_traj=xtr)
        r0 = s.fit(xt, ut, max_iter=0)
    finally:
        s.close()
    fj, lj, lfj = rbd_floating_arm(jet_ns())
    o = CF.fit(x, u, fj, lj, lfj, *rbd_cost_quads(), x_traj=xtraj, max_iter=5, tol=1e-6)
    assert r.iters.tolist() == o["iters"].tolist() and r.status.tolist() == o["status"].tolist()
    assert rel(r.x, o["x"]) < 1e-8 and rel(r.cost, o["cost"]) < 1e-8
    assert torch.equal(r.x, r2.x) and torch.equal(r.u, r2.u) and torch.equal(r.cost, r2.cost)
    assert torch.equal(r0.x, xt) and torch.equal(r0.u, ut)
    assert r0.status.tolist() == [_lib.TRAJ_MAX_ITER] * nb and r0.iters.tolist() == [0] * nb


def _problem_of(model):
    from ilqr_amd.floating import FloatingProblem
    from ilqr_amd.urdf import Chain
    ch = Chain(["j1", "j2"], np.array(model["R0"], float), np.array(model["p"], float),
               np.array(model["axis"], float), np.array(model["mass"], float), np.array(model["com"], float),
               np.array(model["Ic"], float), np.zeros(3), float(model["base_mass"]),
               np.array(model["base_com"], float), np.array(model["base_Ic"], float))
    return FloatingProblem(ch)


def test_floating_general_mechanism_vs_restatement(gpu):
    """A mechanism with every term nonzero (tests/closures.py coupled_floating_model:
    tilted and oblique joints, COMs off the joint origins, a base with products of
    inertia): one step, the Jacobians, a fit and energy conservation at u = 0."""
    from closures import coupled_floating_model, floating_energy
    md = coupled_floating_model()
    p = _problem_of(md)
    fj, lj, lfj = rbd_floating_arm(jet_ns(), model=md)
    x, u = random_states(129, seed=8)
    s = FloatingSolver(p, 1, 1)
    try:
        y = s.dynamics(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda())
        # energy at u = 0 over 200 steps on the device
        xe = torch.from_numpy(x[:8].copy()).cuda()
        z = torch.zeros(8, 8, dtype=torch.float64, device="cuda")
        e0 = floating_energy(x[:8], md)
        for _ in range(200):
            xe = s.dynamics(xe, z)
        e1 = floating_energy(xe.cpu().numpy(), md)
    finally:
        s.close()
    assert rel(y, fj(x, u)) < 1e-12
    assert np.abs(e1 - e0).max() / e0.max() < 1e-7
    nb, T = 2, 50
    x0 = np.zeros((nb, T + 1, 16))
    x0[:, 0] = rbd_initial_state()
    x0[1, 0, 8:] = 0.05
    uu = np.zeros((nb, T, 8))
    for t in range(T):
        x0[:, t + 1] = fj(x0[:, t], uu[:, t])
    s = FloatingSolver(p, T, nb)
    try:
        A, Bm = s.linearize(torch.from_numpy(x0).cuda(), torch.from_numpy(uu).cuda())
        r = s.fit(torch.from_numpy(x0).cuda(), torch.from_numpy(uu).cuda(), max_iter=4)
    finally:
        s.close()
    Aj, Bj = jet.jacobians(fj, x0[:, :T].reshape(-1, 16), uu.reshape(-1, 8))
    assert rel(A.reshape(-1, 16, 16), Aj) < 1e-10 and rel(Bm.reshape(-1, 16, 8), Bj) < 1e-10
    o = CF.fit(x0, uu, fj, lj, lfj, *rbd_cost_quads(), max_iter=4)
    assert r.iters.tolist() == o["iters"].tolist() and r.status.tolist() == o["status"].tolist()
    assert rel(r.x, o["x"]) < 1e-8 and rel(r.u, o["u"]) < 1e-8


def test_linearize_dynamics_helper_dispatches(gpu):
    """iLQR.linearize_dynamics (backward_pass.jl:25-40) with the family's dynamics callable:
    the dual-number kernel, one point and a trajectory, against oracle.jet."""
    from ilqr_amd.helpers import linearize_dynamics
    from ilqr_amd.floating import FloatingDynamics
    fj, _, _ = rbd_floating_arm(jet_ns())
    x, u = random_states(6, seed=31)
    f = FloatingDynamics(rbd_example_problem())
    A1, B1 = linearize_dynamics(x[0], u[0], f)
    AT, BT = linearize_dynamics(x, u[:5], f)          # N = T + 1 rows
    Aj, Bj = jet.jacobians(fj, x[:5], u[:5])
    assert rel(A1, Aj[0]) < 1e-10 and rel(B1, Bj[0]) < 1e-10
    assert rel(AT, Aj) < 1e-10 and rel(BT, Bj) < 1e-10


@pytest.mark.parametrize("name", ["2dof_arm", "coupled"])
def test_floating_device_conserves_world_linear_momentum(gpu, name):
    """Zero gravity, u = 0: the device RK4 keeps the world-frame linear momentum
    R(p)·(M v)[3:6] over 300 steps to RK4 accuracy, with M from the independent
    Jacobian formulation (tests/closures.py floating_mass_matrix_jacobians; the CPU pins
    are tests/test_floating_pins.py)."""
    from closures import coupled_floating_model, floating_linear_momentum_world
    model = None if name == "2dof_arm" else coupled_floating_model()
    p = rbd_example_problem() if model is None else _problem_of(model)
    x, _ = random_states(16, seed=21)
    s = FloatingSolver(p, 1, 1)
    try:
        xe = torch.from_numpy(x).cuda()
        z = torch.zeros(16, 8, dtype=torch.float64, device="cuda")
        for _ in range(300):
            xe = s.dynamics(xe, z)
        x1 = xe.cpu().numpy()
    finally:
        s.close()
    p0 = floating_linear_momentum_world(x, model)
    p1 = floating_linear_momentum_world(x1, model)
    assert np.abs(p0).max() > 1.0
    assert np.abs(p1 - p0).max() / np.abs(p0).max() < 1e-7, (p0, p1)


@pytest.mark.parametrize("nb,cand", [(1, 64), (9, 16), (70, 4)])
def test_floating_forward_rollout_equals_stepping_the_dynamics(gpu, nb, cand, monkeypatch):
    """The forward's trial-1 x̄ equals stepping the dynamics kernel (fb_step) under its ū,
    bit for bit — at 64, 16 and 4 lanes a trajectory (B = 1, 9, 70), i.e. for every split of
    the RK4 step over the forward's waves (ilqr_floating.hip is built with
    -ffp-contract=on: DESIGN.md §4 'Then four waves'); and a second call repeats its bits."""
    T = 60
    x, u = script_batch(nb, T, seed=nb)
    u = u + 0.3 * np.random.default_rng(nb).standard_normal(u.shape)
    fj, _, _ = rbd_floating_arm(jet_ns())
    for t in range(T):
        x[:, t + 1] = fj(x[:, t], u[:, t])
    tl = CF.derivative_tiles(x, u, fj, *rbd_cost_quads())
    from oracle import cref
    d, K, _ = cref.tiles_backward(tl, mu=0.01, symmetrize=True)
    monkeypatch.setenv("ILQR_FB_CAND", str(cand))
    s = FloatingSolver(rbd_example_problem(), T, nb)
    try:
        args = [torch.from_numpy(a).cuda() for a in (x, u, d, K)]
        pc = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
        xn, un, cost, trials, st = [v.clone() for v in s.forward(*args, pc)]
        xr = s.rollout(xn[:, 0], un)
        again = s.forward(*args, pc)
    finally:
        s.close()
    assert trials.tolist() == [1] * nb and torch.isfinite(xn).all()
    assert torch.equal(xr.view(torch.int64), xn.view(torch.int64))
    assert torch.equal(again[0].view(torch.int64), xn.view(torch.int64))
    assert torch.equal(again[2].view(torch.int64), cost.view(torch.int64))
