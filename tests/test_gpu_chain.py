"""GPU parity tests of the RBD family (ILQR_PROBLEM_CHAIN) through the C ABI.

Reference: test/RBD_2_link_example/RBD_helper_functions.jl (RK4 of
v̇ = M \\ (−dynamics_bias + u), weighted joint costs) on test/urdf/2Dof_arm.urdf with a
fixed base (BASELINE config 5), driven by src/backward_pass.jl / src/forward_pass.jl.
Oracle: oracle.rbd (recursive Newton-Euler + RK4, exact Jacobians by forward-mode
AD) through oracle.ilqr_oracle, frozen in tests/golden/chain2_*.npz and
chain6_dynamics.npz (make_golden.py). RigidBodyDynamics.jl itself cannot run here:
the oracle is pinned by known answers (tests/test_chain_oracle.py) — parity against
the executed reference is unpinned.

Tolerances, written per dtype and linearisation:
  fp64, dual numbers: rollout 1e-12, A/B 1e-11, gains 1e-9, forward 1e-10, fit 1e-8
    (the device uses FMA contraction and its own sincos: rounding-level differences);
  fp64, central differences: A/B 1e-7 (truncation O(h²) with h = ε^⅓·max(1,|z|)),
    gains 1e-6;
  fp32 (BASELINE config 5), dual: rollout 2e-5, A/B 5e-5, gains 5e-4, forward 5e-4;
  fp32, central differences: A/B 2e-2 (ε_f32^⅔ ≈ 2.4e-5 relative to the largest
    entry, but entries of size ~dt² carry absolute error ~1e-5·max), gains 5e-3.
"""
import os

import numpy as np
import pytest
import torch

from ilqr_amd import _lib
from ilqr_amd.chain import (ChainSolver as _ChainSolver, chain_closures, load_robot, rbd_2dof_problem,
                            ChainProblem)

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")

# Every test of this module runs with both dynamics evaluators of 2-joint chains: the
# closed form (the default, ilqr_chain_set_dynamics AUTO) and the recursive
# Newton-Euler that restates RigidBodyDynamics.jl's calls, against the same oracle and
# tolerances.
_MODE = ["closed_form"]


@pytest.fixture(params=["closed_form", "rnea"], autouse=True)
def dyn_mode(request):
    _MODE[0] = request.param
    yield request.param


def ChainSolver(pr, *a, **k):  # noqa: N802 — shadows the import for this module's handles
    s = _ChainSolver(pr, *a, **k)
    if pr.n_joints == 2:
        s.set_dynamics(_MODE[0])
        assert s.dynamics_mode == _MODE[0]
    return s


def rel(a, b):
    a = a.double().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a, float)
    b = b.double().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b, float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def dev(a, dtype):
    return torch.as_tensor(np.ascontiguousarray(a)).to("cuda", dtype).contiguous()


def load(name):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def g2():
    return load("chain2_t100")


@pytest.fixture(scope="module")
def g1():
    return load("chain2_nu1_t50")


TOL = {  # (dtype, linearisation) → tolerances
    (torch.float64, "dual"): dict(roll=1e-12, AB=1e-11, gain=1e-9, fw=1e-10),
    (torch.float64, "fd"): dict(roll=1e-12, AB=1e-7, gain=1e-6, fw=1e-6),
    (torch.float32, "dual"): dict(roll=2e-5, AB=5e-5, gain=5e-4, fw=5e-4),
    (torch.float32, "fd"): dict(roll=2e-5, AB=2e-2, gain=5e-3, fw=5e-3),
}
CASES = list(TOL)


def solver(g, dtype, lin, nu=2):
    nb, T = g["u"].shape[:2]
    return ChainSolver(rbd_2dof_problem(nu), T, nb, dtype=dtype, linearization=lin)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_chain_rollout(gpu, g2, dtype):
    """dynamicsf (RNEA + RK4 functor) rollout from x₀ with u = 0."""
    s = solver(g2, dtype, "dual")
    x = s.rollout(dev(g2["x"][:, 0], dtype), dev(g2["u"], dtype))
    assert rel(x, g2["x"]) < TOL[(dtype, "dual")]["roll"]


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_chain6_dynamics(gpu, dtype):
    """One RK4 step of the coupled 6-DoF arm (test/urdf/6Dof_arm.urdf) vs the oracle."""
    g = load("chain6_dynamics")
    pr = ChainProblem(load_robot("6dof_arm"), 6, 0.01)
    s = ChainSolver(pr, 1, 1, dtype=dtype)
    xn = s.dynamics(dev(g["x"], dtype), dev(g["u"], dtype))
    assert rel(xn, g["x_next"]) < (1e-12 if dtype == torch.float64 else 5e-5)
    # the state moved: a wrong M or bias would show in the velocity rows
    assert rel(xn[:, 6:], g["x_next"][:, 6:]) < (1e-12 if dtype == torch.float64 else 5e-5)


@pytest.mark.parametrize("nu", [1, 2])
@pytest.mark.parametrize("dtype,lin,tol", [(torch.float64, "dual", 1e-11), (torch.float64, "fd", 1e-7),
                                           (torch.float32, "dual", 5e-5), (torch.float32, "fd", 2e-2)])
def test_chain_linearize_ragged(gpu, dtype, lin, tol, nu):
    """linearize_dynamics (backward_pass.jl:25-40), one lane per (b, t, direction), on a
    ragged batch (37 × 5 points × 5 or 6 directions: partial last workgroup, records
    straddling waves) at random states vs the oracle's exact forward-mode Jacobians."""
    from oracle import rbd
    pr = rbd_2dof_problem(nu)
    nb, T = 37, 5
    rng = np.random.default_rng(11 + nu)
    x = np.concatenate([rng.uniform(-2, 2, (nb, T + 1, 2)), rng.uniform(-1, 1, (nb, T + 1, 2))], axis=2)
    u = rng.uniform(-3, 3, (nb, T, nu))
    Ar, Br = rbd.ChainModel(pr.chain, pr.dt).linearize(x[:, :T].reshape(-1, 4), u.reshape(-1, nu))
    s = ChainSolver(pr, T, nb, dtype=dtype, linearization=lin)
    A, B = s.linearize(dev(x, dtype), dev(u, dtype))
    ea, eb = rel(A.reshape(-1, 4, 4), Ar), rel(B.reshape(-1, 4, nu), Br)
    assert ea < tol and eb < tol, (ea, eb)


@pytest.mark.parametrize("dtype,lin", CASES)
def test_chain_linearize(gpu, g2, dtype, lin):
    """linearize_dynamics (backward_pass.jl:25-40) at every (b, t)."""
    s = solver(g2, dtype, lin)
    A, B = s.linearize(dev(g2["x"], dtype), dev(g2["u"], dtype))
    t = TOL[(dtype, lin)]["AB"]
    assert rel(A, g2["A"]) < t and rel(B, g2["B"]) < t, (rel(A, g2["A"]), rel(B, g2["B"]))


@pytest.mark.parametrize("dtype,lin", CASES)
def test_chain_backward(gpu, g2, dtype, lin):
    """backward_pass (backward_pass.jl:324-357) gains vs the oracle."""
    s = solver(g2, dtype, lin)
    d, K, st = s.backward(dev(g2["x"], dtype), dev(g2["u"], dtype))
    assert (st.cpu().numpy() == 0).all()
    t = TOL[(dtype, lin)]["gain"]
    assert rel(K, g2["K"]) < t and rel(d, g2["d"]) < t, (rel(K, g2["K"]), rel(d, g2["d"]))


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_chain_forward(gpu, g2, dtype):
    """forward_pass (forward_pass.jl:55-93) from the oracle's gains, prev_cost = Inf."""
    s = solver(g2, dtype, "dual")
    nb = g2["u"].shape[0]
    pc = torch.full((nb,), float("inf"), dtype=dtype, device="cuda")
    xn, un, c, tr, st = s.forward(dev(g2["x"], dtype), dev(g2["u"], dtype), dev(g2["d"], dtype),
                                  dev(g2["K"], dtype), pc)
    t = TOL[(dtype, "dual")]["fw"]
    assert (tr.cpu().numpy() == 1).all() and (st.cpu().numpy() == 0).all()
    assert rel(xn, g2["fw_x"]) < t and rel(un, g2["fw_u"]) < t and rel(c, g2["fw_cost"]) < t


def test_chain_fit_f64(gpu, g2):
    """fit (forward_pass.jl:148-179): same iteration counts, iterates and costs."""
    s = solver(g2, torch.float64, "dual")
    r = s.fit(dev(g2["x"], torch.float64), dev(g2["u"], torch.float64), max_iter=20, tol=1e-6)
    assert np.array_equal(r.iters.cpu().numpy(), g2["fit_iters"])
    assert (r.status.cpu().numpy() == g2["fit_status"]).all()
    assert rel(r.x, g2["fit_x"]) < 1e-8 and rel(r.u, g2["fit_u"]) < 1e-8
    last = g2["fit_cost"][np.arange(len(g2["fit_iters"])), g2["fit_iters"] - 1]
    assert rel(r.cost, last) < 1e-10


@pytest.mark.parametrize("lin", ["dual", "fd"])
def test_chain_fit_f32(gpu, g2, lin):
    """BASELINE config 5 precision (fp32): the fit reaches the oracle's optimum."""
    s = solver(g2, torch.float32, lin)
    r = s.fit(dev(g2["x"], torch.float32), dev(g2["u"], torch.float32), max_iter=20, tol=1e-6)
    st = r.status.cpu().numpy()
    assert set(st.tolist()) <= {_lib.TRAJ_CONVERGED, _lib.TRAJ_LS_EXHAUSTED}, st
    last = g2["fit_cost"][np.arange(len(g2["fit_iters"])), g2["fit_iters"] - 1]
    assert rel(r.cost, last) < 1e-4
    assert rel(r.u, g2["fit_u"]) < 2e-3


def test_chain_nu1(gpu, g1):
    """nu = 1 (joint 1 driven only): gains, forward pass and the fit iterate (fp64).
    The oracle's trajectory 0 reaches a stationary point where the reference's line
    search would loop forever; either stop (converged / exhausted) returns the same
    iterate."""
    s = solver(g1, torch.float64, "dual", nu=1)
    x, u = dev(g1["x"], torch.float64), dev(g1["u"], torch.float64)
    d, K, _ = s.backward(x, u)
    assert rel(K, g1["K"]) < 1e-9 and rel(d, g1["d"]) < 1e-9
    nb = u.shape[0]
    pc = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
    xn, un, c, _, _ = s.forward(x, u, dev(g1["d"], torch.float64), dev(g1["K"], torch.float64), pc)
    assert rel(xn, g1["fw_x"]) < 1e-10 and rel(c, g1["fw_cost"]) < 1e-10
    r = s.fit(x, u, max_iter=20, tol=1e-6)
    assert set(r.status.cpu().numpy().tolist()) <= {_lib.TRAJ_CONVERGED, _lib.TRAJ_LS_EXHAUSTED}
    assert rel(r.x, g1["fit_x"]) < 1e-8 and rel(r.u, g1["fit_u"]) < 1e-8


def test_chain_api_mirror_keeps_eltype(gpu, g2):
    """ilqr_amd.fit with the chain closures: Float32 inputs solve in fp32 (the reference
    is generic in the element type), Float64 in fp64."""
    import ilqr_amd
    dyn, cost, fcost = chain_closures(rbd_2dof_problem(2))
    x32 = g2["x"][0].astype(np.float32)
    u32 = g2["u"][0].astype(np.float32)
    xo, uo = ilqr_amd.fit(x32, u32, dyn, cost, fcost, max_iter=20, tol=1e-6)
    assert uo.dtype == np.float32 and rel(uo, g2["fit_u"][0]) < 2e-3
    xo, uo = ilqr_amd.fit(g2["x"][0], g2["u"][0], dyn, cost, fcost, max_iter=20, tol=1e-6)
    assert uo.dtype == np.float64 and rel(uo, g2["fit_u"][0]) < 1e-8
    d, K = ilqr_amd.backward_pass(g2["x"][0], g2["u"][0], dyn, cost, fcost)
    assert rel(K, g2["K"][0]) < 1e-9


# -- a coupled chain: dense q-dependent M, Coriolis and gravity in the bias ----------------
# The 2Dof_arm's fixed-base M is the constant diag(4, 0.5) with zero bias, so the tests
# above cannot see a wrong joint angle, permutation sign or rotation in the 16-lane
# Newton-Euler forward (per-lane sin/cos + DPP quad broadcasts, row_newbcast b/M
# gathers), nor in the central differences' joint rotations. These run the same kernels on
# ilqr_amd.chain.coupled_2dof_problem against the oracle (tests/golden/chain2c_*.npz).
@pytest.fixture(scope="module")
def gc():
    return load("chain2c_t40")


@pytest.fixture(scope="module")
def gc1():
    return load("chain2c_nu1_t40")


def coupled_solver(g, dtype, lin, nu=2):
    from ilqr_amd.chain import coupled_2dof_problem
    nb, T = g["u"].shape[:2]
    return ChainSolver(coupled_2dof_problem(nu), T, nb, dtype=dtype, linearization=lin)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_coupled_chain_dynamics_kernel(gpu, dtype):
    """chain_dynamics_kernel (one lane per point) at random states vs the oracle."""
    from ilqr_amd.chain import coupled_2dof_problem
    from oracle import rbd
    pr = coupled_2dof_problem(2)
    rng = np.random.default_rng(3)
    n = 97
    x = np.concatenate([rng.uniform(-2.5, 2.5, (n, 2)), rng.uniform(-2, 2, (n, 2))], axis=1)
    u = rng.uniform(-20, 20, (n, 2))
    ref = rbd.ChainModel(pr.chain, pr.dt).step(x, u)
    s = ChainSolver(pr, 1, 1, dtype=dtype)
    xn = s.dynamics(dev(x, dtype), dev(u, dtype))
    assert rel(xn, ref) < (1e-12 if dtype == torch.float64 else 5e-5)
    assert rel(xn[:, 2:], ref[:, 2:]) < (1e-12 if dtype == torch.float64 else 1e-4)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_coupled_chain_forward_rollout(gpu, gc, dtype):
    """The 16-lane component-parallel forward kernel (chain_forward_lane): with δu = K = 0
    and prev_cost = Inf it is the rollout the fixture starts from; with the oracle's
    gains it is forward_pass (forward_pass.jl:55-93)."""
    s = coupled_solver(gc, dtype, "dual")
    nb, T = gc["u"].shape[:2]
    x, u = dev(gc["x"], dtype), dev(gc["u"], dtype)
    pc = torch.full((nb,), float("inf"), dtype=dtype, device="cuda")
    z_d, z_K = torch.zeros((nb, T, 2), dtype=dtype, device="cuda"), torch.zeros((nb, T, 2, 4), dtype=dtype, device="cuda")
    xr, _, _, _, _ = s.forward(x, u, z_d, z_K, pc)
    t = TOL[(dtype, "dual")]
    assert rel(xr, gc["x"]) < (1e-11 if dtype == torch.float64 else 1e-4)
    assert rel(xr[..., 2:], gc["x"][..., 2:]) < (1e-10 if dtype == torch.float64 else 2e-4)
    xn, un, c, tr, st = s.forward(x, u, dev(gc["d"], dtype), dev(gc["K"], dtype), pc)
    assert (st.cpu().numpy() == 0).all() and (tr.cpu().numpy() == 1).all()
    assert rel(xn, gc["fw_x"]) < t["fw"] * 10 and rel(un, gc["fw_u"]) < t["fw"] * 10
    assert rel(c, gc["fw_cost"]) < t["fw"] * 10


@pytest.mark.parametrize("dtype,lin", CASES)
def test_coupled_chain_linearize(gpu, gc, dtype, lin):
    """linearize_dynamics at every (b, t) of the coupled chain: dual numbers and the
    central differences (fp32: the ± pair packed, stages 2-4 by shifted sin/cos), fp64
    and fp32."""
    s = coupled_solver(gc, dtype, lin)
    A, B = s.linearize(dev(gc["x"], dtype), dev(gc["u"], dtype))
    t = TOL[(dtype, lin)]["AB"]
    assert rel(A, gc["A"]) < t and rel(B, gc["B"]) < t, (rel(A, gc["A"]), rel(B, gc["B"]))
    # the coupling block ∂q̈/∂q alone, relative to its own size
    ta = 1e-9 if dtype == torch.float64 and lin == "dual" else (1e-5 if dtype == torch.float64 else 5e-2)
    assert rel(A[..., 2:, :2], gc["A"][..., 2:, :2]) < ta


def test_coupled_chain_fd_large_steps(gpu):
    """fp32 central differences where the RK4 stages' angle shifts leave |h| ≤ 1/8
    (fast velocities: chain_trig_rk4_pm flags the pair and re-evaluates it on the general
    step) mixed lane by lane with ordinary states, against the fp64 dual-number Jacobian
    of the same states."""
    from ilqr_amd.chain import coupled_2dof_problem
    pr = coupled_2dof_problem(2)
    nb, T = 64, 8
    rng = np.random.default_rng(11)
    x = np.concatenate([rng.uniform(-3, 3, (nb, T + 1, 2)), rng.uniform(-2, 2, (nb, T + 1, 2))], axis=2)
    fast = rng.random((nb, T + 1)) < 0.5
    x[..., 2:] += np.where(fast, 1.0, 0.0)[..., None] * rng.choice([-1, 1], (nb, T + 1, 2)) * (40.0 / (pr.dt / 0.01))
    u = rng.uniform(-5, 5, (nb, T, 2))
    A64, B64 = ChainSolver(pr, T, nb, dtype=torch.float64, linearization="dual").linearize(
        dev(x, torch.float64), dev(u, torch.float64))
    A32, B32 = ChainSolver(pr, T, nb, dtype=torch.float32, linearization="fd").linearize(
        dev(x, torch.float32), dev(u, torch.float32))
    assert torch.isfinite(A32).all() and torch.isfinite(B32).all()
    # A at the fp32 central-difference tolerance; B's small entries carry the fp32 rounding
    # of f at |q̇| ≈ 40 rad/s over 2h: 2.8e-2 on the recursion's general step, 2.7e-2 on the
    # closed form's general step, 3.6e-2 with its shifted stages (measured): 1e-1
    assert rel(A32, A64) < TOL[(torch.float32, "fd")]["AB"], rel(A32, A64)
    assert rel(B32, B64) < 1e-1, rel(B32, B64)


@pytest.mark.parametrize("dtype,lin", CASES)
def test_coupled_chain_backward(gpu, gc, dtype, lin):
    s = coupled_solver(gc, dtype, lin)
    d, K, st = s.backward(dev(gc["x"], dtype), dev(gc["u"], dtype))
    assert (st.cpu().numpy() == 0).all()
    # fp32 central differences on the coupled robot: A/B err ~1e-3 (gravity and Coriolis
    # terms are O(1), differenced in fp32), amplified to ~1e-2 in the gains
    t = TOL[(dtype, lin)]["gain"] if (dtype, lin) != (torch.float32, "fd") else 2e-2
    assert rel(K, gc["K"]) < t and rel(d, gc["d"]) < t, (rel(K, gc["K"]), rel(d, gc["d"]))


def test_coupled_chain_fit_f64(gpu, gc):
    s = coupled_solver(gc, torch.float64, "dual")
    r = s.fit(dev(gc["x"], torch.float64), dev(gc["u"], torch.float64), max_iter=20, tol=1e-6)
    assert np.array_equal(r.iters.cpu().numpy(), gc["fit_iters"])
    assert (r.status.cpu().numpy() == gc["fit_status"]).all()
    assert rel(r.x, gc["fit_x"]) < 1e-8 and rel(r.u, gc["fit_u"]) < 1e-8


@pytest.mark.parametrize("dtype,lin", [(torch.float64, "dual"), (torch.float32, "fd")])
def test_coupled_chain_nu1(gpu, gc1, dtype, lin):
    """nu = 1 (τ = [u₁, 0]) on the coupled chain: gains and forward pass."""
    s = coupled_solver(gc1, dtype, lin, nu=1)
    x, u = dev(gc1["x"], dtype), dev(gc1["u"], dtype)
    d, K, _ = s.backward(x, u)
    t = dict(TOL[(dtype, lin)])
    if (dtype, lin) == (torch.float32, "fd"):
        t["gain"] = 2e-2  # as in test_coupled_chain_backward
    assert rel(K, gc1["K"]) < t["gain"] and rel(d, gc1["d"]) < t["gain"]
    nb = u.shape[0]
    pc = torch.full((nb,), float("inf"), dtype=dtype, device="cuda")
    xn, un, c, _, _ = s.forward(x, u, dev(gc1["d"], dtype), dev(gc1["K"], dtype), pc)
    assert rel(xn, gc1["fw_x"]) < t["fw"] * 10 and rel(c, gc1["fw_cost"]) < t["fw"] * 10


# -- BASELINE config 5 as stated: nu = 1, fp32, central differences, T = 100 ---------------
@pytest.fixture(scope="module")
def g5():
    return load("chain2_nu1_t100")


def test_config5_nu1_fp32_fd_fixture(gpu, g5):
    """Gains, forward pass and fit of the nu = 1, T = 100 fixture in the config-5
    arithmetic (fp32, central-difference linearisation on the device)."""
    s = solver(g5, torch.float32, "fd", nu=1)
    x, u = dev(g5["x"], torch.float32), dev(g5["u"], torch.float32)
    A, B = s.linearize(x, u)
    t = TOL[(torch.float32, "fd")]
    assert rel(A, g5["A"]) < t["AB"] and rel(B, g5["B"]) < t["AB"]
    d, K, st = s.backward(x, u)
    assert (st.cpu().numpy() == 0).all()
    assert rel(K, g5["K"]) < t["gain"] and rel(d, g5["d"]) < t["gain"], (rel(K, g5["K"]), rel(d, g5["d"]))
    nb = u.shape[0]
    pc = torch.full((nb,), float("inf"), dtype=torch.float32, device="cuda")
    xn, un, c, _, _ = s.forward(x, u, dev(g5["d"], torch.float32), dev(g5["K"], torch.float32), pc)
    assert rel(xn, g5["fw_x"]) < t["fw"] and rel(c, g5["fw_cost"]) < t["fw"]
    r = s.fit(x, u, max_iter=20, tol=1e-6)
    assert set(r.status.cpu().numpy().tolist()) <= {_lib.TRAJ_CONVERGED, _lib.TRAJ_LS_EXHAUSTED}
    last = g5["fit_cost"][np.arange(nb), g5["fit_iters"] - 1]
    assert rel(r.cost, last) < 1e-4 and rel(r.u, g5["fit_u"]) < 2e-3


def test_config5_batch2048_iteration_vs_c_oracle(gpu):
    """The config-5 bench step (tools/bench_rbd.py --nu 1: B = 2048, T = 100, fp32,
    central differences, one fit iteration from cold) against the C restatement
    (oracle_chain_iterate: fp64, central differences) on 64 sampled trajectories."""
    from ilqr_amd.chain import rbd_initial_states
    from oracle import cref
    pr = rbd_2dof_problem(1)
    B, T = 2048, 100
    x0 = rbd_initial_states(B, 2)
    s = ChainSolver(pr, T, B, dtype=torch.float32, linearization="fd")
    u = torch.zeros((B, T, 1), dtype=torch.float32, device="cuda")
    x = s.rollout(torch.from_numpy(x0).to("cuda", torch.float32), u)
    xn, un = torch.empty_like(x), torch.empty_like(u)
    pc = torch.empty((B,), dtype=torch.float32, device="cuda")
    st = torch.zeros((B,), dtype=torch.int32, device="cuda")
    tr = torch.empty((B,), dtype=torch.int32, device="cuda")
    s.iterate(x, u, xn, un, None, st, pc, trials=tr, options=_lib.default_options(tol=-1.0))
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all() and (tr.cpu().numpy() == 1).all()
    idx = np.arange(0, B, 32)
    d, K, xo, uo, co, tro = cref.chain_iterate(pr, x[idx].double().cpu().numpy(),
                                               u[idx].double().cpu().numpy())
    t = TOL[(torch.float32, "fd")]
    assert (tro == 1).all()
    assert rel(un.cpu().numpy()[idx], uo) < t["fw"] and rel(xn.cpu().numpy()[idx], xo) < t["fw"]
    assert rel(pc.cpu().numpy()[idx], co) < t["fw"]


@pytest.mark.parametrize("name", ["rbd", "coupled"])
@pytest.mark.parametrize("nu", [1, 2])
def test_closed_form_equals_recursion(gpu, name, nu):
    """The closed form (trigonometric M(q₂), bilinear g, Christoffel velocity term, its
    coefficients sampled from the recursion at creation) against the recursion at
    random states, fp64, one RK4 step and the creation check's own figure."""
    from ilqr_amd.chain import coupled_2dof_problem
    pr = rbd_2dof_problem(nu) if name == "rbd" else coupled_2dof_problem(nu)
    n = 512
    s = _ChainSolver(pr, 1, n, dtype=torch.float64)
    assert s.closed_form_error < 1e-12, s.closed_form_error
    rng = np.random.default_rng(11)
    x = torch.from_numpy(np.concatenate([rng.uniform(-4, 4, (n, 2)), rng.uniform(-6, 6, (n, 2))], 1)).cuda()
    u = torch.from_numpy(rng.uniform(-3, 3, (n, nu))).cuda()
    s.set_dynamics("closed_form")
    a = s.dynamics(x, u)
    s.set_dynamics("rnea")
    b = s.dynamics(x, u)
    assert rel(a, b) < 1e-13
    assert s.dynamics_mode == "rnea"
    s.set_dynamics("auto")
    assert s.dynamics_mode == "closed_form"


def chain_fit_replay(s, x0, u0, max_iter, tol, max_trials, x_traj=None):
    """fit (forward_pass.jl:148-179) restated as ilqr_chain_iterate calls: prev_cost = Inf,
    each iteration on the still-running trajectories, a trajectory that stops keeps the
    iteration's INPUT (converged: the pre-update iterate, :171; NaN / exhausted search:
    the last accepted one), the running ones the last accepted iterate and MAX_ITER."""
    nb = x0.shape[0]
    dt = x0.dtype
    s._bind()
    o = _lib.default_options(max_iter=max_iter, tol=tol, max_trials=max_trials)
    x, u = x0.clone(), u0.clone()
    pc = torch.full((nb,), float("inf"), dtype=dt, device="cuda")
    st = torch.zeros((nb,), dtype=torch.int32, device="cuda")
    tr = torch.zeros((nb,), dtype=torch.int32, device="cuda")
    it_out = torch.zeros((nb,), dtype=torch.int32, device="cuda")
    rx, ru = x0.clone(), u0.clone()
    for it in range(1, max_iter + 1):
        run = st == 0
        if not bool(run.any()):
            break
        xn, un = torch.empty_like(x), torch.empty_like(u)
        tr.fill_(-1)
        s.iterate(x, u, xn, un, pc, st, pc, trials=tr, x_traj=x_traj, options=o)
        it_out[run & (tr != -1)] = it   # the forward ran it (a NaN backward stops before)
        stopped = run & (st != 0)
        rx[stopped], ru[stopped] = x[stopped], u[stopped]
        keep = run & (st == 0)
        x = torch.where(keep[:, None, None], xn, x)
        u = torch.where(keep[:, None, None], un, u)
    run = st == 0
    rx[run], ru[run] = x[run], u[run]
    st = torch.where(run, torch.full_like(st, _lib.TRAJ_MAX_ITER), st)
    s_np = st.cpu().numpy()
    cs = _lib.ERR_NAN if (s_np == _lib.TRAJ_NAN).any() else (
        _lib.ERR_LS_EXHAUSTED if (s_np == _lib.TRAJ_LS_EXHAUSTED).any() else _lib.OK)
    return rx, ru, pc, it_out, st, cs


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("max_iter,tol,max_trials,nan,inplace", [
    (20, 1e-6, None, True, False),     # early convergence: the poll stops the loop
    (6, -1.0, 2, True, False),         # exhausted searches and a NaN, to max_iter
    (5, 1e-6, None, False, True),      # x_out = x_init: no direct output, copies
    (4, -1.0, None, False, "xtraj"),   # x_out = x_traj (a tracking target): read by every
                                       # iteration, written only by the gather
    (1, -1.0, None, False, False),
    (0, -1.0, None, False, False),     # the input is the result
])
def test_chain_fit_equals_iterate_replay(gpu, g2, dtype, max_iter, tol, max_trials, nan, inplace):
    """The chain fit driver (one init launch, iteration 1 on the caller's x_init in place,
    the last iteration into x_out, the running-count poll, one gather + the published
    call status) returns exactly what the same iterations through ilqr_chain_iterate do:
    x, u, cost, iterations, status and call status, bit for bit."""
    import ctypes as C
    s = solver(g2, dtype, "fd" if dtype == torch.float32 else "dual")
    x0, u0 = dev(g2["x"], dtype), dev(g2["u"], dtype)
    if nan:
        x0[1, 3, 2] = float("nan")
    xt0 = None
    if inplace == "xtraj":
        xt0 = x0.flip(1).contiguous()  # some other trajectory of states as the target
    ref = chain_fit_replay(s, x0, u0, max_iter, tol, max_trials, x_traj=xt0)
    for _ in range(2):   # twice: the re-armed call-status words
        xi, ui = x0.clone(), u0.clone()
        if inplace == "xtraj":
            nb = xi.shape[0]
            xt = xt0.clone()
            uo = torch.empty_like(ui)
            cost = torch.empty((nb,), dtype=dtype, device="cuda")
            it = torch.empty((nb,), dtype=torch.int32, device="cuda")
            st = torch.empty((nb,), dtype=torch.int32, device="cuda")
            s._bind()
            o = _lib.default_options(max_iter=max_iter, tol=tol, max_trials=max_trials)
            p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
            cs = s.lib.ilqr_chain_fit(s.h, C.byref(o), p(xi), p(ui), p(xt), p(xt), p(uo), p(cost), p(it), p(st))
            got = (xt, uo, cost, it, st, cs)
        elif inplace:
            nb = xi.shape[0]
            cost = torch.empty((nb,), dtype=dtype, device="cuda")
            it = torch.empty((nb,), dtype=torch.int32, device="cuda")
            st = torch.empty((nb,), dtype=torch.int32, device="cuda")
            s._bind()
            o = _lib.default_options(max_iter=max_iter, tol=tol, max_trials=max_trials)
            p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
            cs = s.lib.ilqr_chain_fit(s.h, C.byref(o), p(xi), p(ui), None, p(xi), p(ui), p(cost), p(it), p(st))
            got = (xi, ui, cost, it, st, cs)
        else:
            r = s.fit(xi, ui, max_iter=max_iter, tol=tol,
                      options=_lib.default_options(max_iter=max_iter, tol=tol, max_trials=max_trials))
            got = (r.x, r.u, r.cost, r.iters, r.status, r.call_status)
        assert got[5] == ref[5]
        for a, b in zip(got[:4], ref[:4]):
            torch.testing.assert_close(a, b, rtol=0, atol=0, equal_nan=True)
        assert torch.equal(got[4], ref[4])
    if nan and max_iter > 0:
        assert ref[4][1].item() == _lib.TRAJ_NAN
