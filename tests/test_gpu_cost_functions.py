"""GPU parity tests of cost_functions.jl's factories on the RBD family (through the C ABI,
ilqr_chain_set_simple_costs).

Reference: src/cost_functions.jl:5-54 — simple_final_cost(mechanism, body, point,
final_target, weight) = weight·Σₖ (p_z − final_targetₖ)² for p = transform_to_root(state,
body) * point, and simple_immediate_cost = Σ uᵢ² — driven by src/backward_pass.jl /
src/forward_pass.jl on the fixed-base 2Dof_arm and the coupled 2-joint chain.
Oracle: oracle.cost_functions (the kinematics composed with oracle.rbd's joint model,
differentiated by the ForwardDiff restatement) through oracle.ilqr_oracle, frozen in
tests/golden/chaintask_*.npz (make_golden.py). RigidBodyDynamics.jl is absent: parity
against the executed reference is unpinned; the kinematics are pinned by the dynamics
(tests/test_cost_functions.py).

Tolerances (relative to the largest entry): fp64 gains 1e-8, forward 1e-10, fit 1e-8 —
the device evaluates the point's coordinates as the trigonometric polynomial sampled at
handle setup (rounding-level differences from composing the transforms) and the
terminal derivatives analytically instead of by nested duals; fp32 as the chain family's
fp32 tolerances (tests/test_gpu_chain.py).
"""
import os

import numpy as np
import pytest
import torch

from ilqr_amd import _lib
from ilqr_amd.chain import ChainDynamics, ChainSolver, coupled_2dof_problem, rbd_2dof_problem

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = ["chaintask_t60", "chaintask_c_nu1_t40", "chaintask_c_euc_t40"]


def rel(a, b):
    a = a.double().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a, float)
    b = b.double().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b, float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def dev(a, dtype):
    return torch.as_tensor(np.ascontiguousarray(a)).to("cuda", dtype).contiguous()


def load(name):
    import json
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    g = {k: z[k] for k in z.files}
    g["meta"] = json.loads(str(g["meta"]))
    return g


def problem(g):
    m = g["meta"]
    return (rbd_2dof_problem if m["robot"] == "2dof_arm" else coupled_2dof_problem)(m["nu"])


def solver(g, dtype, lin="dual", batch=None):
    nb, T = g["u"].shape[:2]
    s = ChainSolver(problem(g), T, batch or nb, dtype=dtype, linearization=lin)
    c = g["meta"]["simple"]
    s.set_simple_costs(c["body"], c["point"], c["final_target"], c["weight"], c["euclidean"])
    assert s.cost_mode == ("simple_euclidean" if c["euclidean"] else "simple")
    return s


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-8), (torch.float32, 5e-4)])
def test_simple_costs_backward(gpu, name, dtype, tol):
    """backward_pass with the task-space terminal quadratization (backward_pass.jl:134-153
    on cost_functions.jl:16-24) and ℓ = Σu² (its Hessian 2I, zero state rows)."""
    g = load(name)
    s = solver(g, dtype)
    d, K, st = s.backward(dev(g["x"], dtype), dev(g["u"], dtype))
    assert (st.cpu().numpy() == 0).all()
    assert rel(K, g["K"]) < tol and rel(d, g["d"]) < tol, (rel(K, g["K"]), rel(d, g["d"]))


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-10), (torch.float32, 5e-4)])
def test_simple_costs_forward(gpu, name, dtype, tol):
    """forward_pass from the oracle's gains: rollout, Σu² stage costs and the final cost
    weight·Σₖ(p_z − tₖ)² (or the squared distance) of the point at x̄_N."""
    g = load(name)
    s = solver(g, dtype)
    nb = g["u"].shape[0]
    pc = torch.full((nb,), float("inf"), dtype=dtype, device="cuda")
    xn, un, c, tr, st = s.forward(dev(g["x"], dtype), dev(g["u"], dtype), dev(g["d"], dtype),
                                  dev(g["K"], dtype), pc)
    assert (tr.cpu().numpy() == 1).all() and (st.cpu().numpy() == 0).all()
    assert rel(xn, g["fw_x"]) < tol and rel(un, g["fw_u"]) < tol and rel(c, g["fw_cost"]) < tol


@pytest.mark.parametrize("name", CASES)
def test_simple_costs_fit_f64(gpu, name):
    """fit: the oracle's iteration counts, statuses, iterates and final costs. At the fp64
    cost floor (chaintask_c_euc_t40's trajectory 1: iterations 4 and 5 cost the same to
    all 14 printed digits) whether the last trial counts as a decrease is decided by the
    last bit: the oracle converges there, the device may exhaust the line search instead —
    both return the iterate the failing or converging iteration started from (the x̄, ū
    checks below)."""
    g = load(name)
    s = solver(g, torch.float64)
    r = s.fit(dev(g["x"], torch.float64), dev(g["u"], torch.float64), max_iter=20, tol=1e-6)
    assert np.array_equal(r.iters.cpu().numpy(), g["fit_iters"])
    st, want = r.status.cpu().numpy(), g["fit_status"]
    tie = (want == _lib.TRAJ_CONVERGED) & (st == _lib.TRAJ_LS_EXHAUSTED)
    assert ((st == want) | tie).all(), (st, want)
    assert rel(r.x, g["fit_x"]) < 1e-8 and rel(r.u, g["fit_u"]) < 1e-8
    last = g["fit_cost"][np.arange(len(g["fit_iters"])), g["fit_iters"] - 1]
    assert rel(r.cost, last) < 1e-10


def test_simple_costs_fit_f32(gpu):
    """fp32 (config 5's precision): the fit reaches the oracle's optimum."""
    g = load("chaintask_c_nu1_t40")
    s = solver(g, torch.float32)
    r = s.fit(dev(g["x"], torch.float32), dev(g["u"], torch.float32), max_iter=20, tol=1e-6)
    assert set(r.status.cpu().numpy().tolist()) <= {_lib.TRAJ_CONVERGED, _lib.TRAJ_LS_EXHAUSTED}
    last = g["fit_cost"][np.arange(len(g["fit_iters"])), g["fit_iters"] - 1]
    assert rel(r.cost, last) < 1e-4


def test_simple_costs_wide_batch_equals_fixture(gpu):
    """BASELINE config 5's batch (2048, fp64): every replica of the fixture's trajectories
    fits to the oracle's iterate (batch-size independence of the cost mode, both launch
    shapes of the forward group and all 4-trajectory backward slots)."""
    g = load("chaintask_c_nu1_t40")
    nb = g["u"].shape[0]
    Bw = 2048
    idx = np.arange(Bw) % nb
    s = solver(g, torch.float64, batch=Bw)
    r = s.fit(dev(g["x"][idx], torch.float64), dev(g["u"][idx], torch.float64), max_iter=20, tol=1e-6)
    assert np.array_equal(r.iters.cpu().numpy(), g["fit_iters"][idx])
    assert rel(r.u, g["fit_u"][idx]) < 1e-8 and rel(r.x, g["fit_x"][idx]) < 1e-8


def test_simple_costs_api_mirror(gpu):
    """ilqr_amd.fit / backward_pass with ChainDynamics + simple_immediate_cost +
    simple_final_cost solve on the device in the handle's simple-cost mode."""
    import ilqr_amd
    g = load("chaintask_c_euc_t40")
    pr = problem(g)
    c = g["meta"]["simple"]
    a = (pr.chain, c["body"], c["point"], c["final_target"], c["weight"])
    lf = ilqr_amd.simple_final_cost(*a, euclidean=True)
    l = ilqr_amd.simple_immediate_cost(*a)
    dyn = ChainDynamics(pr)
    xo, uo = ilqr_amd.fit(g["x"][1], g["u"][1], dyn, l, lf, max_iter=20, tol=1e-6)
    assert rel(uo, g["fit_u"][1]) < 1e-8
    d, K = ilqr_amd.backward_pass(g["x"][0], g["u"][0], dyn, l, lf)
    assert rel(K, g["K"][0]) < 1e-8
    # the host evaluation of the callables agrees with the device's final cost
    xn, un, cost = ilqr_amd.forward_pass(g["x"][0], g["u"][0], None, g["d"][0], g["K"][0], np.inf,
                                         dyn, l, lf)
    host = sum(l(xn[t], un[t]) for t in range(un.shape[0])) + lf(xn[-1])
    assert abs(cost - host) <= 1e-10 * abs(host)


def test_simple_costs_mode_switching(gpu):
    """RNEA is refused while a simple cost is set; ILQR_CHAIN_COST_JOINT restores the
    problem's joint-space costs (the same gains as a fresh handle)."""
    g = load("chaintask_c_nu1_t40")
    s = solver(g, torch.float64)
    with pytest.raises(_lib.IlqrError):
        s.set_dynamics("rnea")
    s.set_joint_costs()
    assert s.cost_mode == "joint"
    x, u = dev(g["x"], torch.float64), dev(g["u"], torch.float64)
    d, K, _ = s.backward(x, u)
    f = ChainSolver(problem(g), g["u"].shape[1], g["u"].shape[0], dtype=torch.float64)
    d2, K2, _ = f.backward(x, u)
    assert torch.equal(K, K2) and torch.equal(d, d2)
    s.set_dynamics("rnea")   # allowed again
    with pytest.raises(_lib.IlqrError):
        s.set_simple_costs(1, [0, 0, 0], [0, 0, 0], 1.0)
