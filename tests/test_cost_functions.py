"""CPU tests of cost_functions.jl's factories: the oracle restatement (oracle/cost_functions.py),
the host mirror (ilqr_amd.cost_functions) and the C-ABI argument checks.

RigidBodyDynamics.jl's transform_to_root is absent, so the kinematics are pinned by
  * known answers on the 2Dof_arm (root-frame tip positions worked out by hand from
    test/urdf/2Dof_arm.urdf's joint origins and axes);
  * an independent formulation (oracle.rbd.world_frames: accumulated world rotations
    by the matrix exponential of each axis) on the 6-DoF arm and the coupled chain;
  * the dynamics restatement: the recursion's gravity torque equals −Σᵢ mᵢ ∂(g·p_cᵢ)/∂q
    of the COM positions (the potential's gradient), by the ForwardDiff restatement.
"""
import ctypes as C
import json
import math
import os

import numpy as np
import pytest

from ilqr_amd import _lib
from ilqr_amd import cost_functions as CF
from ilqr_amd.chain import coupled_2dof_problem, load_robot, rbd_2dof_problem
from oracle import cost_functions as OC
from oracle import dual
from oracle import ilqr_oracle as O
from oracle import rbd as RBD

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_known_answers_2dof_arm():
    """2Dof_arm: joint 1 about z at (0.5, 0.5, 0), joint 2 about y at (1, 0, 0) of link 1.
    The point (0, 0, 0.5) of link 2 sits at (1.5, 0.5, 0.5) at q = 0; q₂ = π/2 turns it
    onto link 2's x axis: (2.0, 0.5, 0.0); q₁ = π/2 swings link 2's origin to (0.5, 1.5, 0)."""
    ch = load_robot("2dof_arm")
    pt = [0.0, 0.0, 0.5]
    for q, want in [((0.0, 0.0), (1.5, 0.5, 0.5)), ((0.0, math.pi / 2), (2.0, 0.5, 0.0)),
                    ((math.pi / 2, 0.0), (0.5, 1.5, 0.5))]:
        assert np.allclose(OC.point_position(ch, 1, pt, list(q)), want, atol=1e-15)
        assert np.allclose(CF.point_position(ch, 1, pt, np.array(q)), want, atol=1e-15)
    # the fixed base (−1): the point itself; link 1 (body 0): one joint
    assert np.allclose(OC.point_position(ch, -1, pt, [0.3, 0.2]), pt)
    assert np.allclose(OC.point_position(ch, 0, [1.0, 0.0, 0.0], [math.pi / 2, 0.0]), (0.5, 1.5, 0.0))
    # the reference's reading at q = 0: weight · Σₖ (p_z − tₖ)² = 2·((0.5−0.3)² + 0 + (0.5−0.4)²)
    lf = OC.simple_final_cost(ch, 1, pt, [0.3, 0.5, 0.4], 2.0)
    assert lf(np.zeros(4)) == pytest.approx(0.1, rel=1e-14)
    # squared distance: 2·((1.5−0.3)² + 0 + (0.5−0.4)²)
    lfe = OC.simple_final_cost(ch, 1, pt, [0.3, 0.5, 0.4], 2.0, euclidean=True)
    assert lfe(np.zeros(4)) == pytest.approx(2.0 * (1.2 ** 2 + 0.1 ** 2), rel=1e-14)
    assert OC.simple_immediate_cost(ch, 1, pt, [0, 0, 0], 2.0)(np.zeros(4), [1.0, -2.0]) == 5.0


@pytest.mark.parametrize("robot", ["6dof_arm", "coupled"])
def test_kinematics_independent_formulation(robot):
    ch = coupled_2dof_problem(2).chain if robot == "coupled" else load_robot("6dof_arm")
    rng = np.random.default_rng(3)
    for _ in range(8):
        q = rng.uniform(-3, 3, ch.n)
        frames = RBD.world_frames(ch, q)
        for b in range(ch.n):
            pt = rng.uniform(-1, 1, 3)
            o, _, R = frames[b]
            want = o + R @ pt
            assert np.allclose(OC.point_position(ch, b, pt, list(q)), want, rtol=0, atol=1e-13)
            assert np.allclose(CF.point_position(ch, b, pt, q), want, rtol=0, atol=1e-13)


@pytest.mark.parametrize("robot", ["6dof_arm", "coupled"])
def test_kinematics_pinned_by_gravity_torque(robot):
    """τ_gravity(q) = ∂V/∂q with V = −Σᵢ mᵢ g·p_cᵢ(q): ties the point positions to the
    Newton-Euler restatement (itself pinned in tests/test_chain_oracle.py)."""
    if robot == "coupled":
        ch = coupled_2dof_problem(2).chain
    else:
        c6 = load_robot("6dof_arm")
        c6.gravity = np.array([0.3, -1.1, -9.81])
        ch = c6
    m = RBD.ChainModel(ch, 0.01)
    g = ch.gravity
    rng = np.random.default_rng(4)
    for _ in range(4):
        q = rng.uniform(-2, 2, ch.n)
        tau = m.rnea([np.array([v]) for v in q], None, [np.zeros(1)] * ch.n, gravity=True)

        def V(qq):
            acc = 0.0
            for i in range(ch.n):
                p = OC.point_position(ch, i, ch.com[i], qq)
                acc = acc - float(ch.mass[i]) * (g[0] * p[0] + g[1] * p[1] + g[2] * p[2])
            return acc
        dV = dual.gradient(V, q)
        assert np.allclose([t[0] for t in tau], dV, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("euclidean", [False, True])
def test_host_mirror_equals_oracle(euclidean):
    pr = coupled_2dof_problem(1)
    rng = np.random.default_rng(5)
    for _ in range(6):
        pt, tg, w = rng.uniform(-1, 1, 3), rng.uniform(-1, 1, 3), rng.uniform(0.1, 10)
        b = int(rng.integers(-1, 2))
        x = rng.uniform(-3, 3, 4)
        lf = CF.simple_final_cost(pr, b, pt, tg, w, euclidean=euclidean)
        lo = OC.simple_final_cost(pr.chain, b, pt, tg, w, euclidean=euclidean)
        assert lf(x) == pytest.approx(lo(x), rel=1e-13)
        u = rng.uniform(-2, 2, 1)
        assert CF.simple_immediate_cost(pr, b, pt, tg, w)(x, u) == OC.simple_immediate_cost(
            pr.chain, b, pt, tg, w)(x, u)
    # bodies by joint name; the reference's quirk: only p_z enters
    lf = CF.simple_final_cost("2dof_arm", "joint_2", [0, 0, 0.5], [9.0, 9.0, 0.0], 1.0)
    assert lf.body == 1 and lf(np.zeros(4)) == pytest.approx(2 * 8.5 ** 2 + 0.5 ** 2)   # p = (1.5, 0.5, 0.5)
    with pytest.raises(ValueError):
        CF.simple_final_cost("2dof_arm", 2, [0, 0, 0], [0, 0, 0], 1.0)
    with pytest.raises(AssertionError):   # @assert 3 == length(final_target) (:12, :41)
        CF.simple_immediate_cost("2dof_arm", 1, [0, 0, 0], [0, 0], 1.0)


def test_api_recognises_the_factories():
    from ilqr_amd.chain import ChainDynamics, chain_problem_of
    pr = coupled_2dof_problem(2)
    a = (pr.chain, 1, [0.1, 0, 0.2], [0.0, 0.0, 0.5], 3.0)
    l, lf = CF.simple_immediate_cost(*a), CF.simple_final_cost(*a)
    assert chain_problem_of(ChainDynamics(pr), l, lf) is pr
    assert CF.simple_costs_of(pr, l, lf) is lf
    other = rbd_2dof_problem(2).chain   # a different chain: not this problem's costs
    assert CF.simple_costs_of(pr, l, CF.simple_final_cost(other, 1, [0, 0, 0], [0, 0, 0], 1.0)) is None


@pytest.mark.parametrize("name", ["chaintask_t60", "chaintask_c_nu1_t40", "chaintask_c_euc_t40"])
def test_golden_fixtures_consistent(name):
    """Each fixture's first trajectory re-derived by the oracle: the backward gains (the
    fixture was generated by tests/golden/make_golden.py)."""
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    c = meta["simple"]
    pr = (rbd_2dof_problem if meta["robot"] == "2dof_arm" else coupled_2dof_problem)(meta["nu"])
    model = RBD.ChainModel(pr.chain, pr.dt)
    f, _, _ = RBD.chain_closures(model, RBD.ChainCost(pr.target, pr.q_weight, pr.r_weight, pr.qf_weight))
    a = (pr.chain, c["body"], c["point"], c["final_target"], c["weight"])
    l, lf = OC.simple_immediate_cost(*a), OC.simple_final_cost(*a, euclidean=c["euclidean"])
    d, K = O.backward_pass(z["x"][0], z["u"][0], f, l, lf)
    assert np.abs(K - z["K"][0]).max() <= 1e-12 * np.abs(z["K"][0]).max()
    assert np.abs(d - z["d"][0]).max() <= 1e-12 * max(np.abs(z["d"][0]).max(), 1e-300)
    # the terminal quadratization: ForwardDiff-restated vs central differences; the
    # velocity rows and columns are zero
    xN = z["x"][0, -1]
    _, gN, HN = O.final_cost_quadratization(xN, lf)
    h = 1e-5
    for i in range(2):
        e = np.zeros(4)
        e[i] = h
        assert gN[i] == pytest.approx((lf(xN + e) - lf(xN - e)) / (2 * h), rel=1e-6, abs=1e-6)
    assert np.allclose(HN[2:], 0) and np.allclose(HN[:, 2:], 0) and np.allclose(HN, HN.T)


def test_simple_costs_abi_validates_without_gpu():
    """Argument checks of ilqr_chain_set_simple_costs happen before any HIP call."""
    lib = _lib.load()
    pt = (C.c_double * 3)(0.0, 0.0, 0.5)
    assert lib.ilqr_chain_set_simple_costs(None, _lib.CHAIN_COST_SIMPLE, 1, pt, pt, 1.0) == _lib.ERR_BAD_ARG
    assert lib.ilqr_chain_get_cost_mode(None) == -1
