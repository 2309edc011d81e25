"""cost_functions.jl's factories for the RBD family (src/cost_functions.jl:5-54).

    simple_final_cost(mechanism, body, point, final_target, weight)     (:5-27)
        → final_cost(x) = weight · Σₖ (work_space_traj[end] − final_targetₖ)²
    simple_immediate_cost(mechanism, body, point, final_target, weight) (:34-54)
        → immediate_cost(x, u) = Σ uᵢ²

where work_space_traj = (transform_to_root(state, body) * point).v is the root-frame
position of a point fixed on `body` (:20). The reference takes its LAST coordinate
(`work_space_traj[end]`, p_z) and differences it against every component of
final_target (`.- transpose(final_target)`, :21): that reading is the default here, and
`euclidean=True` gives Σₖ (pₖ − final_targetₖ)², the squared distance the name
suggests. One repair, forced: the reference calls `set_configuration!(state, xₙ)` with
the whole state (:19; a BoundsError for the fixed base's nq = n_joints); the joint angles
xₙ[0:n_joints] are what it can mean. `weight`, unused by simple_immediate_cost, stays
unused, and both factories keep `@assert 3 == length(final_target)` (:12, :41).

The mechanism is a chain of this package (ilqr_amd.urdf.Chain, a ChainProblem or a
robot name for load_robot); `body` is the index of the link joint `body` moves (or that
joint's name; −1 = the fixed base). With ChainDynamics on a 2-joint chain both callables
are recognised by ilqr_amd.fit / backward_pass / forward_pass, which then solve on the
device with ilqr_chain_set_simple_costs (the task cost's coefficients are sampled once
per handle; no host evaluation inside the iteration). Called directly they evaluate on
the host (one state: the reference's closure semantics).
"""
from __future__ import annotations

import numpy as np

from .chain import ChainProblem, body_index, load_robot
from .urdf import Chain


def _chain_of(mechanism) -> Chain:
    if isinstance(mechanism, Chain):
        return mechanism
    if isinstance(mechanism, ChainProblem):
        return mechanism.chain
    if isinstance(mechanism, str):
        return load_robot(mechanism)
    raise TypeError("mechanism: an ilqr_amd.urdf.Chain, a ChainProblem or a robot name")


def _check_target(final_target):
    if np.asarray(final_target).size != 3:
        raise AssertionError("3 == length(final_target)")   # cost_functions.jl:12, :41


def point_position(chain: Chain, body: int, point, q) -> np.ndarray:
    """transform_to_root(state, body) * point at joint angles q (fp64, host): composes
    x_parent = p_i + R0_i·Rot(a_i, q_i)·x_child from `body` down to the base."""
    w = np.asarray(point, float).reshape(3).copy()
    for i in range(body, -1, -1):
        a = chain.axis[i]
        c, s = np.cos(q[i]), np.sin(q[i])
        r = c * w + s * np.cross(a, w) + (1.0 - c) * float(a @ w) * a
        w = chain.p[i] + chain.R0[i] @ r
    return w


class SimpleFinalCost:
    """final_cost(xₙ) of simple_final_cost (cost_functions.jl:16-24)."""

    def __init__(self, mechanism, body, point, final_target, weight, euclidean=False):
        _check_target(final_target)
        self.chain = _chain_of(mechanism)
        self.body = body_index(self.chain, body)
        self.point = np.asarray(point, float).reshape(3).copy()
        self.final_target = np.asarray(final_target, float).reshape(3).copy()
        self.weight = float(weight)
        self.euclidean = bool(euclidean)

    def __call__(self, x):
        p = point_position(self.chain, self.body, self.point, np.asarray(x, float)[: self.chain.n])
        e = (p if self.euclidean else np.full(3, p[2])) - self.final_target
        acc = 0.0
        for k in range(3):   # sum((z .- transpose(final_target)) .^ 2), in order (:9)
            acc += e[k] * e[k]
        return self.weight * acc


class SimpleImmediateCost:
    """immediate_cost(x, u) of simple_immediate_cost (cost_functions.jl:45-51): Σ uᵢ²."""

    def __init__(self, mechanism, body, point, final_target, weight):
        _check_target(final_target)
        self.chain = _chain_of(mechanism)
        self.body = body_index(self.chain, body)

    def __call__(self, x, u):
        acc = 0.0
        for v in np.asarray(u, float).reshape(-1):
            acc += v * v
        return acc


def simple_final_cost(mechanism, body, point, final_target, weight, *, euclidean=False):
    """iLQR.simple_final_cost (cost_functions.jl:5-27); euclidean=True is the
    squared-distance reading (not the reference's)."""
    return SimpleFinalCost(mechanism, body, point, final_target, weight, euclidean)


def simple_immediate_cost(mechanism, body, point, final_target, weight):
    """iLQR.simple_immediate_cost (cost_functions.jl:34-54)."""
    return SimpleImmediateCost(mechanism, body, point, final_target, weight)


def _same_chain(a: Chain, b: Chain) -> bool:
    return a is b or (a.n == b.n and all(np.array_equal(getattr(a, k), getattr(b, k))
                                         for k in ("R0", "p", "axis")))


def simple_costs_of(problem: ChainProblem, immediate_cost, final_cost):
    """The SimpleFinalCost to set on a ChainProblem's handle when the pair is
    cost_functions.jl's on the problem's chain, else None."""
    if (isinstance(immediate_cost, SimpleImmediateCost) and isinstance(final_cost, SimpleFinalCost)
            and _same_chain(final_cost.chain, problem.chain)
            and _same_chain(immediate_cost.chain, problem.chain)):
        return final_cost
    return None
