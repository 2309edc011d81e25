"""CPU restatement of src/cost_functions.jl — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
anything under oracle/.

The reference's factories (src/cost_functions.jl:5-54):

    simple_final_cost(mechanism, body, point, final_target, weight)
        @assert 3 == length(final_target)                                   (:12)
        state = MechanismState(mechanism)                                   (:14)
        final_cost(xₙ):                                                     (:16-24)
            set_configuration!(state, xₙ)                                   (:19)
            work_space_traj .= (transform_to_root(state, body) * point).v  (:20)
            final_dist = sum((work_space_traj[end] .- transpose(final_target)) .^ 2)  (:21)
            return weight * final_dist                                      (:23)
    simple_immediate_cost(...) → immediate_cost(x, u) = sum(u .^ 2)         (:45-51)

transform_to_root is RigidBodyDynamics.jl's (not vendored, absent here; pinned in
docs/Manifest.toml): the composition of the joint transforms from `body` to the root,
restated with this oracle's own joint model (oracle.rbd: x_parent = p_i + R0_i·
Rot(a_i, q_i)·x_child, the same joint frames the dynamics restatement uses). The
configuration is the joint angles xₙ[0:n] — the reference hands set_configuration! the
whole state, which throws for the fixed base (nq = n < nx): the one meaning it can
have. The closures are generic in the element type (floats or oracle.dual duals), so
the oracle's backward pass differentiates them the way ForwardDiff does.

Parity is unpinned against the executed reference (Julia and RigidBodyDynamics.jl are
absent); the kinematics are pinned by the dynamics restatement instead: the gravity
torque of oracle.rbd's recursion equals −Σᵢ mᵢ ∂(g·p_cᵢ)/∂q of this module's COM
positions (tests/test_chain_oracle.py).
"""
from __future__ import annotations

from . import dual as D
from .rbd import _add, _fl, _matvec, _rod


def point_position(chain, body, point, q):
    """(transform_to_root(state, body) * point).v with configuration q (generic scalars)."""
    R0, p, ax = _fl(chain.R0), _fl(chain.p), _fl(chain.axis)
    w = [float(v) for v in point]
    for i in range(body, -1, -1):
        w = _add(p[i], _matvec(R0[i], _rod(ax[i], D.cos(q[i]), D.sin(q[i]), w)))
    return w


def simple_final_cost(chain, body, point, final_target, weight, euclidean=False):
    """cost_functions.jl:5-27 (euclidean=True: Σₖ (pₖ − tₖ)², not the reference's)."""
    n = chain.n
    tgt = [float(v) for v in final_target]

    def final_cost(x):
        ws = point_position(chain, body, point, [x[i] for i in range(n)])
        acc = 0.0
        for k in range(3):
            e = (ws[k] if euclidean else ws[2]) - tgt[k]   # work_space_traj[end] .- tᵀ
            acc = acc + e * e
        return weight * acc

    return final_cost


def simple_immediate_cost(chain, body, point, final_target, weight):
    """cost_functions.jl:34-54: Σ uᵢ² (mechanism, body, point, target, weight unused)."""

    def immediate_cost(x, u):
        acc = 0.0
        for k in range(len(u)):
            acc = acc + u[k] * u[k]
        return acc

    return immediate_cost
