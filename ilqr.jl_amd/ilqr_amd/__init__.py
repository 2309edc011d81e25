"""ilqr_amd — MI355X-native batched iLQR (host-side mirror of aabouman/iLQR.jl's
`iLQR` module over the C ABI of libilqr_hip.so; see include/ilqr.h)."""
from .problems import (LinearDynamics, LQBatch, QuadraticCost, QuadraticFinalCost, TwoLinkArm,
                       TwoLinkCost, TwoLinkDynamics, TwoLinkDynamicsNu1, TwoLinkFinalCost, lq_from_closures,
                       quadrotor_batch, quadrotor_instance, random_lq_batch, two_link_closures,
                       two_link_initial_states)

__all__ = ["LinearDynamics", "QuadraticCost", "QuadraticFinalCost", "LQBatch",
           "lq_from_closures", "TwoLinkArm", "TwoLinkDynamics", "TwoLinkDynamicsNu1", "TwoLinkCost",
           "TwoLinkFinalCost", "two_link_closures", "two_link_initial_states", "quadrotor_batch", "quadrotor_instance", "random_lq_batch",
           "fit", "backward_pass", "forward_pass", "Solver", "selftest", "LineSearchExhausted",
           "ChainSolver", "ChainProblem", "rbd_2dof_problem", "chain_closures", "load_robot",
           "rbd_initial_states", "simple_final_cost", "simple_immediate_cost",
           "linearize_dynamics", "immediate_cost_quadratization", "final_cost_quadratization",
           "optimal_controller_param", "feedback_parameters", "step_back",
           "FloatingSolver", "FloatingProblem", "rbd_example_problem", "floating_closures"]

_HELPERS = ("linearize_dynamics", "immediate_cost_quadratization", "final_cost_quadratization",
            "optimal_controller_param", "feedback_parameters", "step_back")


def __getattr__(name):
    # the device API needs torch + libilqr_hip.so; import it lazily so problem
    # definitions stay usable without them
    if name in ("fit", "backward_pass", "forward_pass", "LineSearchExhausted"):
        from . import api
        return getattr(api, name)
    if name in _HELPERS:  # the reference's documented per-step API (docs/src/documentation.md)
        from . import helpers
        return getattr(helpers, name)
    if name in ("ChainSolver", "ChainProblem", "rbd_2dof_problem", "chain_closures", "load_robot",
                "rbd_initial_states"):
        from . import chain
        return getattr(chain, name)
    if name in ("FloatingSolver", "FloatingProblem", "rbd_example_problem", "floating_closures"):
        from . import floating
        return getattr(floating, name)
    if name in ("simple_final_cost", "simple_immediate_cost"):
        from . import cost_functions
        return getattr(cost_functions, name)
    if name in ("Solver", "selftest", "FitResult"):
        from . import solver
        return getattr(solver, name)
    raise AttributeError(name)
