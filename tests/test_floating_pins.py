"""Pins of the floating-base restatement (tests/closures.py rbd_floating_arm, the checker
of the ilqr_floating_* family and of the closure path at the reference RBD caller's shape,
test/RBD_2_link_example/RBD_helper_functions.jl:7, :48-79, test/urdf/2Dof_arm.urdf) that
do not share its formulation:

- the mass matrix against Σᵢ Jᵢᵀ 𝕀ᵢ Jᵢ with Jacobians from composed URDF transforms (no
  CRBA, no spatial algebra), at 1e-12;
- world-frame linear momentum R(p)·(M v)[3:6] conserved at u = 0 and zero gravity over
  300 RK4 steps. Unlike the energy test this ties M's base rows, the Newton-Euler bias
  and the MRP kinematics together: a COM or joint-frame error made the same way in M
  and the bias conserves energy but not this.

Parity against RigidBodyDynamics.jl itself stays unpinned (not runnable here)."""
import numpy as np
import pytest

from closures import (coupled_floating_model, floating_linear_momentum_world,
                      floating_mass_matrix_jacobians, jet_ns, rbd_floating_arm)

MODELS = {"2dof_arm": None, "coupled": coupled_floating_model()}


def states(n, seed):
    rng = np.random.default_rng(seed)
    x = np.zeros((n, 16))
    x[:, 0:3] = 0.4 * rng.standard_normal((n, 3))
    x[:, 3:6] = rng.standard_normal((n, 3))
    x[:, 6:8] = rng.uniform(-3.0, 3.0, (n, 2))
    x[:, 8:16] = rng.standard_normal((n, 8))
    return x


@pytest.mark.parametrize("name", list(MODELS))
def test_mass_matrix_equals_jacobian_formulation(name):
    model = MODELS[name]
    f, _, _ = rbd_floating_arm(jet_ns(), model=model)
    x = states(64, seed=11)
    Mc = f.mass_matrix(x)
    Mj = floating_mass_matrix_jacobians(x, model)
    assert np.abs(Mc - Mj).max() / np.abs(Mj).max() < 1e-12
    # and the independent one is a mass matrix: symmetric, positive definite
    assert np.abs(Mj - np.swapaxes(Mj, 1, 2)).max() < 1e-12 * np.abs(Mj).max()
    assert np.linalg.eigvalsh(Mj).min() > 0


def test_jacobian_formulation_sees_a_frame_error():
    """The KAT has teeth: moving link 2's COM (an error CRBA and RNEA would share) or
    turning joint 2's axis frame changes M well above the tolerance."""
    model = coupled_floating_model()
    x = states(8, seed=12)
    M = floating_mass_matrix_jacobians(x, model)
    bad = dict(model, com=(model["com"][0], tuple(np.add(model["com"][1], (0.0, 0.0, 1e-3)))))
    assert np.abs(floating_mass_matrix_jacobians(x, bad) - M).max() / np.abs(M).max() > 1e-6
    f, _, _ = rbd_floating_arm(jet_ns(), model=bad)
    assert np.abs(f.mass_matrix(x) - floating_mass_matrix_jacobians(x, bad)).max() / np.abs(M).max() < 1e-12


@pytest.mark.parametrize("name", list(MODELS))
def test_world_linear_momentum_is_conserved(name):
    model = MODELS[name]
    f, _, _ = rbd_floating_arm(jet_ns(), model=model)
    x = states(6, seed=13)
    p0 = floating_linear_momentum_world(x, model)
    u = np.zeros((x.shape[0], 8))
    for _ in range(300):
        x = f(x, u)
    p1 = floating_linear_momentum_world(x, model)
    scale = np.abs(p0).max()
    assert scale > 1.0
    assert np.abs(p1 - p0).max() / scale < 1e-7, (p0, p1)
