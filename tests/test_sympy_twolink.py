"""Independent symbolic pin of the 2-link arm's linearisation.

The oracle differentiates the reference's dynamicsf (test/2_link_example/
2_link_helper_functions.jl:29-79) with forward-mode duals (oracle/dual.py, the
ForwardDiff restatement); the device does the same with Dual<4+NU> (ilqr_twolink.hip).
Here A = ∂f/∂x and B = ∂f/∂u (src/backward_pass.jl:25-40) are derived a different way:
sympy builds the continuous dynamics from the reference's formulas — InertiaMatrix
(:29-33), CoriolisMatrix with its literal index expression and the `for k in
length(θ)` quirk (:36-47; ∇M = jacobian(InertiaMatrix, θ) reshaped column-major,
:37-38), state_dot (:51-69) — and differentiates it symbolically; the RK4 step (:71-78)
is then differentiated by the chain rule through its four stages. Both the nu = 2
reference shape and the nu = 1 variant f(x, [u₁, 0]) are checked at seeded points.
"""
import math

import numpy as np
import pytest
import sympy as sp

from oracle import dual
from oracle import ilqr_oracle as O

TL = O.TwoLink


def _continuous():
    th1, th2, w1, w2, u1, u2 = sp.symbols("th1 th2 w1 w2 u1 u2", real=True)
    a, b, d = sp.Float(TL.alpha, 30), sp.Float(TL.beta, 30), sp.Float(TL.delta, 30)
    th = [th1, th2]
    M = sp.Matrix([[a + 2 * b * sp.cos(th2), d + b * sp.cos(th2)],
                   [d + b * sp.cos(th2), d]])                                   # :29-33
    # ∇M = jacobian(InertiaMatrix, θ) is 4×2 over vec(M) (column-major); reshaped to
    # (2,2,2) column-major, ∇M[p,q,r] = ∂M[p,q]/∂θ_r (1-based in the reference)
    dM = lambda p, q, r: sp.diff(M[p, q], th[r])                                # noqa: E731
    k = 1  # `for k in length(θ)`: the single value k = length(θ) = 2 (0-based 1)
    C = sp.Matrix(2, 2, lambda i, j: sp.Rational(1, 2) * (dM(k, i, j) + dM(j, i, k) - dM(i, k, j)) * [w1, w2][k])
    acc = -(M.inv() * C) * sp.Matrix([w1, w2]) + M.inv() * sp.Matrix([u1, u2])  # :56-66
    f = sp.Matrix([w1, w2, acc[0], acc[1]])
    z = sp.Matrix([th1, th2, w1, w2, u1, u2])
    J = f.jacobian(z)
    args = (th1, th2, w1, w2, u1, u2)
    return sp.lambdify(args, f, "numpy"), sp.lambdify(args, J, "numpy")


F_C, J_C = _continuous()


def fc(x, u):
    return np.array(F_C(*x, *u), dtype=float).reshape(4)


def jc(x, u):
    return np.array(J_C(*x, *u), dtype=float).reshape(4, 6)


def rk4_jacobian(x, u):
    """f = RK4(Δt) of the symbolic continuous dynamics and d f / d(x, u) by the chain rule."""
    dt = TL.dt
    E = np.hstack([np.eye(4), np.zeros((4, 2))])          # dx/dz
    Eu = np.hstack([np.zeros((2, 4)), np.eye(2)])          # du/dz
    k1 = dt * fc(x, u)
    dk1 = dt * jc(x, u) @ np.vstack([E, Eu])
    y2, dy2 = x + k1 / 2, E + dk1 / 2
    k2 = dt * fc(y2, u)
    dk2 = dt * jc(y2, u) @ np.vstack([dy2, Eu])
    y3, dy3 = x + k2 / 2, E + dk2 / 2
    k3 = dt * fc(y3, u)
    dk3 = dt * jc(y3, u) @ np.vstack([dy3, Eu])
    y4, dy4 = x + k3, E + dk3
    k4 = dt * fc(y4, u)
    dk4 = dt * jc(y4, u) @ np.vstack([dy4, Eu])
    out = x + (1 / 6) * (k1 + 2 * k2 + 2 * k3 + k4)
    J = E + (1 / 6) * (dk1 + 2 * dk2 + 2 * dk3 + dk4)
    return out, J[:, :4], J[:, 4:]


def points(n, seed):
    rng = np.random.default_rng(seed)
    return [(np.concatenate([rng.uniform(-math.pi, math.pi, 2), rng.uniform(-3, 3, 2)]),
             rng.uniform(-5, 5, 2)) for _ in range(n)]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_sympy_rk4_jacobians_match_dual_ad_nu2(seed):
    for x, u in points(6, seed):
        f_s, A_s, B_s = rk4_jacobian(x, u)
        f_o = TL.dynamicsf(x, u)
        A_o = dual.jacobian(lambda z: TL.dynamicsf(z, u), x)       # backward_pass.jl:32
        B_o = dual.jacobian(lambda v: TL.dynamicsf(x, v), u)       # backward_pass.jl:33
        assert np.abs(f_s - f_o).max() <= 1e-13 * max(1.0, np.abs(f_o).max())
        assert np.abs(A_s - A_o).max() <= 1e-12 * max(1.0, np.abs(A_o).max())
        assert np.abs(B_s - B_o).max() <= 1e-12 * max(1.0, np.abs(B_o).max())


def test_sympy_rk4_jacobians_match_dual_ad_nu1():
    """f₁(x, u) = f(x, [u₁, 0]): A is f's A at [u₁, 0], B is f's first B column."""
    for x, u in points(8, 7):
        u1 = np.array([u[0], 0.0])
        _, A_s, B_s = rk4_jacobian(x, u1)
        A_o = dual.jacobian(lambda z: TL.dynamicsf_nu1(z, u[:1]), x)
        B_o = dual.jacobian(lambda v: TL.dynamicsf_nu1(x, v), u[:1])
        assert np.abs(A_s - A_o).max() <= 1e-12 * max(1.0, np.abs(A_o).max())
        assert np.abs(B_s[:, :1] - B_o).max() <= 1e-12 * max(1.0, np.abs(B_o).max())


def test_sympy_coriolis_matrix_structure():
    """What the reference's CoriolisMatrix (:36-47) computes, symbolically: its index
    expression ½(∇M[k,i,j] + ∇M[j,i,k] − ∇M[i,k,j])θ̇ₖ reduces (M symmetric) to
    ½(∂M_ij/∂θ_k)θ̇ₖ, i.e. C = ½Ṁ — not the Christoffel-symbol Coriolis matrix — and the
    `for k in length(θ)` loop (k = 2 only) loses nothing for this arm because M does not
    depend on θ₁. The restatement and the device reproduce C = ½ ∂M/∂θ₂ · θ̇₂ literally."""
    th1, th2, w1, w2 = sp.symbols("th1 th2 w1 w2", real=True)
    a, b, d = TL.alpha, TL.beta, TL.delta
    M = sp.Matrix([[a + 2 * b * sp.cos(th2), d + b * sp.cos(th2)], [d + b * sp.cos(th2), d]])
    th, w = [th1, th2], [w1, w2]
    dM = lambda p, q, r: sp.diff(M[p, q], th[r])  # noqa: E731
    ref = lambda ks: sp.Matrix(2, 2, lambda i, j: sum(  # noqa: E731
        sp.Rational(1, 2) * (dM(k, i, j) + dM(j, i, k) - dM(i, k, j)) * w[k] for k in ks))
    half_mdot = sp.Matrix(2, 2, lambda i, j: sp.Rational(1, 2) * sum(dM(i, j, k) * w[k] for k in range(2)))
    christoffel = sp.Matrix(2, 2, lambda i, j: sum(
        sp.Rational(1, 2) * (dM(i, j, k) + dM(i, k, j) - dM(j, k, i)) * w[k] for k in range(2)))
    assert sp.simplify(ref([1]) - ref([0, 1])) == sp.zeros(2, 2)      # the k-loop quirk is harmless here
    assert sp.simplify(ref([1]) - half_mdot) == sp.zeros(2, 2)        # C = ½Ṁ
    assert sp.simplify(christoffel - half_mdot) != sp.zeros(2, 2)     # ... which is not Christoffel's
