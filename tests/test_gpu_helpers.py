"""GPU tests of linearize_dynamics (/root/reference/src/backward_pass.jl:25-40) through the
new C entry ilqr_linearize and the re-exposed Python helper.

* LQ family: the repaired known answer of test/test_linearize_dynamics.jl:24-25 — a linear
  f returns A, B exactly (bit-equal, every step), also on padded shapes.
* 2-link arm: ilqr_linearize's Dual<4+nu> Jacobians against the oracle's dual-number AD
  (oracle.dual, ForwardDiff's restatement) at rel 1e-12, on the committed golden
  trajectories (tests/golden/twolink_t50.npz), nu = 2 and nu = 1; the trajectory form the
  reference's test calls (x, u with 100 rows → 𝐀s[i, :, :]); the vector form; and the
  one-step prediction f(x + δx, u + δu) ≈ f + Aδx + Bδu to second order.
* chains and arbitrary torch closures through the same helper.
"""
import ctypes as C
import os

import numpy as np
import pytest
import torch

from ilqr_amd import _lib, helpers as H
from ilqr_amd.problems import LinearDynamics, random_lq_batch, two_link_closures
from ilqr_amd.solver import Solver, _ptr
from oracle import ilqr_oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a = a.cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = b.cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


@pytest.mark.parametrize("nx,nu", [(12, 4), (4, 2), (7, 3)])
def test_ilqr_linearize_lq_exact(gpu, nx, nu):
    """Linear f: every step's (A_t, B_t) is the instance's (A, B) bit for bit."""
    B, T = 37, 9
    lq, x, u = random_lq_batch(B, nx, nu, T, seed=nx)
    s = Solver(nx, nu, T, B)
    s.set_problem(lq)
    A = torch.empty((B, T, nx, nx), dtype=torch.float64, device="cuda")
    Bm = torch.empty((B, T, nx, nu), dtype=torch.float64, device="cuda")
    s._bind_stream()
    rc = s.lib.ilqr_linearize(s.h, s._p(), None, None, _ptr(A), _ptr(Bm))
    torch.cuda.synchronize()
    s.close()
    assert rc == _lib.OK
    assert np.array_equal(A.cpu().numpy(), np.broadcast_to(lq.A[:, None], (B, T, nx, nx)))
    assert np.array_equal(Bm.cpu().numpy(), np.broadcast_to(lq.B[:, None], (B, T, nx, nu)))


def test_ilqr_linearize_bad_args(gpu):
    s = Solver(4, 2, 5, 3, kind=_lib.PROBLEM_TWO_LINK)
    A = torch.empty((3, 5, 4, 4), dtype=torch.float64, device="cuda")
    Bm = torch.empty((3, 5, 4, 2), dtype=torch.float64, device="cuda")
    assert s.lib.ilqr_linearize(s.h, s._p(), None, None, _ptr(A), _ptr(Bm)) == _lib.ERR_BAD_ARG
    assert s.lib.ilqr_linearize(s.h, None, None, None, _ptr(A), _ptr(Bm)) == _lib.ERR_BAD_ARG
    s.close()


@pytest.mark.parametrize("nu", [2, 1])
def test_ilqr_linearize_two_link_vs_dual_oracle(gpu, nu):
    z = np.load(os.path.join(GOLD, "twolink_t50.npz"), allow_pickle=False)
    x, u = z["x"], z["u"][..., :nu].copy()
    nb, T = u.shape[:2]
    s = Solver(4, nu, T, nb, kind=_lib.PROBLEM_TWO_LINK)
    xd, ud = torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda()
    A = torch.empty((nb, T, 4, 4), dtype=torch.float64, device="cuda")
    Bm = torch.empty((nb, T, 4, nu), dtype=torch.float64, device="cuda")
    s._bind_stream()
    assert s.lib.ilqr_linearize(s.h, s._p(), _ptr(xd), _ptr(ud), _ptr(A), _ptr(Bm)) == _lib.OK
    torch.cuda.synchronize()
    s.close()
    f = O.TwoLink.dynamicsf if nu == 2 else O.TwoLink.dynamicsf_nu1
    for b in range(nb):
        for t in range(0, T, 7):
            Ao, Bo = O.linearize_dynamics(x[b, t], u[b, t], f)
            assert rel(A[b, t], Ao) < 1e-12, (b, t)
            assert rel(Bm[b, t], Bo) < 1e-12, (b, t)


def test_linearize_dynamics_trajectory_form_two_link(gpu):
    """test/test_linearize_dynamics.jl:7-10 repaired: state_traj (100, 4), input_traj
    (100, 2) → 𝐀s (100, 4, 4), 𝐁s (100, 4, 2) — each the point form at that row, and the
    point form equal to the oracle's; the linearisation predicts a nearby step to second
    order (the test's comparison, which as written compares A x + B u with f(x, u) — only
    true for linear f, whose exact case is test_ilqr_linearize_lq_exact)."""
    f, _, _ = two_link_closures()
    rng = np.random.default_rng(0)
    xs, us = rng.random((100, 4)), rng.random((100, 2))
    As, Bs = H.linearize_dynamics(xs, us, f)
    assert As.shape == (100, 4, 4) and Bs.shape == (100, 4, 2)
    for i in (0, 41, 99):
        A1, B1 = H.linearize_dynamics(xs[i], us[i], f)
        assert np.array_equal(A1, As[i]) and np.array_equal(B1, Bs[i])
        Ao, Bo = O.linearize_dynamics(xs[i], us[i], O.TwoLink.dynamicsf)
        assert rel(As[i], Ao) < 1e-12 and rel(Bs[i], Bo) < 1e-12
    for eps in (1e-3, 1e-4):
        dx, du = eps * rng.standard_normal((100, 4)), eps * rng.standard_normal((100, 2))
        err = max(np.abs(f(xs[i] + dx[i], us[i] + du[i]) - f(xs[i], us[i]) - As[i] @ dx[i] - Bs[i] @ du[i]).max()
                  for i in range(100))
        assert err < 50 * eps ** 2, (eps, err)


def test_linearize_dynamics_lq_and_closures(gpu):
    """LinearDynamics through ilqr_linearize (exact), the same f as a torch closure through
    torch.func (exact too: a linear map), and a nonlinear torch closure against its
    analytic Jacobian."""
    lq, x, u = random_lq_batch(1, 6, 2, 10, seed=5)
    f = LinearDynamics(lq.A[0], lq.B[0])
    As, Bs = H.linearize_dynamics(x[0], u[0], f)
    assert np.array_equal(As, np.broadcast_to(lq.A[0], (10, 6, 6)))
    assert np.array_equal(Bs, np.broadcast_to(lq.B[0], (10, 6, 2)))
    At = torch.from_numpy(lq.A[0]).cuda()
    Bt = torch.from_numpy(lq.B[0]).cuda()
    Ag, Bg = H.linearize_dynamics(torch.from_numpy(x[0]).cuda(), torch.from_numpy(u[0]).cuda(),
                                  lambda xx, uu: At @ xx + Bt @ uu)
    assert torch.equal(Ag, At.expand(10, 6, 6)) and torch.equal(Bg, Bt.expand(10, 6, 2))

    def g(xx, uu):
        return torch.stack([torch.sin(xx[0]) * uu[0], xx[1] ** 2 + xx[0] * uu[0]])

    xv = torch.tensor([0.3, -0.7], dtype=torch.float64, device="cuda")
    uv = torch.tensor([1.5], dtype=torch.float64, device="cuda")
    A1, B1 = H.linearize_dynamics(xv, uv, g)
    assert torch.allclose(A1, torch.tensor([[np.cos(0.3) * 1.5, 0.0], [1.5, -1.4]], dtype=torch.float64,
                                           device="cuda"), rtol=1e-14)
    assert torch.allclose(B1, torch.tensor([[np.sin(0.3)], [0.3]], dtype=torch.float64, device="cuda"), rtol=1e-14)


def test_linearize_dynamics_chain(gpu):
    """ChainDynamics through ilqr_chain_linearize (fp64, dual numbers) against central
    differences of the chain's own dynamics."""
    from ilqr_amd.chain import chain_closures, rbd_2dof_problem
    pr = rbd_2dof_problem(2)
    f, _, _ = chain_closures(pr)
    rng = np.random.default_rng(2)
    xs, us = rng.uniform(-1, 1, (6, 4)), rng.uniform(-1, 1, (6, 2))
    As, Bs = H.linearize_dynamics(xs, us, f)
    assert As.shape == (6, 4, 4) and Bs.shape == (6, 4, 2)
    for i in (0, 5):
        h = 1e-6
        Afd = np.stack([(f(xs[i] + h * e, us[i]) - f(xs[i] - h * e, us[i])) / (2 * h) for e in np.eye(4)], axis=1)
        Bfd = np.stack([(f(xs[i], us[i] + h * e) - f(xs[i], us[i] - h * e)) / (2 * h) for e in np.eye(2)], axis=1)
        assert rel(As[i], Afd) < 1e-7 and rel(Bs[i], Bfd) < 1e-7


def test_linearize_two_link_past_the_grid_y_limit_and_cached(gpu):
    """A horizon past HIP's 65,535 limit on gridDim.y (the Jacobian kernel strides its
    steps, advisor r04), and the helper's device workspace kept between calls
    (ilqr_amd.cache: one Solver for repeated calls of one shape)."""
    from ilqr_amd import cache
    f, _, _ = two_link_closures()
    rng = np.random.default_rng(3)
    T = 70_000
    xs, us = rng.random((T + 1, 4)), rng.random((T, 2))
    cache.clear()
    made = []
    orig = Solver.__init__

    def counting(self, *a, **k):
        made.append(a)
        orig(self, *a, **k)
    Solver.__init__ = counting
    try:
        As, Bs = H.linearize_dynamics(xs, us, f)
        As2, Bs2 = H.linearize_dynamics(xs, us, f)
    finally:
        Solver.__init__ = orig
    assert len(made) == 1 and np.array_equal(As, As2) and np.array_equal(Bs, Bs2)
    for i in (0, 65_534, 65_535, 65_536, T - 1):
        Ao, Bo = O.linearize_dynamics(xs[i], us[i], O.TwoLink.dynamicsf)
        assert rel(As[i], Ao) < 1e-12 and rel(Bs[i], Bo) < 1e-12, i
    cache.clear()
