"""CPU tests of the reference's documented per-step API as re-exposed by ilqr_amd.helpers
(docs/src/documentation.md:13-51; /root/reference/src/backward_pass.jl:81-109, 134-153,
177-186, 207-218, 262-273) against the oracle's restatement (oracle/ilqr_oracle.py).

The algebra helpers run with torch on the inputs' device (host algebra, numpy in → numpy
out) — here the CPU. Tolerance: rel 1e-12 (matmul association and the LU of
torch.linalg.solve vs numpy's differ in rounding only). The cost quadratizations'
closed forms are checked against the oracle's dual-number AD (ForwardDiff's role),
exactly for the quadratic costs and at 1e-12 otherwise. linearize_dynamics runs on the
device: tests/test_gpu_helpers.py.
"""
import numpy as np
import pytest
import torch

from ilqr_amd import helpers as H
from ilqr_amd.problems import (QuadraticCost, QuadraticFinalCost, TwoLinkCost, TwoLinkFinalCost,
                               random_lq_batch, two_link_closures)
from oracle import ilqr_oracle as O

TOL = 1e-12


def rel(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def _step_inputs(n, m, seed):
    rng = np.random.default_rng(seed)
    A = np.eye(n) + 0.1 * rng.standard_normal((n, n))
    B = rng.standard_normal((n, m))
    r, s = rng.standard_normal(m), rng.standard_normal(n)
    P = rng.standard_normal((m, n))
    Mr = rng.standard_normal((m, m))
    R = Mr @ Mr.T + np.eye(m)
    Ms = rng.standard_normal((n, n))
    S = Ms @ Ms.T + np.eye(n)
    return A, B, r, P, R, s, S


@pytest.mark.parametrize("n,m", [(12, 4), (4, 2), (4, 1), (7, 3)])
def test_algebra_helpers_equal_oracle(n, m):
    A, B, r, P, R, s, S = _step_inputs(n, m, seed=n * 10 + m)
    g, G, Hm = H.optimal_controller_param(A, B, r, P, R, s, S)
    go, Go, Ho = O.optimal_controller_param(A, B, r, P, R, s, S)
    assert rel(g, go) < TOL and rel(G, Go) < TOL and rel(Hm, Ho) < TOL
    du, K = H.feedback_parameters(g, G, Hm)
    duo, Ko = O.feedback_parameters(go, Go, Ho)
    assert rel(du, duo) < TOL and rel(K, Ko) < TOL
    q, qv = 0.7, np.random.default_rng(1).standard_normal(n)
    Q = np.eye(n) * 2.0
    sn, svn, Sn = H.step_back(A, q, qv, Q, g, G, Hm, du, K, 1.5, s, S)
    so, svo, So = O.step_back(A, q, qv, Q, go, Go, Ho, duo, Ko, 1.5, s, S)
    assert isinstance(sn, float)
    assert abs(sn - so) / abs(so) < TOL and rel(svn, svo) < TOL and rel(Sn, So) < TOL


def test_algebra_helpers_batched_and_torch():
    """Leading batch dimensions broadcast; torch in → torch out."""
    ins = [_step_inputs(12, 4, seed=b) for b in range(5)]
    stk = [np.stack([x[k] for x in ins]) for k in range(7)]
    g, G, Hm = H.optimal_controller_param(*(torch.from_numpy(a) for a in stk))
    assert isinstance(g, torch.Tensor) and g.shape == (5, 4) and G.shape == (5, 4, 12)
    du, K = H.feedback_parameters(g, G, Hm)
    for b in range(5):
        go, Go, Ho = O.optimal_controller_param(*ins[b])
        duo, Ko = O.feedback_parameters(go, Go, Ho)
        assert rel(du[b].numpy(), duo) < TOL and rel(K[b].numpy(), Ko) < TOL


def test_feedback_parameters_fixed_regulariser():
    """H_reg = H + 0.01 I (backward_pass.jl:214), no adaptation: a singular H still solves."""
    g, G = np.array([1.0, -2.0]), np.arange(8.0).reshape(2, 4)
    Hm = np.zeros((2, 2))
    du, K = H.feedback_parameters(g, G, Hm)
    assert np.allclose(du, -g / 0.01) and np.allclose(K, -G / 0.01)


def test_quadratizations_quadratic_family():
    lq, x, u = random_lq_batch(1, 6, 3, 4, seed=3)
    lc, lf = QuadraticCost(lq.Q[0], lq.R[0]), QuadraticFinalCost(lq.Qf[0])
    got = H.immediate_cost_quadratization(x[0, 1], u[0, 1], lc)
    ref = O.immediate_cost_quadratization(x[0, 1], u[0, 1], lc)   # the oracle's dual-number AD
    for a, b in zip(got, ref):
        assert rel(a, b) < TOL, (a, b)
    gf = H.final_cost_quadratization(x[0, -1], lf)
    rf = O.final_cost_quadratization(x[0, -1], lf)
    for a, b in zip(gf, rf):
        assert rel(a, b) < TOL


def test_quadratizations_two_link():
    f, lc, lf = two_link_closures()
    rng = np.random.default_rng(7)
    for _ in range(4):
        x, u = rng.standard_normal(4), rng.standard_normal(2)
        got = H.immediate_cost_quadratization(x, u, lc)
        ref = O.immediate_cost_quadratization(x, u, O.TwoLink.immediate_cost)
        for a, b in zip(got, ref):
            assert rel(a, b) < TOL
        gf = H.final_cost_quadratization(x, lf)
        rf = O.final_cost_quadratization(x, O.TwoLink.final_cost)
        for a, b in zip(gf, rf):
            assert rel(a, b) < TOL
    assert isinstance(lc, TwoLinkCost) and isinstance(lf, TwoLinkFinalCost)


def test_quadratizations_torch_closure():
    """An arbitrary torch closure goes through torch.func (ForwardDiff's role): a cost with
    a cross term gives the nu × nx 𝐏 (backward_pass.jl:98, 105)."""
    W = torch.tensor([[1.0, 2.0, 0.0], [0.0, -1.0, 3.0]], dtype=torch.float64)

    def lc(x, u):
        return (x ** 4).sum() + u @ (W @ x) + torch.sin(u).sum()

    x = torch.tensor([0.3, -0.2, 0.5], dtype=torch.float64)
    u = torch.tensor([0.1, -0.4], dtype=torch.float64)
    q, qv, r, Q, P, R = H.immediate_cost_quadratization(x, u, lc)
    assert torch.allclose(qv, 4 * x ** 3 + W.T @ u, rtol=1e-14)
    assert torch.allclose(r, W @ x + torch.cos(u), rtol=1e-14)
    assert torch.allclose(Q, torch.diag(12 * x ** 2), rtol=1e-14)
    assert torch.allclose(P, W, rtol=1e-14) and P.shape == (2, 3)
    assert torch.allclose(R, torch.diag(-torch.sin(u)), rtol=1e-14)


def test_helpers_compose_into_backward_pass():
    """The reference's backward_pass loop (:335-350) written with the re-exposed helpers
    (the oracle's linearisation, CPU) equals the oracle's backward_pass — the 2-link arm."""
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "twolink_t50.npz"), allow_pickle=False)
    x, u = z["x"][0], z["u"][0]
    f, lc, lf = two_link_closures()
    N = x.shape[0]
    qn, qvn, Qn = H.final_cost_quadratization(x[N - 1], lf)
    s1, sv1, S1 = qn, qvn, Qn
    dus, Ks = np.zeros((N - 1, 2)), np.zeros((N - 1, 2, 4))
    for i in range(N - 2, -1, -1):
        A, B = O.linearize_dynamics(x[i], u[i], O.TwoLink.dynamicsf)
        q, qv, r, Q, P, R = H.immediate_cost_quadratization(x[i], u[i], lc)
        g, G, Hm = H.optimal_controller_param(A, B, r, P, R, sv1, S1)
        dus[i], Ks[i] = H.feedback_parameters(g, G, Hm)
        s1, sv1, S1 = H.step_back(A, q, qv, Q, g, G, Hm, dus[i], Ks[i], s1, sv1, S1)
    d_ref, K_ref = O.backward_pass(x, u, O.TwoLink.dynamicsf, O.TwoLink.immediate_cost, O.TwoLink.final_cost)
    assert rel(dus, d_ref) < 1e-10 and rel(Ks, K_ref) < 1e-10
