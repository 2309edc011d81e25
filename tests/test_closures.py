"""CPU checks of the generic-closure machinery behind the reference's RBD caller
(test/RBD_2_link_example/animate_RBD_2_link.jl:31: iLQR.fit with 16-state / 8-input
closures, RBD_helper_functions.jl:48-116):

* the floating-base arm closure (tests/closures.py::rbd_floating_arm) — its oracle.jet
  Jacobians against central differences, energy conservation of the unforced RK4
  rollout (M and dynamics_bias consistent), the mass matrix's known translational block;
* the torch form of the same closure against the numpy one, and the product's
  derivative tiles (ilqr_amd.tiles, reverse mode) against oracle.jet — including the
  PyTorch forward-mode-under-vmap solve defect that made tiles.py use jacrev;
* the batched closure oracle (oracle/closure_fit.py) pinned to the per-trajectory
  restatement (oracle/ilqr_oracle.fit on oracle.dual) on a small nonlinear problem.
"""
import numpy as np
import pytest
import torch

from closures import (coupled_pendula, coupled_pendula_arr, jet_ns, oracle_ns, rbd_cost_quads,
                      rbd_floating_arm, rbd_initial_state, torch_arr_ns)
from oracle import closure_fit as CF
from oracle import ilqr_oracle as O
from oracle import jet


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def points(P=64, seed=0):
    rng = np.random.default_rng(seed)
    return 0.5 * rng.standard_normal((P, 16)), rng.standard_normal((P, 8))


def test_rbd_jet_jacobians_match_central_differences():
    f, _, _ = rbd_floating_arm(jet_ns())
    x, u = points(8)
    A, B = jet.jacobians(f, x, u)
    h = 1e-6
    for i in range(3):
        Afd = np.stack([(f(x[i:i + 1] + h * e, u[i:i + 1]) - f(x[i:i + 1] - h * e, u[i:i + 1]))[0] / (2 * h)
                        for e in np.eye(16)], axis=1)
        Bfd = np.stack([(f(x[i:i + 1], u[i:i + 1] + h * e) - f(x[i:i + 1], u[i:i + 1] - h * e))[0] / (2 * h)
                        for e in np.eye(8)], axis=1)
        assert rel(A[i], Afd) < 1e-8 and rel(B[i], Bfd) < 1e-7


def test_rbd_mass_matrix_and_energy():
    f, _, _ = rbd_floating_arm(jet_ns())
    x, _ = points(16, seed=1)
    M = f.mass_matrix(x)
    assert np.allclose(M, np.swapaxes(M, 1, 2), atol=1e-12)
    assert (np.linalg.eigvalsh(M) > 0).all()
    # translational block of the base: the total mass 30 + 3 + 3, in body axes
    assert np.allclose(M[:, 3:6, 3:6], 36.0 * np.eye(3), atol=1e-12)
    # unforced, zero gravity: ½ vᵀ M(θ) v is conserved (to RK4's O(Δt⁴) drift); it is
    # only if dynamics_bias is the Coriolis term of this M
    xs = rbd_initial_state()[None].repeat(4, 0)
    xs[:, 8:] = 0.4 * np.random.default_rng(2).standard_normal((4, 8))
    energy = lambda s: 0.5 * np.einsum("bi,bij,bj->b", s[:, 8:], f.mass_matrix(s), s[:, 8:])  # noqa: E731
    e0 = energy(xs)
    for _ in range(300):
        xs = f(xs, np.zeros((4, 8)))
    assert rel(energy(xs), e0) < 1e-8
    # not vacuous: the velocity-product forces are far from zero along the way
    assert np.abs(f.dynamics_bias(xs)).max() > 1e-3


def test_rbd_torch_closure_and_tiles_match_the_oracle():
    """The product's derivative tiles (torch.func on the closure, tiles.py) equal the
    oracle's forward-mode Jacobians and the exact cost quadratizations."""
    from ilqr_amd.tiles import derivative_tiles
    fj, lj, lfj = rbd_floating_arm(jet_ns())
    ft, lt, lft = rbd_floating_arm(torch_arr_ns("cpu"))
    x, u = points(3 * 5 + 3, seed=3)
    xb = torch.from_numpy(x[:18].reshape(3, 6, 16).copy())
    ub = torch.from_numpy(u[:15].reshape(3, 5, 8).copy())
    assert rel(ft(xb, torch.cat([ub, ub[:, :1]], 1)).numpy(), fj(xb.numpy(), np.concatenate([ub, ub[:, :1]], 1))) < 1e-15
    tl = derivative_tiles(xb, ub, ft, lt, lft)
    A, B = jet.jacobians(fj, xb[:, :5].reshape(-1, 16).numpy(), ub.reshape(-1, 8).numpy())
    assert rel(tl["A"].reshape(-1, 16, 16), A) < 1e-13 and rel(tl["B"].reshape(-1, 16, 8), B) < 1e-13
    q, fq = rbd_cost_quads()
    lx, lu, lxx, lux, luu = q(xb[:, :5].reshape(-1, 16).numpy(), ub.reshape(-1, 8).numpy())
    for k, v in (("lx", lx), ("lu", lu), ("lxx", lxx), ("luu", luu)):
        assert rel(tl[k].reshape(v.shape), v) < 1e-14, k
    assert np.abs(tl["lux"].numpy()).max() == 0.0 and lux.max() == 0.0
    lfx, lfxx = fq(xb[:, 5].numpy())
    assert rel(tl["lfx"], lfx) < 1e-14 and rel(tl["lfxx"], lfxx) < 1e-14


def test_vmapped_forward_mode_solve_defect_is_avoided():
    """torch 2.10: vmap(jacfwd) through linalg.solve is wrong; vmap(jacrev), what
    tiles.py uses, is right. Recorded so that a fixed PyTorch is noticed."""
    from torch.func import jacfwd, jacrev, vmap
    g = torch.Generator().manual_seed(0)
    M = torch.randn(5, 8, 8, dtype=torch.float64, generator=g) + 8 * torch.eye(8, dtype=torch.float64)
    b = torch.randn(5, 8, dtype=torch.float64, generator=g)
    fn = lambda M, b: torch.linalg.solve(M, b.unsqueeze(-1)).squeeze(-1)  # noqa: E731
    inv = torch.linalg.inv(M)
    assert (vmap(jacrev(fn, argnums=1))(M, b) - inv).abs().max() < 1e-12
    fwd_err = float((vmap(jacfwd(fn, argnums=1))(M, b) - inv).abs().max())
    print("vmap(jacfwd) through linalg.solve: max error", fwd_err)


def test_closure_fit_oracle_matches_per_trajectory_oracle():
    """oracle/closure_fit.py (batched, oracle.jet, C recursion) against ilqr_oracle.fit
    (one trajectory at a time on oracle.dual scalars) on the coupled pendula."""
    nb, T = 3, 15
    fd, ld, lfd = coupled_pendula(oracle_ns())
    fa, la, lfa = coupled_pendula_arr(jet_ns())
    rng = np.random.default_rng(4)
    x = np.zeros((nb, T + 1, 4))
    u = 0.3 * rng.standard_normal((nb, T, 2))
    x[:, 0] = rng.uniform(-1, 1, (nb, 4))
    for t in range(T):
        x[:, t + 1] = fa(x[:, t], u[:, t])
    q, fq = CF.dual_quads(ld, lfd)
    r = CF.fit(x, u, fa, la, lfa, q, fq, max_iter=25, tol=1e-6)
    for b in range(nb):
        h = []
        xo, uo = O.fit(x[b], u[b], fd, ld, lfd, max_iter=25, tol=1e-6, max_trials=64, history=h,
                       symmetrize=True)
        assert int(r["iters"][b]) == len(h)
        assert [int(v) for v in r["history"]["trials"][:len(h), b]] == [e["trials"] for e in h]
        assert rel(r["x"][b], xo) < 1e-9 and rel(r["u"][b], uo) < 1e-9


def test_jet_matches_dual_forward_mode():
    """oracle.jet (array-valued forward mode) against oracle.dual (the ForwardDiff
    restatement, scalar duals) on the same closure written both ways: the Jacobians of
    linearize_dynamics (src/backward_pass.jl:32-33) agree to rounding."""
    from oracle import dual
    fa, _, _ = coupled_pendula_arr(jet_ns())
    fd, _, _ = coupled_pendula(oracle_ns())
    rng = np.random.default_rng(5)
    x, u = rng.uniform(-1, 1, (6, 4)), rng.standard_normal((6, 2))
    A, B = jet.jacobians(fa, x, u)
    for p in range(6):
        Ad = dual.jacobian(lambda z: fd(z, u[p]), x[p])
        Bd = dual.jacobian(lambda v: fd(x[p], v), u[p])
        assert rel(A[p], Ad) < 1e-15 and rel(B[p], Bd) < 1e-15


def test_jet_elementary_rules():
    """solve / matmul / cat / tr / division on Jets against central differences."""
    rng = np.random.default_rng(6)
    M0 = rng.standard_normal((3, 4, 4)) + 4 * np.eye(4)
    b0 = rng.standard_normal((3, 4))

    def g(x):  # x (P, 4) → (P, 4): a mix of every Jet operation the closures use
        M = M0 + jet.tr(x[..., :, None] * x[..., None, :]) * 0.1
        y = jet.solve(M, b0 + x)
        z = jet.cat([y[..., :2] / (2.0 + x[..., 2:3] * x[..., 2:3]), jet.sin(y[..., 2:]) - jet.cos(x[..., :2])])
        return (M @ z[..., None])[..., 0] * 0.5
    x = rng.standard_normal((3, 4))
    J, _ = jet.jacobians(lambda a, _u: g(a), x, np.zeros((3, 1)))
    h = 1e-6
    Jfd = np.stack([(g(x + h * e) - g(x - h * e)) / (2 * h) for e in np.eye(4)], axis=-1)
    assert rel(J, Jfd) < 1e-8


def test_rollout_graph_bookkeeping_on_cpu():
    """The capture-time linalg mode leaves torch.linalg alone outside it and in other
    threads; CPU tensors never build a graph (the product path is the device); a cached
    graph does not keep its closure alive."""
    import gc
    import threading
    import weakref
    import torch
    from ilqr_amd import tiles
    A = torch.tensor([[2.0, 1.0], [1.0, 3.0]], dtype=torch.float64)
    b = torch.tensor([[1.0], [2.0]], dtype=torch.float64)
    Z = torch.zeros(2, 2, dtype=torch.float64)
    ref = torch.linalg.solve(A, b)
    seen = {}

    def other_thread():
        try:
            torch.linalg.solve(Z, b)
            seen["raised"] = False
        except RuntimeError:
            seen["raised"] = True
    with tiles._capturable_linalg():
        assert torch.equal(torch.linalg.solve(A, b), ref)
        assert torch.equal(torch.linalg.inv(A), torch.linalg.inv_ex(A)[0])
        # a singular system: no host-side check, non-finite values instead of an exception
        assert not torch.isfinite(torch.linalg.solve(Z, b)).all()
        # under vmap too (the rollout calls the closure through vmap)
        from torch.func import vmap
        assert torch.equal(vmap(lambda M, v: torch.linalg.solve(M, v))(A[None], b.T), ref.T)
        t = threading.Thread(target=other_thread)
        t.start()
        t.join()
    assert seen["raised"] is True           # the mode is this thread's only
    with pytest.raises(RuntimeError):
        torch.linalg.solve(Z, b)
    x = torch.zeros(1, 3, 2, dtype=torch.float64)
    u = torch.zeros(1, 2, 1, dtype=torch.float64)
    f = lambda a, v: a  # noqa: E731
    assert tiles._rollout_graph(f, x, u) is None
    assert f not in tiles._GRAPHS
    # a cached graph holds no reference to its closure: the entry goes with the closure
    g = lambda a, v: a  # noqa: E731
    wr = weakref.ref(g)
    tiles._GRAPHS[g] = {"entry": tiles._RolloutGraph(x, u)}
    n = len(tiles._GRAPHS)
    del g
    gc.collect()
    assert wr() is None and len(tiles._GRAPHS) == n - 1


def test_rollout_graph_cache_is_bounded_and_clearable():
    """The cached graphs' static buffers stay under MAX_GRAPH_BYTES (least recently used
    evicted first) and api.clear_cache() releases them all."""
    import torch
    from ilqr_amd import api, tiles
    x = torch.zeros(4, 11, 3, dtype=torch.float64)
    u = torch.zeros(4, 10, 2, dtype=torch.float64)
    one = tiles._RolloutGraph(x, u).nbytes
    fs = [lambda a, v, i=i: a for i in range(3)]
    old = tiles.MAX_GRAPH_BYTES
    try:
        tiles.clear_graphs()
        tiles.MAX_GRAPH_BYTES = 2 * one
        for i, f in enumerate(fs):
            g = tiles._RolloutGraph(x, u)
            g.seq = i + 1
            with tiles._GRAPHS_LOCK:
                assert tiles._evict_for(g.nbytes)
                tiles._GRAPHS[f] = {"k": g}
        assert tiles._graph_bytes() <= tiles.MAX_GRAPH_BYTES
        assert not tiles._GRAPHS.get(fs[0]) and tiles._GRAPHS[fs[1]] and tiles._GRAPHS[fs[2]]
        with tiles._GRAPHS_LOCK:                       # larger than the bound: refused
            assert not tiles._evict_for(3 * one)
        api.clear_cache()
        assert len(tiles._GRAPHS) == 0
    finally:
        tiles.MAX_GRAPH_BYTES = old


def test_floating_restatement_conserves_energy():
    """With u = 0 and zero gravity the floating mechanism's kinetic energy is conserved
    (up to RK4's O(dt⁴) error): the restated mass matrix and Newton-Euler bias belong
    to one mechanism — for the 2Dof_arm and for a model with every term nonzero."""
    from closures import coupled_floating_model, floating_energy, jet_ns, rbd_floating_arm
    rng = np.random.default_rng(4)
    for model in (None, coupled_floating_model()):
        f, _, _ = rbd_floating_arm(jet_ns(), model=model)
        x = np.zeros((6, 16))
        x[:, 0:3] = 0.3 * rng.standard_normal((6, 3))
        x[:, 6:8] = rng.uniform(-2, 2, (6, 2))
        x[:, 8:16] = rng.standard_normal((6, 8))
        e0 = floating_energy(x, model)
        u = np.zeros((6, 8))
        for _ in range(200):
            x = f(x, u)
        e1 = floating_energy(x, model)
        assert np.abs(e1 - e0).max() / e0.max() < 1e-7, (e0, e1)
