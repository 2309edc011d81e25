"""GPU parity of ilqr_backward_tiles (backward_pass for
arbitrary closures from caller-supplied derivative tiles) and of the generic
closure path of the Python mirror.

Tolerances (fp64): same recursion as the LQ kernel (exact step_back rewrite, LDLᵀ,
periodic symmetrisation), so gains agree with the oracle to rounding amplified by
the recursion: rel 1e-10 on short literal cases, 1e-10 vs the symmetrised oracle on
T = 100; the LQ problem through tiles agrees with the fused LQ kernel to 1e-12.
"""
import os

import numpy as np
import pytest
import torch

from closures import coupled_pendula, oracle_ns, torch_ns, two_link_torch
from ilqr_amd import _lib, api
from ilqr_amd.problems import LQBatch, quadrotor_batch
from ilqr_amd.solver import Solver
from ilqr_amd.tiles import derivative_tiles
from oracle import cref
from oracle import ilqr_oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a = a.cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a, float)
    b = b.cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b, float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def to_dev(tl):
    return {k: (None if v is None else torch.as_tensor(np.ascontiguousarray(v)).cuda()) for k, v in tl.items()}


def to_np(tl):
    return {k: (None if v is None else v.cpu().numpy()) for k, v in tl.items()}


def pendula_batch(nb, T, seed=0):
    fo, _, _ = coupled_pendula(oracle_ns())
    rng = np.random.default_rng(seed)
    x = np.zeros((nb, T + 1, 4))
    u = 0.3 * rng.standard_normal((nb, T, 2))
    x[:, 0] = rng.uniform(-1, 1, (nb, 4))
    for b in range(nb):
        for t in range(T):
            x[b, t + 1] = np.asarray(fo(x[b, t], u[b, t]), float)
    return x, u


def lq_tiles(lq, x, u):
    """The LQ family's exact derivative tiles along (x, u)."""
    nb, T = u.shape[:2]
    Qs = lq.Q + lq.Q.transpose(0, 2, 1)
    Rs = lq.R + lq.R.transpose(0, 2, 1)
    Qfs = lq.Qf + lq.Qf.transpose(0, 2, 1)
    rep = lambda a: np.ascontiguousarray(np.broadcast_to(a[:, None], (nb, T) + a.shape[1:]))
    return {"A": rep(lq.A), "B": rep(lq.B), "lx": np.einsum("bij,btj->bti", Qs, x[:, :T]),
            "lu": np.einsum("bij,btj->bti", Rs, u), "lxx": rep(Qs), "lux": None, "luu": rep(Rs),
            "lfx": np.einsum("bij,bj->bi", Qfs, x[:, T]), "lfxx": Qfs}


def test_tiles_supported_shapes(gpu):
    lib = _lib.load()
    for nx in range(1, 17):
        for nu in range(1, 9):
            assert lib.ilqr_supported(_lib.PROBLEM_TILES, nx, nu) == 1
    for nx, nu in ((17, 1), (12, 9), (16, 9), (0, 1), (4, 0)):
        assert lib.ilqr_supported(_lib.PROBLEM_TILES, nx, nu) == 0


def random_tiles(nb, T, n, m, seed):
    rng = np.random.default_rng(seed)
    A = np.eye(n) + 0.03 * rng.standard_normal((nb, T, n, n))
    Bm = 0.2 * rng.standard_normal((nb, T, n, m))
    Mq = rng.standard_normal((nb, T, n, n))
    lxx = 0.1 * np.einsum("btij,btkj->btik", Mq, Mq) / n + np.eye(n)
    Mr = rng.standard_normal((nb, T, m, m))
    luu = 0.05 * np.einsum("btij,btkj->btik", Mr, Mr) / m + 0.2 * np.eye(m)
    Mf = rng.standard_normal((nb, n, n))
    return {"A": A, "B": Bm, "lx": rng.standard_normal((nb, T, n)), "lu": rng.standard_normal((nb, T, m)),
            "lxx": lxx, "lux": 0.05 * rng.standard_normal((nb, T, m, n)), "luu": luu,
            "lfx": rng.standard_normal((nb, n)), "lfxx": 0.1 * np.einsum("bij,bkj->bik", Mf, Mf) + 2 * np.eye(n)}


@pytest.mark.parametrize("n,m", [(1, 1), (2, 1), (3, 2), (5, 3), (6, 4), (7, 4), (9, 2), (11, 3), (12, 1)])
def test_tiles_every_shape_vs_oracle(gpu, n, m):
    """ilqr_backward_tiles is compiled for every nx ≤ 12, nu ≤ 4 (one MFMA tile)."""
    nb, T = 9, 40
    tl = random_tiles(nb, T, n, m, seed=100 * n + m)
    s = Solver(n, m, T, nb, kind=_lib.PROBLEM_TILES)
    d, K, st = s.backward_tiles(to_dev(tl))
    assert (st.cpu().numpy() == 0).all()
    dr, Kr, _ = cref.tiles_backward(tl, symmetrize=True)
    assert rel(d, dr) < 1e-10 and rel(K, Kr) < 1e-10


@pytest.mark.parametrize("n,m", [(13, 1), (16, 4), (4, 8), (1, 5), (12, 5), (15, 7), (16, 8)])
def test_tiles_wide_shapes_vs_oracle(gpu, n, m):
    """Shapes past one MFMA tile (nx ≤ 16, nu ≤ 8) run on the tiled wide kernel."""
    nb, T = 6, 40
    tl = random_tiles(nb, T, n, m, seed=1000 + 100 * n + m)
    s = Solver(n, m, T, nb, kind=_lib.PROBLEM_TILES)
    d, K, st = s.backward_tiles(to_dev(tl))
    assert (st.cpu().numpy() == 0).all()
    dr, Kr, _ = cref.tiles_backward(tl, symmetrize=True)
    assert rel(d, dr) < 1e-10 and rel(K, Kr) < 1e-10
    tl0 = dict(tl, lux=None)  # 𝐏 = NULL reads as zeros
    d0, K0, _ = s.backward_tiles(to_dev(tl0))
    dr0, Kr0, _ = cref.tiles_backward(tl0, symmetrize=True)
    assert rel(d0, dr0) < 1e-10 and rel(K0, Kr0) < 1e-10
    s.close()


@pytest.mark.parametrize("n,m", [(16, 5), (13, 7), (4, 6), (16, 8)])
def test_tiles_wide_mu_zero_padded_pivots(gpu, n, m):
    """μ = 0 on the wide kernel: with nu < 8 its padded LDLᵀ pivots were μ,
    so μ = 0 made them 0 and NaN reached the real gains. luu is positive definite here,
    so the unregularised system is solvable and the gains must match the oracle's."""
    nb, T = 5, 30
    tl = random_tiles(nb, T, n, m, seed=7000 + 10 * n + m)
    s = Solver(n, m, T, nb, kind=_lib.PROBLEM_TILES)
    try:
        d, K, st = s.backward_tiles(to_dev(tl), mu=0.0)
    finally:
        s.close()
    assert (st.cpu().numpy() == 0).all()
    dr, Kr, _ = cref.tiles_backward(tl, mu=0.0, symmetrize=True)
    assert np.isfinite(d.cpu().numpy()).all() and np.isfinite(K.cpu().numpy()).all()
    assert rel(d, dr) < 1e-10 and rel(K, Kr) < 1e-10


def test_tiles_wide_rbd_shape_long_horizon(gpu):
    """The reference RBD caller's shape: nx = 16, nu = 8, T = 1000
    (test/RBD_2_link_example/animate_RBD_2_link.jl:8,19-20)."""
    nb, T, n, m = 3, 1000, 16, 8
    tl = random_tiles(nb, T, n, m, seed=16008)
    s = Solver(n, m, T, nb, kind=_lib.PROBLEM_TILES)
    d, K, st = s.backward_tiles(to_dev(tl))
    assert (st.cpu().numpy() == 0).all()
    dr, Kr, _ = cref.tiles_backward(tl, symmetrize=True)
    assert rel(d, dr) < 1e-10 and rel(K, Kr) < 1e-10
    # a NaN tile is reported per trajectory, as backward_pass.jl:353-354 asserts
    tl["A"][1, 500, 3, 3] = np.nan
    _, _, st = s.backward_tiles(to_dev(tl))
    assert st.cpu().numpy().tolist() == [0, _lib.TRAJ_NAN, 0]
    s.close()


def test_tiles_pendula_vs_oracle(gpu):
    nb, T = 8, 20
    x, u = pendula_batch(nb, T)
    tl = derivative_tiles(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda(),
                          *coupled_pendula(torch_ns()))
    s = Solver(4, 2, T, nb, kind=_lib.PROBLEM_TILES)
    d, K, st = s.backward_tiles(tl)
    assert (st.cpu().numpy() == 0).all()
    dr, Kr, _ = cref.tiles_backward(to_np(tl))
    assert rel(d, dr) < 1e-10 and rel(K, Kr) < 1e-10
    fo, lo, lfo = coupled_pendula(oracle_ns())
    do, Ko = O.backward_pass(x[0], u[0], fo, lo, lfo)
    assert rel(d[0], do) < 1e-10 and rel(K[0], Ko) < 1e-10


def test_tiles_random_time_varying_12x4(gpu):
    """Time-varying A_t, B_t, dense SPD lxx/luu and a non-zero 𝐏 = lux, T = 100."""
    nb, T, n, m = 64, 100, 12, 4
    rng = np.random.default_rng(5)
    A = np.eye(n) + 0.03 * rng.standard_normal((nb, T, n, n))
    Bm = 0.2 * rng.standard_normal((nb, T, n, m))
    Mq = rng.standard_normal((nb, T, n, n))
    lxx = 0.1 * np.einsum("btij,btkj->btik", Mq, Mq) / n + np.eye(n)
    Mr = rng.standard_normal((nb, T, m, m))
    luu = 0.05 * np.einsum("btij,btkj->btik", Mr, Mr) / m + 0.2 * np.eye(m)
    lux = 0.05 * rng.standard_normal((nb, T, m, n))
    Mf = rng.standard_normal((nb, n, n))
    tl = {"A": A, "B": Bm, "lx": rng.standard_normal((nb, T, n)), "lu": rng.standard_normal((nb, T, m)),
          "lxx": lxx, "lux": lux, "luu": luu, "lfx": rng.standard_normal((nb, n)),
          "lfxx": 0.1 * np.einsum("bij,bkj->bik", Mf, Mf) + 2 * np.eye(n)}
    s = Solver(n, m, T, nb, kind=_lib.PROBLEM_TILES)
    d, K, st = s.backward_tiles(to_dev(tl))
    assert (st.cpu().numpy() == 0).all()
    dr, Kr, _ = cref.tiles_backward(tl, symmetrize=True)
    assert rel(d, dr) < 1e-10 and rel(K, Kr) < 1e-10
    # 𝐏 matters: dropping it changes the gains
    tl0 = dict(tl, lux=None)
    d0, _, _ = s.backward_tiles(to_dev(tl0))
    assert rel(d0, dr) > 1e-6


def test_tiles_reproduce_the_fused_lq_kernel(gpu):
    lq, x, u = quadrotor_batch(256, T=100, seed0=7)
    s = Solver(12, 4, 100, 256)
    s.set_problem(lq)
    xd, ud = torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda()
    d_lq, K_lq, _ = s.backward(xd, ud)
    st_ = Solver(12, 4, 100, 256, kind=_lib.PROBLEM_TILES)
    d_t, K_t, _ = st_.backward_tiles(to_dev(lq_tiles(lq, x, u)))
    assert rel(d_t, d_lq) < 1e-12 and rel(K_t, K_lq) < 1e-12


def test_tiles_two_link_torch_closures_vs_fixture(gpu):
    g = np.load(os.path.join(GOLD, "twolink_t50.npz"))
    d, K = api.backward_pass(torch.from_numpy(g["x"]).cuda(), torch.from_numpy(g["u"]).cuda(),
                             *two_link_torch())
    assert rel(d, g["d"]) < 1e-10 and rel(K, g["K"]) < 1e-10


def test_generic_closures_fit_vs_oracle(gpu):
    """iLQR.fit with arbitrary (torch) closures: tiles on the device + HIP Riccati +
    torch rollout, against the oracle's fit with the same closures on duals."""
    nb, T = 2, 20
    x, u = pendula_batch(nb, T, seed=9)
    ft = coupled_pendula(torch_ns())
    xf, uf, info = api.fit(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda(), *ft,
                           max_iter=30, tol=1e-6, return_info=True)
    fo, lo, lfo = coupled_pendula(oracle_ns())
    for b in range(nb):
        h = []
        xo, uo = O.fit(x[b], u[b], fo, lo, lfo, max_iter=30, tol=1e-6, max_trials=64, history=h)
        assert int(info["iters"][b]) == len(h)
        assert rel(xf[b], xo) < 1e-9 and rel(uf[b], uo) < 1e-9


def rbd_batch(nb, T):
    """The reference RBD script's start (animate_RBD_2_link.jl:19-27: rest state, zero
    inputs, x_init = rollout) plus perturbed copies."""
    from closures import jet_ns, rbd_floating_arm, rbd_initial_state
    fj, _, _ = rbd_floating_arm(jet_ns())
    x = np.zeros((nb, T + 1, 16))
    x[:, 0] = rbd_initial_state()
    x[1:, 0, 8:] = 0.05 * np.random.default_rng(7).standard_normal((nb - 1, 8))
    u = np.zeros((nb, T, 8))
    for t in range(T):
        x[:, t + 1] = fj(x[:, t], u[:, t])
    return x, u


def test_rbd_caller_backward_pass_t1000(gpu):
    """iLQR.backward_pass with the RBD example's 16 × 8 closures at T = 1000: tiles by
    torch.func on the device + the wide HIP recursion, against oracle.jet tiles + the C
    recursion."""
    from closures import jet_ns, rbd_cost_quads, rbd_floating_arm, torch_arr_ns
    from oracle import closure_fit as CF
    x, u = rbd_batch(2, 1000)
    u = u + 0.1 * np.random.default_rng(8).standard_normal(u.shape)
    d, K = api.backward_pass(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda(),
                             *rbd_floating_arm(torch_arr_ns()))
    q, fq = rbd_cost_quads()
    tl = CF.derivative_tiles(x, u, rbd_floating_arm(jet_ns())[0], q, fq)
    dr, Kr, st = cref.tiles_backward(tl, symmetrize=True)
    assert (st == 0).all()
    assert rel(d, dr) < 1e-10 and rel(K, Kr) < 1e-10


def test_rbd_caller_fit_t1000(gpu):
    """iLQR.fit on the reference's RBD caller shape (nx = 16, nu = 8, T = 1000) through
    the generic closure path, against the batched closure oracle: iteration counts and
    per-iteration trials exact, iterates and costs within 1e-8."""
    from closures import jet_ns, rbd_cost_quads, rbd_floating_arm, torch_arr_ns
    from oracle import closure_fit as CF
    nb, T, iters = 2, 1000, 4
    x, u = rbd_batch(nb, T)
    xf, uf, info = api.fit(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda(),
                           *rbd_floating_arm(torch_arr_ns()), max_iter=iters, tol=1e-6, return_info=True)
    fj, lj, lfj = rbd_floating_arm(jet_ns())
    r = CF.fit(x, u, fj, lj, lfj, *rbd_cost_quads(), max_iter=iters, tol=1e-6)
    assert info["iters"].tolist() == r["iters"].tolist()
    assert info["status"].tolist() == r["status"].tolist()
    assert info["history"]["trials"][:iters].tolist() == r["history"]["trials"].tolist()
    assert rel(info["cost"], r["cost"]) < 1e-8
    assert rel(xf, r["x"]) < 1e-8 and rel(uf, r["u"]) < 1e-8


def test_closure_path_reuses_one_handle_and_is_thread_safe(gpu):
    """fit with closures keeps one tiles handle per shape between calls (ilqr_amd.cache),
    and two threads fitting DIFFERENT problems of the same shape at once each get their
    own result (the advisor's reentrancy case for the Julia shim, here for the mirror)."""
    import threading
    from ilqr_amd import cache
    api.clear_cache()
    created = []
    orig = Solver.__init__

    def counting(self, *a, **k):
        created.append(a)
        orig(self, *a, **k)
    ft = coupled_pendula(torch_ns())
    xs = [pendula_batch(2, 20, seed=s) for s in (21, 22)]
    ref = [api.fit(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda(), *ft, max_iter=10) for x, u in xs]
    Solver.__init__ = counting
    try:
        for _ in range(3):
            api.fit(torch.from_numpy(xs[0][0]).cuda(), torch.from_numpy(xs[0][1]).cuda(), *ft, max_iter=10)
        assert created == []                        # the cached handle, no new one
        out = [None, None]

        def run(i):
            x, u = xs[i]
            for _ in range(3):
                out[i] = api.fit(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda(), *ft, max_iter=10)
        ths = [threading.Thread(target=run, args=(i,)) for i in range(2)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
    finally:
        Solver.__init__ = orig
    for i in range(2):
        assert torch.equal(out[i][0], ref[i][0]) and torch.equal(out[i][1], ref[i][1])
    # overlapping calls each build a handle of their own; the surplus is closed on check-in
    assert len(created) <= 3 and cache.size() == 1
    api.clear_cache()
    assert cache.size() == 0


def test_tiles_wide_zero_input_equals_narrow(gpu):
    """A (12, 4) problem with a fifth, zero input column runs on the wide kernel: its
    gains for the four real inputs equal the narrow kernel's (other summation order:
    rel 1e-12) and the fifth input's gains are exactly zero (H₅₅ + μ = μ, g₅ = G₅ = 0)."""
    nb, T, n, m = 5, 60, 12, 4   # ragged: the last workgroup holds one trajectory
    tl = random_tiles(nb, T, n, m, seed=77)
    s4 = Solver(n, m, T, nb, kind=_lib.PROBLEM_TILES)
    d4, K4, st4 = s4.backward_tiles(to_dev(tl))
    pad = dict(tl)
    pad["B"] = np.concatenate([tl["B"], np.zeros((nb, T, n, 1))], axis=3)
    pad["lu"] = np.concatenate([tl["lu"], np.zeros((nb, T, 1))], axis=2)
    pad["lux"] = np.concatenate([tl["lux"], np.zeros((nb, T, 1, n))], axis=2)
    luu = np.zeros((nb, T, m + 1, m + 1))
    luu[:, :, :m, :m] = tl["luu"]
    pad["luu"] = luu
    s5 = Solver(n, m + 1, T, nb, kind=_lib.PROBLEM_TILES)
    d5, K5, st5 = s5.backward_tiles(to_dev(pad))
    assert (st4.cpu().numpy() == 0).all() and (st5.cpu().numpy() == 0).all()
    assert rel(d5[..., :m], d4) < 1e-12 and rel(K5[:, :, :m], K4) < 1e-12
    assert (d5[..., m] == 0).all() and (K5[:, :, m] == 0).all()
    s4.close()
    s5.close()


def test_tiles_wide_single_step(gpu):
    """T = 1: the terminal value function and one step (the prefetch clamps at t = 0)."""
    nb, T, n, m = 3, 1, 16, 8
    tl = random_tiles(nb, T, n, m, seed=91)
    s = Solver(n, m, T, nb, kind=_lib.PROBLEM_TILES)
    d, K, st = s.backward_tiles(to_dev(tl))
    dr, Kr, _ = cref.tiles_backward(tl, symmetrize=True)
    assert (st.cpu().numpy() == 0).all() and rel(d, dr) < 1e-12 and rel(K, Kr) < 1e-12
    s.close()


def test_rollout_graph_matches_eager_rbd(gpu):
    """The HIP-graph rollout (one captured forward_pass step replayed T times; the
    reference RBD caller's closure calls torch.linalg.solve, captured as solve_ex) gives
    the eager rollout's trajectories and line-search outcome, and is cached per closure."""
    from closures import rbd_floating_arm, torch_arr_ns
    from ilqr_amd import tiles
    nb, T = 2, 60
    x, u = rbd_batch(nb, T)
    f, l, lf = rbd_floating_arm(torch_arr_ns())
    xb, ub = torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda()
    tl = derivative_tiles(xb, ub, f, l, lf)
    s = Solver(16, 8, T, nb, kind=_lib.PROBLEM_TILES)
    try:
        d, K, _ = s.backward_tiles(tl)
    finally:
        s.close()
    prev = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
    xt = torch.zeros_like(xb)
    old = tiles.ROLLOUT_GRAPHS
    try:
        tiles.ROLLOUT_GRAPHS = False
        e = tiles.rollout_forward(xb, ub, xt, d, K, prev, f, l, lf, 64)
        tiles.ROLLOUT_GRAPHS = True
        g = tiles.rollout_forward(xb, ub, xt, d, K, prev, f, l, lf, 64)
        g2 = tiles.rollout_forward(xb, ub, xt, d, K, prev * 0.0, f, l, lf, 8)   # every trial rejected
        tiles.ROLLOUT_GRAPHS = False
        e2 = tiles.rollout_forward(xb, ub, xt, d, K, prev * 0.0, f, l, lf, 8)
    finally:
        tiles.ROLLOUT_GRAPHS = old
    entry = tiles._GRAPHS[f][(tuple(xb.shape), tuple(ub.shape), xb.dtype, 0)]
    assert entry and entry.graph is not None                     # captured, not the eager fallback
    for a, b in ((g, e), (g2, e2)):
        assert rel(a[0], b[0]) < 1e-12 and rel(a[1], b[1]) < 1e-12 and rel(a[2], b[2]) < 1e-12
        assert a[3].tolist() == b[3].tolist() and a[4].tolist() == b[4].tolist()
    assert g2[3].tolist() == [8, 8] and not bool(g2[4].any())


def test_rollout_graph_falls_back_for_uncapturable_closure(gpu):
    """A closure that synchronises with the host cannot be captured: the rollout runs
    eagerly (still on the device) with the same result, and the closure is remembered."""
    from ilqr_amd import tiles
    ft = coupled_pendula(torch_ns())
    f0 = ft[0]

    def synced(x, u):
        torch.cuda.synchronize()          # a host synchronisation inside the closure
        return f0(x, u)
    x, u = pendula_batch(2, 20, seed=5)
    xf, uf = api.fit(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda(), f0, ft[1], ft[2], max_iter=5)
    xs, us = api.fit(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda(), synced, ft[1], ft[2], max_iter=5)
    assert rel(xs, xf) < 1e-12 and rel(us, uf) < 1e-12
    assert list(tiles._GRAPHS[synced].values()) == [False]
    assert tiles._GRAPHS[f0] and all(v and v.graph is not None for v in tiles._GRAPHS[f0].values())


def test_rollout_graph_follows_a_changed_closure(gpu):
    """A closure that reads Python state (here Δt from a dict, like the reference's
    closures capture globals): after the state changes, the cached graph's replay no
    longer equals the eager step, so forward_pass captures again — the
    result equals the eager rollout with the new state. clear_cache() releases the graphs."""
    from ilqr_amd import tiles
    state = {"dt": 0.05}

    def f(x, u):
        dt = state["dt"]
        return torch.stack([x[0] + dt * x[2], x[1] + dt * x[3],
                            x[2] + dt * (-9.81 * torch.sin(x[0]) + u[0]),
                            x[3] + dt * (-9.81 * torch.sin(x[1]) + u[1])])

    _, l, lf = coupled_pendula(torch_ns())
    x, u = pendula_batch(3, 25, seed=9)
    xb, ub = torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda()
    d = 0.1 * torch.ones_like(ub)
    K = torch.zeros((3, 25, 2, 4), dtype=torch.float64, device="cuda")
    prev = torch.full((3,), float("inf"), dtype=torch.float64, device="cuda")
    old = tiles.ROLLOUT_GRAPHS
    try:
        tiles.ROLLOUT_GRAPHS = True
        g1 = tiles.rollout_forward(xb, ub, None, d, K, prev, f, l, lf, 4)
        state["dt"] = 0.1
        g2 = tiles.rollout_forward(xb, ub, None, d, K, prev, f, l, lf, 4)
        tiles.ROLLOUT_GRAPHS = False
        e2 = tiles.rollout_forward(xb, ub, None, d, K, prev, f, l, lf, 4)
    finally:
        tiles.ROLLOUT_GRAPHS = old
    assert not torch.equal(g1[0], g2[0])
    assert torch.equal(g2[0], e2[0]) and torch.equal(g2[1], e2[1]) and torch.equal(g2[2], e2[2])
    entry = tiles._GRAPHS[f][(tuple(xb.shape), tuple(ub.shape), xb.dtype, 0)]
    assert entry and entry.graph is not None          # captured again, not the eager fallback
    api.clear_cache()
    assert f not in tiles._GRAPHS
