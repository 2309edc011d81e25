"""CPU tests of the generic-closure path: torch.func derivative
tiles against the oracle's ForwardDiff restatement, and the C oracle's tiles
backward against the Python oracle's backward_pass with the same closures."""
import numpy as np
import pytest
import torch

from closures import coupled_pendula, oracle_ns, torch_ns, two_link_torch
from ilqr_amd.tiles import derivative_tiles, rollout_forward, total_cost
from oracle import cref
from oracle import ilqr_oracle as O


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def pendula_batch(nb=3, T=20, seed=0):
    fo, _, _ = coupled_pendula(oracle_ns())
    rng = np.random.default_rng(seed)
    x = np.zeros((nb, T + 1, 4))
    u = 0.3 * rng.standard_normal((nb, T, 2))
    x[:, 0] = rng.uniform(-1, 1, (nb, 4))
    for b in range(nb):
        for t in range(T):
            x[b, t + 1] = np.asarray(fo(x[b, t], u[b, t]), float)
    return x, u


def test_torch_tiles_equal_forwarddiff_restatement():
    x, u = pendula_batch()
    tl = derivative_tiles(torch.from_numpy(x), torch.from_numpy(u), *coupled_pendula(torch_ns()))
    fo, lo, lfo = coupled_pendula(oracle_ns())
    for b, t in ((0, 0), (1, 7), (2, 19)):
        A, B = O.linearize_dynamics(x[b, t], u[b, t], fo)
        _, qv, r, Q, P, R = O.immediate_cost_quadratization(x[b, t], u[b, t], lo)
        for k, ref in (("A", A), ("B", B), ("lx", qv), ("lu", r), ("lxx", Q), ("lux", P), ("luu", R)):
            assert rel(tl[k][b, t], ref) < 1e-14, k
    _, s, S = O.final_cost_quadratization(x[1, -1], lfo)
    assert rel(tl["lfx"][1], s) < 1e-14 and rel(tl["lfxx"][1], S) < 1e-14
    assert float(np.abs(tl["lux"].numpy()).max()) > 0.01  # the cross term is exercised


def test_c_tiles_backward_matches_oracle_backward_pass():
    x, u = pendula_batch()
    tl = derivative_tiles(torch.from_numpy(x), torch.from_numpy(u), *coupled_pendula(torch_ns()))
    d, K, st = cref.tiles_backward({k: v.numpy() for k, v in tl.items()})
    assert (st == 0).all()
    fo, lo, lfo = coupled_pendula(oracle_ns())
    for b in range(x.shape[0]):
        do, Ko = O.backward_pass(x[b], u[b], fo, lo, lfo)
        assert rel(d[b], do) < 1e-12 and rel(K[b], Ko) < 1e-12


def test_two_link_torch_closure_tiles_match_fixture_gains():
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "twolink_t50.npz"))
    tl = derivative_tiles(torch.from_numpy(g["x"]), torch.from_numpy(g["u"]), *two_link_torch())
    d, K, _ = cref.tiles_backward({k: v.numpy() for k, v in tl.items()})
    assert rel(d, g["d"]) < 1e-11 and rel(K, g["K"]) < 1e-11


def test_rollout_forward_matches_oracle_forward_pass():
    x, u = pendula_batch(nb=2, T=15, seed=3)
    fo, lo, lfo = coupled_pendula(oracle_ns())
    ft, lt, lft = coupled_pendula(torch_ns())
    tl = derivative_tiles(torch.from_numpy(x), torch.from_numpy(u), ft, lt, lft)
    d, K, _ = cref.tiles_backward({k: v.numpy() for k, v in tl.items()})
    d = 4.0 * d  # overshoot so the line search halves α at least once
    c0 = np.array([O.total_cost_generator(np.zeros_like(x[b]), lo, lfo)(x[b], u[b]) for b in range(2)])
    T_ = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    xn, un, c, tr, ok = rollout_forward(T_(x), T_(u), None, T_(d), T_(K), T_(c0), ft, lt, lft)
    for b in range(2):
        st = {}
        xo, uo, co = O.forward_pass(x[b], u[b], np.zeros_like(x[b]), d[b], K[b], c0[b], fo, lo, lfo,
                                    max_trials=64, stats=st)
        assert bool(ok[b]) and int(tr[b]) == st["trials"] and st["trials"] > 1
        assert rel(xn[b], xo) < 1e-13 and rel(un[b], uo) < 1e-13 and abs(float(c[b]) - co) < 1e-12 * co
