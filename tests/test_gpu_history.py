"""fit's per-iteration record (ilqr_fit_ex / ilqr_chain_fit_ex, include/ilqr.h
ilqr_history): what the reference prints on every iteration — `Iteration: i  Total
Cost: new_cost` (src/forward_pass.jl:167) — and the line search's α (:83-85), kept
per trajectory.

* LQ and 2-link fixtures: the history's costs are the oracle fit's per-iteration costs
  (tests/golden/*.npz `fit_cost`, oracle.ilqr_oracle.fit(history=…)), NaN past the
  last iteration, trials > 0 exactly for the iterations run;
* the headline batch: the history equals an ilqr_iterate replay of the same fit
  (costs, trials, Σ(ū − u)² bit for bit) for 5 iterations from cold, with the
  cooperative line search (trials > 1 at the cost floor), α = 0.5^(trials − 1);
* two chunks (B = 32,768: the non-fused schedule, the record behind the side stream);
* the chain family (fp64) against its own iterate replay;
* the mirror's `fit(verbose=True)` prints the reference's line.
"""
import json
import math
import os

import numpy as np
import pytest
import torch

from ilqr_amd import _lib
from ilqr_amd.problems import LQBatch, quadrotor_batch
from ilqr_amd.solver import Solver

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def dev(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a)).to("cuda", dtype).contiguous()


def hist_np(r):
    return {k: v.cpu().numpy() for k, v in r.history.items()}


def check_against_golden(h, g, max_iter):
    nb = g["fit_iters"].shape[0]
    for b in range(nb):
        n = int(g["fit_iters"][b])
        assert (h["trials"][:n, b] > 0).all() and (h["trials"][n:, b] == 0).all(), (b, h["trials"][:, b])
        c = h["cost"][:n, b]
        ref = g["fit_cost"][b, :n]
        assert np.all(np.abs(c - ref) <= 1e-9 * np.abs(ref)), (b, c, ref)
        assert np.isnan(h["cost"][n:, b]).all() and np.isnan(h["du2"][n:, b]).all()
        al = h["alpha"][:n, b]
        assert np.array_equal(al, 0.5 ** (h["trials"][:n, b] - 1.0))


@pytest.mark.parametrize("name", ["quad_t16", "dense_xtraj"])
def test_lq_history_matches_golden(gpu, name):
    g = load(name)
    meta = json.loads(str(g["meta"]))
    lq = LQBatch(g["A"], g["B"], g["Q"], g["R"], g["Qf"])
    s = Solver(lq.nx, lq.nu, g["u"].shape[1], lq.batch)
    s.set_problem(lq)
    xt = dev(g["xtraj"]) if "xtraj" in g else None
    r = s.fit(dev(g["x"]), dev(g["u"]), x_traj=xt, max_iter=meta["fit_max_iter"], tol=meta["tol"], history=True)
    s.close()
    h = hist_np(r)
    assert h["cost"].shape == (meta["fit_max_iter"], lq.batch)
    check_against_golden(h, g, meta["fit_max_iter"])


@pytest.mark.parametrize("name,nu", [("twolink_t50", 2), ("twolink_nu1_t50", 1)])
def test_two_link_history_matches_golden(gpu, name, nu):
    g = load(name)
    meta = json.loads(str(g["meta"]))
    nb, T = g["u"].shape[:2]
    s = Solver(4, nu, T, nb, kind=_lib.PROBLEM_TWO_LINK)
    r = s.fit(dev(g["x"]), dev(g["u"]), max_iter=meta["fit_max_iter"], tol=meta["tol"], history=True)
    s.close()
    check_against_golden(hist_np(r), g, meta["fit_max_iter"])


def replay(s, x, u, iters, nb):
    """fit's iterations as chained ilqr_iterate calls: per iteration (cost, trials, du2)
    of the trajectories still running, exhausted / NaN ones keeping their iterate."""
    xi, ui = dev(x), dev(u)
    xn, un = torch.empty_like(xi), torch.empty_like(ui)
    pc = torch.empty((nb,), dtype=torch.float64, device="cuda")
    st = torch.zeros((nb,), dtype=torch.int32, device="cuda")
    tr = torch.zeros((nb,), dtype=torch.int32, device="cuda")
    du2 = torch.zeros((nb,), dtype=torch.float64, device="cuda")
    out = []
    for it in range(iters):
        s.iterate(xi, ui, xn, un, None if it == 0 else pc, st, du2=du2, trials=tr,
                  options=_lib.default_options(tol=-1.0), new_cost=pc)
        torch.cuda.synchronize()
        stn = st.cpu().numpy()
        ran = np.ones(nb, bool) if it == 0 else prev_running
        acc = ran & (stn == _lib.TRAJ_OK)
        out.append((np.where(acc, pc.cpu().numpy(), np.nan), np.where(ran, tr.cpu().numpy(), 0),
                    np.where(ran, du2.cpu().numpy(), np.nan)))
        prev_running = ran & (stn == _lib.TRAJ_OK)
        keep = torch.from_numpy(stn != _lib.TRAJ_OK).cuda()
        xn[keep] = xi[keep]
        un[keep] = ui[keep]
        xi, xn, ui, un = xn, xi, un, ui
    return out


def test_headline_history_equals_iterate_replay(gpu):
    nb, iters = 4096, 5
    lq, x, u = quadrotor_batch(nb, T=100, seed0=0)
    s = Solver(12, 4, 100, nb)
    s.set_problem(lq)
    try:
        r = s.fit(dev(x), dev(u), max_iter=iters, tol=-1.0, history=True)
        h = hist_np(r)
        ref = replay(s, x, u, iters, nb)
    finally:
        s.close()
    for i, (c, t, d) in enumerate(ref):
        np.testing.assert_array_equal(h["trials"][i], t, err_msg=f"trials, iteration {i + 1}")
        np.testing.assert_array_equal(h["cost"][i], c, err_msg=f"cost, iteration {i + 1}")
        np.testing.assert_array_equal(h["du2"][i], d, err_msg=f"du2, iteration {i + 1}")
    assert (h["trials"][-1] > 1).any()  # the cost floor: searches past trial 1
    ok = ~np.isnan(h["cost"])
    assert np.array_equal(h["alpha"][ok], 0.5 ** (h["trials"][ok] - 1.0))


def test_two_chunk_history(gpu):
    """B = 32,768 on one handle runs two chunks (backward of one overlapping the
    forward of the other, the record behind both): the history is the replay's."""
    nb, T, iters = 32768, 12, 4
    lq, x, u = quadrotor_batch(nb, T=T, seed0=0)
    s = Solver(12, 4, T, nb)
    s.set_problem(lq)
    try:
        r = s.fit(dev(x), dev(u), max_iter=iters, tol=-1.0, history=True)
        h = hist_np(r)
        ref = replay(s, x, u, iters, nb)
    finally:
        s.close()
    for i, (c, t, d) in enumerate(ref):
        np.testing.assert_array_equal(h["trials"][i], t)
        np.testing.assert_array_equal(h["cost"][i], c)


def test_chain_history_equals_iterate_replay(gpu):
    from ilqr_amd.chain import ChainSolver, rbd_2dof_problem, rbd_initial_states
    pr = rbd_2dof_problem(2)
    nb, T, iters = 64, 40, 6
    s = ChainSolver(pr, T, nb, dtype=torch.float64)
    try:
        u0 = torch.zeros((nb, T, 2), dtype=torch.float64, device="cuda")
        x0 = s.rollout(dev(rbd_initial_states(nb, 2)), u0)
        r = s.fit(x0, u0, max_iter=iters, tol=-1.0, history=True)
        h = hist_np(r)
        xi, ui = x0.clone(), u0.clone()
        xn, un = torch.empty_like(xi), torch.empty_like(ui)
        pc = torch.empty((nb,), dtype=torch.float64, device="cuda")
        st = torch.zeros((nb,), dtype=torch.int32, device="cuda")
        tr = torch.zeros((nb,), dtype=torch.int32, device="cuda")
        for it in range(iters):
            s.iterate(xi, ui, xn, un, None if it == 0 else pc, st, pc, trials=tr,
                      options=_lib.default_options(tol=-1.0))
            torch.cuda.synchronize()
            stn = st.cpu().numpy()
            run = stn == _lib.TRAJ_OK
            np.testing.assert_array_equal(np.where(run, pc.cpu().numpy(), np.nan)[run], h["cost"][it][run])
            np.testing.assert_array_equal(tr.cpu().numpy()[run], h["trials"][it][run])
            if not run.all():
                break
            xi, xn, ui, un = xn, xi, un, ui
    finally:
        s.close()


def test_mirror_fit_verbose_prints_reference_lines(gpu, capsys):
    """ilqr_amd.fit(..., verbose=True) prints forward_pass.jl:167's line per iteration."""
    import ilqr_amd
    from ilqr_amd.problems import two_link_closures
    g = load("twolink_t50")
    f, l, lf = two_link_closures(2)
    xf, uf, info = ilqr_amd.fit(g["x"][0], g["u"][0], f, l, lf, max_iter=40, tol=1e-6, verbose=True,
                                return_info=True)
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("Iteration: ")]
    n = int(g["fit_iters"][0])
    assert len(lines) == n
    for i, ln in enumerate(lines):
        head, cost = ln.split("\t\tTotal Cost: ")
        assert head == f"Iteration: {i + 1}"
        assert math.isclose(float(cost), g["fit_cost"][0, i], rel_tol=1e-9)
    assert info["history"]["trials"].shape == (40, 1)
