"""The fused LQ iteration's cooperative line search (ilqr_fwd_ring.h lq_coop_search,
DESIGN.md §4 "line-search tail") against the sequential search it replaces
(ILQR_SCHED_SEQUENTIAL_SEARCH: forward_pass.jl:70-87 trial after trial, capped at
max_trials) — bit for bit: x̄, ū (the LAST trial's rollout for an exhausted search),
new cost, Σ(ū − u)², trial count and status — and against the oracle.

Workloads:
* "forced": one iteration from the cold-start iterate with a line-search objective
  offset by a random x_traj per trajectory (the backward ignores x_traj, so its step is
  not the objective's: forward_pass.jl:67 / backward_pass.jl:324 — the reference's own
  quirk) and prev_cost = the input's cost. Trials spread over 1..64 and exhaustion
  (the C oracle on 512 of these: 84 accept at trial 1, most others at 28-51, 230
  exhaust);
* the headline fit, 5 iterations from cold with tol disabled (SURVEY §8d's protocol),
  whose iterations 4-5 sit at the fp64 cost floor;
* batches that are not co-resident (B = 8192: 512 workgroups on 256 CUs — idle waves
  do not wait) and ragged ones, max_trials 2, 7, 64, and 65 (the sequential search).
"""
import numpy as np
import pytest
import torch

from ilqr_amd import _lib
from ilqr_amd.problems import LQBatch, quadrotor_batch
from ilqr_amd.solver import Solver
from oracle import cref

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.as_tensor(np.ascontiguousarray(a)).to("cuda", torch.float64).contiguous()


def lq_cost(lq, x, u, xt):
    """total_cost (forward_pass.jl:185-193) of (x, u) against x_traj, numpy"""
    e = x - xt
    return (np.einsum("bti,bij,btj->b", e[:, :-1], lq.Q, e[:, :-1]) + np.einsum("bti,bij,btj->b", u, lq.R, u)
            + np.einsum("bi,bij,bj->b", x[:, -1], lq.Qf, x[:, -1]))


def forced_case(nb, T=100, seed=5):
    lq, x, u = quadrotor_batch(nb, T=T, seed0=0)
    d, K, _ = cref.lq_backward(lq, x, u, symmetrize=True)
    x1, u1, _, _ = cref.lq_forward(lq, x, u, None, d, K, np.inf)
    rng = np.random.default_rng(seed)
    scale = 10.0 ** rng.uniform(-3, 1, nb)
    xt = x1 + scale[:, None, None] * rng.standard_normal(x1.shape)
    return lq, x1, u1, xt, lq_cost(lq, x1, u1, xt)


def run_iterate(s, x, u, xt, pc, sequential, max_trials=64):
    s.set_schedule(backward="block", sequential_search=sequential)
    nb = x.shape[0]
    xi, ui = dev(x), dev(u)
    xn = torch.full_like(xi, -7.0)
    un = torch.full_like(ui, -7.0)
    prev = dev(pc)
    cost = torch.full((nb,), -7.0, dtype=torch.float64, device="cuda")
    du2 = torch.full((nb,), -7.0, dtype=torch.float64, device="cuda")
    st = torch.zeros((nb,), dtype=torch.int32, device="cuda")
    tr = torch.zeros((nb,), dtype=torch.int32, device="cuda")
    s.iterate(xi, ui, xn, un, prev, st, du2=du2, trials=tr, x_traj=dev(xt),
              options=_lib.default_options(tol=-1.0, max_trials=max_trials), new_cost=cost)
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in (xn, un, cost, du2, st, tr)]


def assert_same(a, b):
    for name, p, q in zip(("x_new", "u_new", "new_cost", "du2", "status", "trials"), a, b):
        np.testing.assert_array_equal(p, q, err_msg=name)


@pytest.mark.parametrize("nb", [4096, 8192, 37])
def test_coop_equals_sequential_forced(gpu, nb):
    lq, x, u, xt, pc = forced_case(nb)
    s = Solver(12, 4, 100, nb)
    s.set_problem(lq)
    try:
        seq = run_iterate(s, x, u, xt, pc, True)
        coop = run_iterate(s, x, u, xt, pc, False)
    finally:
        s.close()
    tr, st = seq[5], seq[4]
    # the workload really spreads the searches
    assert (tr == 1).any() and ((tr > 4) & (st == _lib.TRAJ_OK)).any()
    if nb >= 512:
        assert (st == _lib.TRAJ_LS_EXHAUSTED).sum() > nb // 10, np.bincount(tr)
    assert_same(coop, seq)


@pytest.mark.parametrize("nb", [4096, 8192])
def test_coop_timeout_exit_variant(gpu, nb):
    """The cooperative search's timeout exit (lq_coop_search: a wave that finds no work but
    a reserved, not yet written list slot waits at most WAIT_TICKS, then leaves) taken at
    every such sighting: the test build libilqr_hip_wait0.so (ILQR_COOP_WAIT_TICKS = 0,
    csrc/Makefile `variants`) must still give the sequential search's bits — correctness
    rests only on every publisher finding its own entries, not on the wait."""
    lq, x, u, xt, pc = forced_case(nb)
    seq_s = Solver(12, 4, 100, nb)
    seq_s.set_problem(lq)
    var = Solver(12, 4, 100, nb, lib_path=_lib.WAIT0_LIB_PATH)
    var.set_problem(lq)
    try:
        seq = run_iterate(seq_s, x, u, xt, pc, True)
        coop = run_iterate(var, x, u, xt, pc, False)
        coop2 = run_iterate(var, x, u, xt, pc, False)   # and again on the re-armed list
    finally:
        seq_s.close()
        var.close()
    assert (seq[4] == _lib.TRAJ_LS_EXHAUSTED).sum() > nb // 10
    assert_same(coop, seq)
    assert_same(coop2, seq)


def test_coop_sequential_coop_on_one_handle(gpu):
    """coop → sequential → coop launches on ONE handle (a sequential launch
    must not advance the list generation, or the next cooperative launch counts in a
    half nobody zeroed): all three bit-equal, over the forced workload's many publications."""
    nb = 4096
    lq, x, u, xt, pc = forced_case(nb)
    s = Solver(12, 4, 100, nb)
    s.set_problem(lq)
    try:
        a = run_iterate(s, x, u, xt, pc, False)
        b = run_iterate(s, x, u, xt, pc, True)
        c = run_iterate(s, x, u, xt, pc, False)
        d = run_iterate(s, x, u, xt, pc, True)
        e = run_iterate(s, x, u, xt, pc, False)
    finally:
        s.close()
    for r in (a, c, d, e):
        assert_same(r, b)


@pytest.mark.parametrize("max_trials", [2, 7, 64, 65])
def test_coop_equals_sequential_max_trials(gpu, max_trials):
    nb = 2048
    lq, x, u, xt, pc = forced_case(nb, T=40, seed=9)
    s = Solver(12, 4, 40, nb)
    s.set_problem(lq)
    try:
        seq = run_iterate(s, x, u, xt, pc, True, max_trials)
        coop = run_iterate(s, x, u, xt, pc, False, max_trials)
    finally:
        s.close()
    assert (seq[5] <= max_trials).all()
    assert_same(coop, seq)


def test_coop_nan_and_unreachable(gpu):
    """A NaN trajectory (status NAN after its search) and unreachable costs (prev_cost
    = −1: every trial rejected, the search ends at the first trial whose α·δu vanished
    or at max_trials) beside ordinary ones."""
    nb = 4096
    lq, x, u, xt, pc = forced_case(nb)
    pc[::7] = -1.0
    x, u, xt = x.copy(), u.copy(), xt.copy()
    x[5, 3, 2] = np.nan
    # trajectory 9 at rest on its target: gradient and δu exactly 0, so α·δu vanishes at
    # trial 1 itself (the published `stop` is clamped to 2: trial 2 repeats trial 1)
    x[9], u[9], xt[9], pc[9] = 0.0, 0.0, 0.0, -1.0
    s = Solver(12, 4, 100, nb)
    s.set_problem(lq)
    try:
        seq = run_iterate(s, x, u, xt, pc, True)
        coop = run_iterate(s, x, u, xt, pc, False)
    finally:
        s.close()
    assert seq[4][5] == _lib.TRAJ_NAN
    assert (seq[4][::7][1:] == _lib.TRAJ_LS_EXHAUSTED).all() and (seq[5][::7][1:] == 64).all()
    assert seq[4][9] == _lib.TRAJ_LS_EXHAUSTED and seq[5][9] == 64
    assert_same(coop, seq)


def test_coop_forced_vs_oracle(gpu):
    """The cooperative search against the C restatement's sequential forward_pass on a
    sample, with prev_cost placed so that every accept/reject decision is far above
    rounding (the forced workload's own small-α decisions sit at the fp64 cost floor,
    where the two summation orders legitimately disagree): from the oracle's cost of
    each trial j = 1..48, a target trial j* drawn up to argmin_j c_j and prev_cost
    halfway between c_j* and min_{i<j*} c_i; every 5th trajectory gets an unreachable
    prev_cost.
    Trial counts and status exactly, rollouts and costs to rounding."""
    nb, J = 4096, 48
    lq, x, u, xt, _ = forced_case(nb)
    idx = np.arange(0, nb, 16)
    sl = LQBatch(lq.A[idx], lq.B[idx], lq.Q[idx], lq.R[idx], lq.Qf[idx])
    d, K, _ = cref.lq_backward(sl, x[idx], u[idx], symmetrize=True)
    cj = np.stack([cref.lq_forward(sl, x[idx], u[idx], xt[idx], d, K, -np.inf, max_trials=j)[2]
                   for j in range(1, J + 1)], 1)                     # (sample, J): trial j's cost
    # costs fall trial by trial down to argmin_j c_j (α halving towards the objective's
    # minimiser): any target j* up to there is the first trial below a threshold set
    # between c_j* and c_{j*-1}
    jm = np.argmin(cj, 1)
    js = (np.random.default_rng(3).random(len(idx)) * (jm + 1)).astype(int)  # 0-based target trial
    before = np.array([cj[k, :js[k]].min() if js[k] > 0 else np.inf for k in range(len(idx))])
    pc_s = np.where(js > 0, 0.5 * (cj[np.arange(len(idx)), js] + before),
                    cj[:, 0] + 1e-6 * np.abs(cj[:, 0]))
    robust = (before - cj[np.arange(len(idx)), js]) > 1e-8 * np.abs(before)
    robust |= js == 0
    unreach = np.arange(len(idx)) % 5 == 0
    pc_s = np.where(unreach, cj.min(1) - 1e-3 * np.abs(cj.min(1)), pc_s)
    pc = np.full(nb, np.inf)
    pc[idx] = pc_s
    s = Solver(12, 4, 100, nb)
    s.set_problem(lq)
    try:
        xn, un, cost, du2, st, tr = run_iterate(s, x, u, xt, pc, False)
    finally:
        s.close()
    xo, uo, co, tro = cref.lq_forward(sl, x[idx], u[idx], xt[idx], d, K, pc_s)
    keep = robust | unreach
    assert keep.sum() > 0.5 * len(idx) and len(np.unique(tro[keep & ~unreach])) > 8, np.unique(tro)
    acc = (tro > 0) & keep
    np.testing.assert_array_equal(np.where(tro > 0, tro, 64)[keep], tr[idx][keep])
    np.testing.assert_array_equal(np.where(tro > 0, _lib.TRAJ_OK, _lib.TRAJ_LS_EXHAUSTED)[keep], st[idx][keep])
    assert (st[idx][unreach] == _lib.TRAJ_LS_EXHAUSTED).all()
    rel = lambda a, b: float(np.abs(a - b).max() / np.abs(b).max())
    assert rel(un[idx][acc], uo[acc]) < 1e-9 and rel(xn[idx][acc], xo[acc]) < 1e-9
    assert rel(cost[idx][acc], co[acc]) < 1e-11


def test_fit5_headline_coop_equals_sequential(gpu):
    """SURVEY §8d's protocol: fit, 5 iterations from cold, tol disabled, at the headline
    batch — iterations 4-5 at the fp64 cost floor, where searches run long or exhaust."""
    lq, x, u = quadrotor_batch(4096, T=100, seed0=0)
    s = Solver(12, 4, 100, 4096)
    s.set_problem(lq)
    outs = []
    try:
        for sequential in (True, False):
            s.set_schedule(backward="block", sequential_search=sequential)
            r = s.fit(dev(x), dev(u), max_iter=5, tol=-1.0)
            outs.append([t.cpu().numpy() for t in (r.x, r.u, r.cost, r.iters, r.status)] + [r.call_status])
    finally:
        s.close()
    for name, p, q in zip(("x", "u", "cost", "iters", "status", "call_status"), *outs):
        np.testing.assert_array_equal(p, q, err_msg=name)


def test_coop_iterations_at_floor_equal_sequential(gpu):
    """The bench's chained iterations (ilqr_iterate, prev_cost in place) for 6
    iterations from cold: every iteration's outputs bit-equal to the sequential
    search's, trial counts included."""
    nb = 4096
    lq, x, u = quadrotor_batch(nb, T=100, seed0=0)
    s = Solver(12, 4, 100, nb)
    s.set_problem(lq)
    res = {}
    try:
        for sequential in (True, False):
            s.set_schedule(backward="block", sequential_search=sequential)
            xi, ui = dev(x), dev(u)
            xn, un = torch.empty_like(xi), torch.empty_like(ui)
            pc = torch.empty((nb,), dtype=torch.float64, device="cuda")
            st = torch.zeros((nb,), dtype=torch.int32, device="cuda")
            tr = torch.zeros((nb,), dtype=torch.int32, device="cuda")
            hist = []
            for it in range(6):
                s.iterate(xi, ui, xn, un, None if it == 0 else pc, st, trials=tr,
                          options=_lib.default_options(tol=-1.0), new_cost=pc)
                torch.cuda.synchronize()
                hist.append([t.cpu().numpy().copy() for t in (xn, un, pc, st, tr)])
                # exhausted / NaN trajectories keep their iterate (fit's rule) and rejoin
                keep = (st != _lib.TRAJ_OK)
                xn[keep] = xi[keep]
                un[keep] = ui[keep]
                st.zero_()
                xi, xn, ui, un = xn, xi, un, ui
            res[sequential] = hist
    finally:
        s.close()
    for it, (a, b) in enumerate(zip(res[True], res[False])):
        for name, p, q in zip(("x_new", "u_new", "cost", "status", "trials"), a, b):
            np.testing.assert_array_equal(p, q, err_msg=f"iteration {it + 1}: {name}")
    assert (res[True][-1][4] > 1).any()  # the floor reached: searches beyond trial 1
