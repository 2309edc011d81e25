"""The single-process multi-device API (include/ilqr.h ilqr_multi_*) with
device-resident problem and trajectories: ilqr_multi_set_problem / ilqr_multi_load /
ilqr_multi_fit_resident / ilqr_multi_gather, here with every shard on the test box's
one GPU. Trajectories are independent, so each shard's block must equal the same
trajectories solved by one handle over the whole batch, bit for bit (same kernels,
same per-trajectory arithmetic) — the resident path, the host-in/host-out path, warm
starts and the per-iteration history alike."""
import ctypes as C

import numpy as np
import pytest
import torch

from ilqr_amd import _lib
from ilqr_amd.multi import HostBuffers, MultiSolver
from ilqr_amd.problems import quadrotor_batch, two_link_initial_states
from ilqr_amd.solver import Solver, alloc_history

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.as_tensor(np.ascontiguousarray(a)).to("cuda", torch.float64).contiguous()


def one_handle(lq, x, u, iters, history=False, schedule=None):
    s = Solver(12, 4, x.shape[1] - 1, x.shape[0])
    s.set_problem(lq)
    if schedule:
        s.set_schedule(**schedule)
    r = s.fit(dev(x), dev(u), max_iter=iters, tol=-1.0, history=history)
    out = {"x": r.x.cpu().numpy(), "u": r.u.cpu().numpy(), "cost": r.cost.cpu().numpy(),
           "iters": r.iters.cpu().numpy(), "status": r.status.cpu().numpy()}
    h = None if r.history is None else {k: v.cpu().numpy() for k, v in r.history.items()}
    s.close()
    return out, h


@pytest.fixture(scope="module")
def config4():
    return quadrotor_batch(32768, T=100, seed0=0)


def test_resident_equals_one_handle_config4(gpu, config4):
    """BASELINE config 4 (32,768 trajectories in 8 shards): problem and trajectories
    uploaded once, fit on the devices, results gathered into pinned host buffers."""
    lq, x, u = config4
    B = x.shape[0]
    ms = MultiSolver([0] * 8, 12, 4, 100, B)
    hb = HostBuffers(x=(x.shape, np.float64), u=(u.shape, np.float64), cost=((B,), np.float64),
                     iters=((B,), np.int32), status=((B,), np.int32))
    try:
        ms.set_problem(lq)
        ms.load(x, u)
        assert ms.fit_resident(max_iter=3, tol=-1.0) == _lib.OK
        res = ms.gather(out=hb.arrays)
        ref, _ = one_handle(lq, x, u, 3)
        for k in ("x", "u", "cost", "iters", "status"):
            np.testing.assert_array_equal(res[k], ref[k], err_msg=k)
    finally:
        hb.close()
        ms.close()


def test_resident_warm_start_and_history(gpu):
    """fit_resident(warm_start) continues from the previous result (a new fit: prev_cost
    = Inf again, forward_pass.jl:159), equal to one handle's fit from that result; the
    whole-batch history assembled from the shards equals one handle's."""
    B, T = 4096, 50
    lq, x, u = quadrotor_batch(B, T=T, seed0=77)
    sched = {"backward": "block"}  # shards of 1,024 would default to the other kernel
    ms = MultiSolver([0] * 4, 12, 4, T, B)
    try:
        ms.set_schedule(backward="block")
        ms.set_problem(lq)
        ms.load(x, u)
        h, hst = alloc_history(4, B, "cuda")
        ms.fit_resident(max_iter=4, tol=-1.0, history=hst)
        r1 = ms.gather(cost=False, iters=False, status=False)
        ref1, href = one_handle(lq, x, u, 4, history=True, schedule=sched)
        np.testing.assert_array_equal(r1["x"], ref1["x"])
        for k in ("cost", "trials", "alpha", "du2"):
            np.testing.assert_array_equal(h[k].cpu().numpy(), href[k], err_msg=k)
        ms.fit_resident(max_iter=2, tol=-1.0, warm_start=True)
        r2 = ms.gather()
        ref2, _ = one_handle(lq, ref1["x"], ref1["u"], 2, schedule=sched)
        for k in ("x", "u", "cost", "iters", "status"):
            np.testing.assert_array_equal(r2[k], ref2[k], err_msg=k)
    finally:
        ms.close()


def test_resident_history_with_tol_leaves_unrun_rows(gpu):
    """with tol ≥ 0 each shard's fit stops polling at its own last iteration, so
    the rows of the (max_iter, batch) record past it must keep what the caller put there
    (include/ilqr.h: "left as they were"), never the shard scratch's stale contents. Rows a
    trajectory ran equal one handle's record bit for bit; every other entry is either the
    caller's sentinel or the "did not run" marker (trials 0, NaN) one handle writes."""
    B, T, n = 4096, 50, 40
    lq, x, u = quadrotor_batch(B, T=T, seed0=11)

    def filled():
        h, hst = alloc_history(n, B, "cuda")
        h["cost"].fill_(-5.0)
        h["trials"].fill_(-1)
        h["alpha"].fill_(-5.0)
        h["du2"].fill_(-5.0)
        return h, hst

    ms = MultiSolver([0] * 4, 12, 4, T, B)
    try:
        ms.set_schedule(backward="block")
        ms.set_problem(lq)
        for rep in range(2):   # the second fit reuses the shards' scratch from the first
            ms.load(x, u)
            h, hst = filled()
            ms.fit_resident(max_iter=n, tol=1e-6, history=hst)
            hm = {k: v.cpu().numpy() for k, v in h.items()}
    finally:
        ms.close()
    s = Solver(12, 4, T, B)
    s.set_problem(lq)
    s.set_schedule(backward="block")
    h1, hst1 = filled()
    xi, ui = dev(x), dev(u)
    xo, uo = s.alloc_traj(zero=False)
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    s._bind_stream()
    rc = s.lib.ilqr_fit_ex(s.h, s._p(), C.byref(_lib.default_options(max_iter=n, tol=1e-6)), P(xi), P(ui), None,
                           P(xo), P(uo), None, None, None, C.byref(hst1))
    torch.cuda.synchronize()
    s.close()
    assert rc == _lib.OK
    h1 = {k: v.cpu().numpy() for k, v in h1.items()}
    ran = h1["trials"] > 0
    assert ran.any() and (~ran).any()
    for k in ("cost", "trials", "alpha", "du2"):
        np.testing.assert_array_equal(hm[k][ran], h1[k][ran], err_msg=k)
    unrun = ~ran
    assert np.all((hm["trials"][unrun] == -1) | (hm["trials"][unrun] == 0))
    for k in ("cost", "alpha", "du2"):
        v = hm[k][unrun]
        assert np.all((v == -5.0) | np.isnan(v)), k
    assert (hm["trials"] == -1).any()   # some shard stopped before the last row: untouched


def test_host_path_equals_resident(gpu):
    B, T = 2048, 30
    lq, x, u = quadrotor_batch(B, T=T, seed0=5)
    ms = MultiSolver([0] * 2, 12, 4, T, B)
    try:
        xo, uo, co, it, st, rc = ms.fit(lq, x, u, max_iter=3, tol=-1.0)
        ms.fit_resident(max_iter=3, tol=-1.0)  # the host call left problem and trajectories resident
        r = ms.gather()
        np.testing.assert_array_equal(r["x"], xo)
        np.testing.assert_array_equal(r["cost"], co)
    finally:
        ms.close()


def test_resident_two_link(gpu):
    B, T = 512, 50
    x0 = two_link_initial_states(B)
    s = Solver(4, 2, T, B, kind=_lib.PROBLEM_TWO_LINK)
    u = torch.zeros((B, T, 2), dtype=torch.float64, device="cuda")
    x = s.rollout(dev(x0), u)
    r = s.fit(x, u, max_iter=20, tol=1e-6)
    ms = MultiSolver([0] * 2, 4, 2, T, B)
    try:
        ms.set_problem(kind=_lib.PROBLEM_TWO_LINK)
        ms.load(x.cpu().numpy(), u.cpu().numpy())
        ms.fit_resident(max_iter=20, tol=1e-6)
        g = ms.gather()
        np.testing.assert_array_equal(g["x"], r.x.cpu().numpy())
        np.testing.assert_array_equal(g["iters"], r.iters.cpu().numpy())
    finally:
        ms.close()
        s.close()


def test_resident_argument_errors(gpu):
    ms = MultiSolver([0] * 2, 12, 4, 10, 64)
    try:
        with pytest.raises(_lib.IlqrError):
            ms.fit_resident(max_iter=2)           # no problem set
        lq, x, u = quadrotor_batch(64, T=10, seed0=0)
        ms.set_problem(lq)
        with pytest.raises(_lib.IlqrError):
            ms.fit_resident(max_iter=2)           # no trajectories loaded
        with pytest.raises(_lib.IlqrError):
            ms.fit_resident(max_iter=2, warm_start=True)  # no previous result
        with pytest.raises(_lib.IlqrError):
            ms.gather()                           # nothing to gather yet
    finally:
        ms.close()
