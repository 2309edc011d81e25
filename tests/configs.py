"""Oracle checks of every BASELINE.json configuration on the GPU, one function per
config — TEST INFRASTRUCTURE: shared by tests/test_gpu_configs.py (collected first
under `-m gpu`, tests/conftest.py) and __graft_entry__.smoke(), so that one driver
run pins all five configs even when a later test module stops `pytest -x`.

Each check runs the device path through the C ABI (libilqr_hip.so) at the config's
size and compares a sample against the C restatement (oracle/ilqr_ref.c via
oracle.cref), returning {name: relative error}. Tolerances are the ones the config's
own test module states (fp64 rollouts/fits rel 1e-9, costs 1e-11; fp32 central
differences 5e-3), asserted here.

Reference: src/forward_pass.jl:148-179 (fit), :55-93 (forward_pass),
src/backward_pass.jl:324-357 (backward_pass); test/2_link_example/animate_2_link.jl:7-25
(config 1), test/test_iLQR.jl:8 (config 2's rand(4) x₀);
test/RBD_2_link_example/RBD_helper_functions.jl:48-79 (config 5).
"""
from __future__ import annotations

import numpy as np
import torch

from ilqr_amd import _lib
from ilqr_amd.problems import LQBatch, quadrotor_batch, two_link_initial_states
from ilqr_amd.solver import Solver
from oracle import cref

TOL_TRAJ = 1e-9
TOL_COST = 1e-11


def rel(a, b) -> float:
    a = a.cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = b.cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def sub(lq, idx) -> LQBatch:
    return LQBatch(lq.A[idx], lq.B[idx], lq.Q[idx], lq.R[idx], lq.Qf[idx])


def _dev(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a)).to("cuda", dtype).contiguous()


def config1() -> dict:
    """Config 1: the 2-link arm at B = 1, T = 50, x₀ = [.1, −.1, 0, 0], u₀ = 0, x_init the
    rollout of u₀ (animate_2_link.jl:11-16), fit(tol = 1e-6, max_iter = 100) — nu = 1
    (BASELINE's shape, f(x, [u₁, 0])) and nu = 2 (the reference's)."""
    out = {}
    for nu in (1, 2):
        T = 50
        s = Solver(4, nu, T, 1, kind=_lib.PROBLEM_TWO_LINK)
        try:
            x0 = _dev(np.array([[0.1, -0.1, 0.0, 0.0]]))
            u0 = torch.zeros((1, T, nu), dtype=torch.float64, device="cuda")
            x = s.rollout(x0, u0)
            r = s.fit(x, u0, max_iter=100, tol=1e-6)
            xo, uo, co, it, st = cref.tl_fit(x.cpu().numpy(), u0.cpu().numpy(), max_iter=100, tol=1e-6,
                                             symmetrize=True)
        finally:
            s.close()
        assert int(r.status[0]) == int(st[0]) == _lib.TRAJ_CONVERGED, (nu, r.status, st)
        assert int(r.iters[0]) == int(it[0]), (nu, r.iters, it)
        e = max(rel(r.u, uo), rel(r.x, xo))
        assert e < TOL_TRAJ, (nu, e)
        out[f"config1_nu{nu}_fit"] = e
    return out


def config2(sample: int = 64) -> dict:
    """Config 2: the 2-link arm, nu = 1, T = 50, B = 1024 random x₀ (rand(4) seeded per
    trajectory), fit(tol = 1e-6, max_iter = 100) on the device against the C
    restatement's fit on a sample: iterates, costs, iteration counts and status."""
    B, T = 1024, 50
    s = Solver(4, 1, T, B, kind=_lib.PROBLEM_TWO_LINK)
    try:
        u0 = torch.zeros((B, T, 1), dtype=torch.float64, device="cuda")
        x = s.rollout(_dev(two_link_initial_states(B)), u0)
        r = s.fit(x, u0, max_iter=100, tol=1e-6)
        idx = np.arange(0, B, B // sample)
        xo, uo, co, it, st = cref.tl_fit(x.cpu().numpy()[idx], u0.cpu().numpy()[idx], max_iter=100,
                                         tol=1e-6, symmetrize=True)
    finally:
        s.close()
    sts = r.status.cpu().numpy()[idx]
    conv = (sts == _lib.TRAJ_CONVERGED) & (st == _lib.TRAJ_CONVERGED)
    assert conv.mean() > 0.9, (np.unique(sts, return_counts=True), np.unique(st, return_counts=True))
    assert np.array_equal(r.iters.cpu().numpy()[idx][conv], it[conv])
    e = max(rel(r.u.cpu().numpy()[idx][conv], uo[conv]), rel(r.x.cpu().numpy()[idx][conv], xo[conv]))
    ec = rel(r.cost.cpu().numpy()[idx][conv], co[conv])
    assert e < TOL_TRAJ and ec < TOL_TRAJ, (e, ec)
    return {"config2_nu1_fit": e, "config2_nu1_cost": ec}


def config3(sample: int = 64, iters: int = 3) -> dict:
    """Config 3 (the headline, bench.py's timed call): ilqr_fit at B = 4096, T = 100,
    `iters` iterations from cold, tol disabled, the default schedule (lq_iter_fused4)
    — against the restatement's fit (symmetrised step_back) on a sample."""
    B, T = 4096, 100
    lq, x, u = quadrotor_batch(B, T=T, seed0=0)
    s = Solver(12, 4, T, B)
    try:
        s.set_problem(lq)
        r = s.fit(_dev(x), _dev(u), max_iter=iters, tol=-1.0)
    finally:
        s.close()
    assert r.call_status == _lib.OK, r.call_status
    idx = np.sort(np.random.default_rng(42).choice(B, sample, replace=False))
    xo, uo, co, it, st = cref.lq_fit(sub(lq, idx), x[idx], u[idx], max_iter=iters, tol=-1.0,
                                     symmetrize=True)
    assert (r.iters.cpu().numpy()[idx] == it).all() and (r.status.cpu().numpy()[idx] == st).all()
    e = max(rel(r.x.cpu().numpy()[idx], xo), rel(r.u.cpu().numpy()[idx], uo))
    ec = rel(r.cost.cpu().numpy()[idx], co)
    assert e < TOL_TRAJ and ec < TOL_COST, (e, ec)
    return {f"config3_fit{iters}": e, f"config3_cost{iters}": ec}


def config4(shards: int = 8, per_shard: int = 512, iters: int = 3) -> dict:
    """Config 4 (the global batch sharded over 8 GPUs), reduced: `shards` contiguous
    shards through ilqr_multi_fit (one handle and host thread per shard, all on device
    0 here) must equal one handle over the whole batch bit for bit, and the oracle on a
    sample spread over every shard."""
    from ilqr_amd.multi import MultiSolver
    B, T = shards * per_shard, 100
    lq, x, u = quadrotor_batch(B, T=T, seed0=0)
    ms = MultiSolver([0] * shards, 12, 4, T, B)
    try:
        # the four-trajectories-per-wave backward in every shard (a shard below 2,048
        # trajectories would default to the one-per-wave kernel: other rounding)
        ms.set_schedule(backward="block")
        xo, uo, co, it, st, rc = ms.fit(lq, x, u, max_iter=iters, tol=-1.0)
    finally:
        ms.close()
    assert rc == _lib.OK, rc
    s = Solver(12, 4, T, B)
    try:
        s.set_problem(lq)
        s.set_schedule(backward="block")
        r = s.fit(_dev(x), _dev(u), max_iter=iters, tol=-1.0)
        bit_equal = (np.array_equal(xo, r.x.cpu().numpy()) and np.array_equal(uo, r.u.cpu().numpy())
                     and np.array_equal(co, r.cost.cpu().numpy()) and np.array_equal(it, r.iters.cpu().numpy())
                     and np.array_equal(st, r.status.cpu().numpy()))
    finally:
        s.close()
    assert bit_equal, "sharded fit differs from one handle"
    idx = np.concatenate([np.arange(k * per_shard, (k + 1) * per_shard, per_shard // 8) for k in range(shards)])
    xr, ur, cr, itr, str_ = cref.lq_fit(sub(lq, idx), x[idx], u[idx], max_iter=iters, tol=-1.0,
                                        symmetrize=True)
    assert np.array_equal(it[idx], itr) and np.array_equal(st[idx], str_)
    e = max(rel(xo[idx], xr), rel(uo[idx], ur))
    ec = rel(co[idx], cr)
    assert e < TOL_TRAJ and ec < TOL_COST, (e, ec)
    return {f"config4_{shards}shards_fit": e, f"config4_{shards}shards_cost": ec,
            "config4_shards_bit_equal_one_handle": 0.0}


def config5(sample: int = 64) -> dict:
    """Config 5: the fixed-base 2Dof_arm chain, nu = 1, T = 100, B = 2048, fp32, central
    differences (tools/bench_rbd.py's step: one fit iteration from cold) against the C
    restatement (fp64, central differences) on a sample."""
    from ilqr_amd.chain import ChainSolver, rbd_2dof_problem, rbd_initial_states
    pr = rbd_2dof_problem(1)
    B, T = 2048, 100
    s = ChainSolver(pr, T, B, dtype=torch.float32, linearization="fd")
    try:
        u = torch.zeros((B, T, 1), dtype=torch.float32, device="cuda")
        x = s.rollout(torch.from_numpy(rbd_initial_states(B, 2)).to("cuda", torch.float32), u)
        xn, un = torch.empty_like(x), torch.empty_like(u)
        pc = torch.empty((B,), dtype=torch.float32, device="cuda")
        st = torch.zeros((B,), dtype=torch.int32, device="cuda")
        tr = torch.empty((B,), dtype=torch.int32, device="cuda")
        s.iterate(x, u, xn, un, None, st, pc, trials=tr, options=_lib.default_options(tol=-1.0))
        torch.cuda.synchronize()
    finally:
        s.close()
    assert (st.cpu().numpy() == 0).all() and (tr.cpu().numpy() == 1).all()
    idx = np.arange(0, B, B // sample)
    d, K, xo, uo, co, tro = cref.chain_iterate(pr, x[idx].double().cpu().numpy(), u[idx].double().cpu().numpy())
    assert (tro == 1).all()
    e = max(rel(un.cpu().numpy()[idx], uo), rel(xn.cpu().numpy()[idx], xo))
    ec = rel(pc.cpu().numpy()[idx], co)
    assert e < 5e-3 and ec < 5e-3, (e, ec)
    return {"config5_fp32_fd_iteration": e, "config5_fp32_fd_cost": ec}


ALL = (config1, config2, config3, config4, config5)
