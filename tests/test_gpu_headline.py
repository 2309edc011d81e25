"""Oracle parity of exactly what bench.py times, at the headline size, and of the
BASELINE.json configurations that need more than one GPU's batch.

* The bench step: `ilqr_fit` for 3 iterations from cold with tol disabled, whose
  iterations are `ilqr_iterate` (lq_iter_backward4 + lq_iter_forward_ring) at
  B = 4096, T = 100 — checked iteration by iteration against the C restatement of
  backward_pass.jl:324-357 + forward_pass.jl:55-93 (oracle/ilqr_ref.c, symmetrised
  step_back) chained the same way on 256 sampled trajectories, and as
  a whole against the restatement's fit (forward_pass.jl:148-179).
* Config 4 (32,768 trajectories sharded over 8 GPUs): the single-process multi-GPU
  fit with 8 shards on the one GPU of the test box — the shards' results must equal
  one handle's bit for bit (trajectories are independent) and match the oracle on a
  sample. The one-process-per-GPU path (bench.py under torch.distributed) shards the
  same way (ilqr_amd.dist, tests/test_dist.py).

Tolerances (fp64): trajectories rel 1e-9 of max|·| over the sample (gains agree to
1e-11, tests/test_gpu_parity.py), costs rel 1e-11, line-search trial counts and
iteration counts exactly — while the cost decrease is far above rounding. Iterations
4-5 of the headline instances reach the fp64 cost floor (relative decrease ~1e-15),
where the accept/reject decision of forward_pass.jl:77-80 is decided by rounding: there
both sides must end on the same fixed point (costs rel 1e-11), trial counts may differ.
"""
import numpy as np
import pytest
import torch

from ilqr_amd import _lib
from ilqr_amd.problems import LQBatch, quadrotor_batch
from ilqr_amd.solver import Solver
from oracle import cref

pytestmark = pytest.mark.gpu

TOL_TRAJ = 1e-9
TOL_COST = 1e-11
FIT_ITERS = 3
SAMPLE = 256


def rel(a, b):
    a = a.cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = b.cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def sub(lq, idx):
    return LQBatch(lq.A[idx], lq.B[idx], lq.Q[idx], lq.R[idx], lq.Qf[idx])


@pytest.fixture(scope="module")
def headline():
    lq, x, u = quadrotor_batch(4096, T=100, seed0=0)
    s = Solver(12, 4, 100, 4096)
    s.set_problem(lq)
    idx = np.sort(np.random.default_rng(42).choice(4096, SAMPLE, replace=False))
    yield s, lq, x, u, idx
    s.close()


@pytest.mark.parametrize("forward_mfma", [False, True])
def test_bench_step_iterations_vs_oracle(gpu, headline, forward_mfma):
    """The chained iterations of the bench's fit, each against the oracle's; then two
    more at the fp64 floor. Both forms of the forward (DPP rows, 4-block MFMA)."""
    s, lq, x, u, idx = headline
    s.set_schedule(forward_mfma=forward_mfma)
    xi, ui = torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda()
    xn, un = torch.empty_like(xi), torch.empty_like(ui)
    pc = torch.empty((4096,), dtype=torch.float64, device="cuda")
    st = torch.zeros((4096,), dtype=torch.int32, device="cuda")
    tr = torch.empty((4096,), dtype=torch.int32, device="cuda")
    o = _lib.default_options(tol=-1.0)
    ls = sub(lq, idx)
    xo, uo, prev = x[idx], u[idx], np.inf
    for it in range(FIT_ITERS + 2):
        s.iterate(xi, ui, xn, un, None if it == 0 else pc, st, trials=tr, options=o, new_cost=pc)
        torch.cuda.synchronize()
        d, K, _ = cref.lq_backward(ls, xo, uo, symmetrize=True)
        xo2, uo2, co, tro = cref.lq_forward(ls, xo, uo, None, d, K, prev)
        if it >= FIT_ITERS:
            # at the floor: an exhausted search keeps the input iterate (and its cost)
            stn = st.cpu().numpy()[idx]
            gpu_cost = np.where(stn == _lib.TRAJ_OK, pc.cpu().numpy()[idx], prev)
            ora_cost = np.where(tro > 0, co, prev)
            assert rel(gpu_cost, ora_cost) < TOL_COST, (it, rel(gpu_cost, ora_cost))
            assert (np.abs(prev - ora_cost) <= 1e-9 * prev).all()  # really the floor
            xo, uo = np.where((tro > 0)[:, None, None], xo2, xo), np.where((tro > 0)[:, None, None], uo2, uo)
            prev = ora_cost
            xi, xn, ui, un = xn, xi, un, ui
            continue
        xo, uo = xo2, uo2
        assert (st.cpu().numpy() == _lib.TRAJ_OK).all(), it
        assert (tro > 0).all()
        np.testing.assert_array_equal(tr.cpu().numpy()[idx], tro, err_msg=f"trials, iteration {it + 1}")
        assert rel(xn.cpu().numpy()[idx], xo) < TOL_TRAJ, (it, rel(xn.cpu().numpy()[idx], xo))
        assert rel(un.cpu().numpy()[idx], uo) < TOL_TRAJ, (it, rel(un.cpu().numpy()[idx], uo))
        assert rel(pc.cpu().numpy()[idx], co) < TOL_COST, (it, rel(pc.cpu().numpy()[idx], co))
        if it > 0:
            assert (co < prev).all()  # @assert(prev_cost > new_cost), forward_pass.jl:168
        prev = co
        xi, xn, ui, un = xn, xi, un, ui


@pytest.mark.parametrize("forward_mfma", [False, True])
def test_bench_fit_vs_oracle_fit(gpu, headline, forward_mfma):
    """ilqr_fit(max_iter = 3, tol < 0) — the bench's timed call — against the
    restatement's fit on the sample: result, cost, iteration count, status."""
    s, lq, x, u, idx = headline
    s.set_schedule(forward_mfma=forward_mfma)
    r = s.fit(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda(), max_iter=FIT_ITERS, tol=-1.0)
    assert r.call_status == _lib.OK
    xo, uo, co, it, st = cref.lq_fit(sub(lq, idx), x[idx], u[idx], max_iter=FIT_ITERS, tol=-1.0,
                                     symmetrize=True)
    assert (r.iters.cpu().numpy() == FIT_ITERS).all() and (it == FIT_ITERS).all()
    assert (r.status.cpu().numpy() == _lib.TRAJ_MAX_ITER).all() and (st == _lib.TRAJ_MAX_ITER).all()
    assert rel(r.x.cpu().numpy()[idx], xo) < TOL_TRAJ and rel(r.u.cpu().numpy()[idx], uo) < TOL_TRAJ
    assert rel(r.cost.cpu().numpy()[idx], co) < TOL_COST


@pytest.fixture(scope="module")
def config4():
    lq, x, u = quadrotor_batch(32768, T=100, seed0=0)
    return lq, x, u


def test_config4_global_batch_eight_shards(gpu, config4):
    """BASELINE.json config 4: the 32,768-trajectory global batch split into 8
    contiguous shards of 4,096 (one handle and host thread per shard, here all on
    device 0), equal to one handle over the whole batch bit for bit, and to the
    oracle on a sample spread over every shard."""
    from ilqr_amd.multi import MultiSolver
    lq, x, u = config4
    ms = MultiSolver([0] * 8, 12, 4, 100, 32768)
    try:
        xo, uo, co, it, st, rc = ms.fit(lq, x, u, max_iter=FIT_ITERS, tol=-1.0)
    finally:
        ms.close()
    assert rc == _lib.OK
    s = Solver(12, 4, 100, 32768)
    s.set_problem(lq)
    try:
        r = s.fit(torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda(), max_iter=FIT_ITERS, tol=-1.0)
        np.testing.assert_array_equal(xo, r.x.cpu().numpy())
        np.testing.assert_array_equal(uo, r.u.cpu().numpy())
        np.testing.assert_array_equal(co, r.cost.cpu().numpy())
        np.testing.assert_array_equal(it, r.iters.cpu().numpy())
        np.testing.assert_array_equal(st, r.status.cpu().numpy())
    finally:
        s.close()
    idx = np.concatenate([np.arange(k * 4096, k * 4096 + 4096, 128) for k in range(8)])
    xr, ur, cr, itr, str_ = cref.lq_fit(sub(lq, idx), x[idx], u[idx], max_iter=FIT_ITERS, tol=-1.0,
                                        symmetrize=True)
    assert np.array_equal(it[idx], itr) and np.array_equal(st[idx], str_)
    assert rel(xo[idx], xr) < TOL_TRAJ and rel(uo[idx], ur) < TOL_TRAJ and rel(co[idx], cr) < TOL_COST


def test_config4_shards_equal_independent_instances(gpu, config4):
    """What one rank of the 8-process run computes (its own 4,096 instances, seeds
    rank·4096 + i, bench.py) is the corresponding block of the global batch."""
    lq, x, u = config4
    r7 = 7
    lq7, x7, u7 = quadrotor_batch(4096, T=100, seed0=r7 * 4096)
    assert np.array_equal(lq7.A, lq.A[r7 * 4096:]) and np.array_equal(x7, x[r7 * 4096:])
    s = Solver(12, 4, 100, 4096)
    s.set_problem(lq7)
    r = s.fit(torch.from_numpy(x7).cuda(), torch.from_numpy(u7).cuda(), max_iter=2, tol=-1.0)
    idx = np.arange(0, 4096, 64)
    xr, ur, cr, itr, _ = cref.lq_fit(sub(lq7, idx), x7[idx], u7[idx], max_iter=2, tol=-1.0, symmetrize=True)
    assert rel(r.u.cpu().numpy()[idx], ur) < TOL_TRAJ and rel(r.cost.cpu().numpy()[idx], cr) < TOL_COST
    s.close()


def test_bench_two_ranks_gloo(gpu):
    """`bench.py --gpus 2` without a launcher spawns its two rank processes (here both on
    the box's one GPU, gloo in place of RCCL): one JSON line, n_gpus = 2, the per-trajectory
    cost all-gather holding both ranks' batches, every gathered cost finite."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["ILQR_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "6",
                        "--warmup", "3", "--settle", "0.1", "--batch", "512", "--no-cpu", "--no-secondary"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 1024
    assert out["allgather_check"]["trajectories"] == 1024 and out["allgather_check"]["finite_costs"] == 1024
    assert out["value"] > 0 and out["iteration"]["all_ok"]
