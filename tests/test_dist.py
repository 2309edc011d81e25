"""CPU multi-process tests (gloo, world_size 2) of the sharded path: each rank fits
its contiguous block of trajectories, then the per-trajectory costs/status are
all-gathered; the result must equal a single-process fit of the whole batch.
The per-rank solver here is the C restatement (CPU); on GPUs bench.py runs the
same sharding and gather over RCCL with the HIP solver."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from ilqr_amd.dist import all_gather_ragged, gather_fit_results, shard_range
from ilqr_amd.problems import quadrotor_batch


def test_shard_range_covers_batch():
    for n in (1, 7, 4096, 32768, 32771):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import torch.distributed as dist
    from oracle import cref
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lq, x, u = quadrotor_batch(n, T=12, seed0=0)
    lo, hi = shard_range(n, rank, world)
    sub = lq.slice(lo, hi)
    _, _, cost, iters, st = cref.lq_fit(sub, x[lo:hi], u[lo:hi], max_iter=20, tol=1e-6, nthreads=1)
    gc, gs = gather_fit_results(torch.from_numpy(cost), torch.from_numpy(st))
    xs = all_gather_ragged(torch.arange(lo, hi, dtype=torch.int64))
    if rank == 0:
        q.put((gc.numpy(), gs.numpy(), xs.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [10, 13])
def test_two_rank_fit_gather_matches_single_process(n):
    from oracle import cref
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    gc, gs, idx = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    lq, x, u = quadrotor_batch(n, T=12, seed0=0)
    _, _, cost, iters, st = cref.lq_fit(lq, x, u, max_iter=20, tol=1e-6, nthreads=1)
    assert np.array_equal(idx, np.arange(n))
    assert np.array_equal(gc, cost) and np.array_equal(gs, st)


def test_bench_gpus_flag_spawns_ranks():
    """`bench.py --gpus 2` with no launcher starts two rank processes itself (before any
    GPU call); rank 0 prints the one JSON line with n_gpus = 2 and the per-trajectory
    all-gather of 2 × batch entries. --dist-selftest runs that plumbing without a GPU
    (gloo, no solve); the GPU form is tests/test_gpu_headline.py::test_bench_two_ranks_gloo."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["ILQR_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dist-selftest",
                        "--batch", "16", "--T", "8"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["allgather_check"]["trajectories"] == 32
    assert out["allgather_check"]["own_block_matches"] and out["allgather_check"]["finite_costs"] == 32
    # every aggregate field is formed from the MAX over ranks of the per-rank times (here
    # stand-in times with rank 1 the slower), the default fit's iterations the mean
    import bench
    t0, i0 = bench.fake_rank_times(0)
    t1, i1 = bench.fake_rank_times(1)
    assert out["rank_times_max"] == {k: max(t0[k], t1[k]) for k in bench.RANK_TIMES}
    assert out["rank_times_max"] == t1 and out["dflt_iters_mean"] == (i0 + i1) / 2
    agg = out["aggregates"]
    assert agg["value"] == 2 * 1000.0 / t1["ms_step"]
    assert agg["co_headline"] == agg["fit5_batched_it_per_s"] == 2 * 5000.0 / t1["fit5_ms"]
    assert agg["fit_default_batched_it_per_s"] == 2 * 1000.0 * (i0 + i1) / 2 / t1["dflt_ms"]
    assert agg["single_iteration_batched_it_per_s"] == 2 * 1000.0 / t1["single_ms"]
    assert agg == bench.aggregate_fields(t1, (i0 + i1) / 2, 2)
