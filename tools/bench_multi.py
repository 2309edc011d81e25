"""Multi-device fit in one process (include/ilqr.h ilqr_multi_*): the transfer-inclusive
host path (ilqr_multi_fit: problem + trajectories up, results down on every call)
against the device-resident path (ilqr_multi_fit_resident; results gathered into
pinned host buffers only when asked), on BASELINE config 4's global batch — 32,768
trajectories in 8 shards — here all on the box's one GPU (shards run concurrently on
its streams). Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]
from ilqr_amd.multi import HostBuffers, MultiSolver  # noqa: E402
from ilqr_amd.problems import quadrotor_batch  # noqa: E402


def med(fn, reps):
    ts = []
    for _ in range(reps + 2):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts[2:])) * 1000.0


def main():
    B, T, shards, iters = 32768, 100, int(os.environ.get("SHARDS", 8)), 3
    lq, x, u = quadrotor_batch(B, T=T, seed0=0)
    ms = MultiSolver([0] * shards, 12, 4, T, B)
    hb = HostBuffers(x=(x.shape, np.float64), u=(u.shape, np.float64), cost=((B,), np.float64))
    xo, uo = np.empty_like(x), np.empty_like(u)
    try:
        host_ms = med(lambda: ms.fit(lq, x, u, max_iter=iters, tol=-1.0), 5)
        ms.set_problem(lq)
        ms.load(x, u)
        res_ms = med(lambda: ms.fit_resident(max_iter=iters, tol=-1.0), 10)
        gather_all_ms = med(lambda: ms.gather(iters=False, status=False, out=hb.arrays), 10)
        gather_cost_ms = med(lambda: ms.gather(x=False, u=False, iters=False, status=False, out=hb.arrays), 10)
        hb.arrays["x"][:] = x
        hb.arrays["u"][:] = u
        load_ms = med(lambda: ms.load(hb.arrays["x"], hb.arrays["u"]), 10)
        host_bytes = 8 * (x.size * 2 + u.size * 2 + lq.A.size + lq.B.size + lq.Q.size + lq.R.size + lq.Qf.size + B)
    finally:
        hb.close()
        ms.close()
    print(json.dumps({
        "workload": f"quadrotor LQ fit, {iters} iterations from cold, tol disabled; B={B} in {shards} shards "
                    f"on one MI355X", "batched_iterations": iters,
        "host_path_ms_per_fit": host_ms,
        "resident_fit_ms": res_ms,
        "resident_gather_x_u_cost_pinned_ms": gather_all_ms,
        "resident_gather_cost_only_ms": gather_cost_ms,
        "resident_load_x_u_pinned_ms": load_ms,
        "host_path_bytes_moved": host_bytes,
        "host_path_effective_gbps": host_bytes / (host_ms * 1e-3) / 1e9,
        "trajectory_iterations_per_s_resident": B * iters / (res_ms * 1e-3),
        "trajectory_iterations_per_s_host_path": B * iters / (host_ms * 1e-3),
    }), flush=True)


if __name__ == "__main__":
    main()
