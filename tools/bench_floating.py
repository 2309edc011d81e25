"""The reference's RBD script fitted natively (ilqr_amd.floating, include/ilqr.h
ilqr_floating_*): test/RBD_2_link_example/animate_RBD_2_link.jl's problem, nx = 16,
nu = 8, T = 1000, from its own start (rest state, zero inputs, x_init = rollout).
Prints one JSON line per batch size: ms per fit iteration (a fit of `iters` iterations
with the convergence test disabled, median of `reps` after a warm-up), beside the
generic closure path's per-iteration cost (profiles/r05/rbd_fit_breakdown_r05.json).

    PYTHONPATH=.:ilqr.jl_amd python tools/bench_floating.py [iters] [reps] [B ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ilqr.jl_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ilqr_amd import _lib  # noqa: E402
from ilqr_amd.floating import FloatingSolver, rbd_example_problem, rbd_initial_state  # noqa: E402


def measure(nb, T=1000, iters=5, reps=3):
    p = rbd_example_problem()
    s = FloatingSolver(p, T, nb)
    try:
        x0 = np.tile(rbd_initial_state(), (nb, 1))
        x0[1:, 8:] = 0.05 * np.random.default_rng(7).standard_normal((nb - 1, 8))
        u = torch.zeros(nb, T, 8, dtype=torch.float64, device="cuda")
        x = s.rollout(torch.from_numpy(x0).cuda(), u)
        o = _lib.default_options(max_iter=iters, tol=-1.0)
        r = s.fit(x, u, options=o)  # warm-up
        times = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = s.fit(x, u, options=o)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
        st = r.status.cpu().numpy()
        return {"workload": "animate_RBD_2_link.jl fit (floating 2Dof_arm, native)", "nx": 16, "nu": 8,
                "T": T, "B": nb, "iters": iters, "ms_per_fit": float(np.median(times)),
                "ms_per_iteration": float(np.median(times)) / iters,
                "batched_it_per_s": 1e3 * iters / float(np.median(times)),
                "status_counts": {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
                "cost0": float(r.cost[0])}
    finally:
        s.close()


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    batches = [int(v) for v in sys.argv[3:]] or [1, 256]
    for nb in batches:
        print(json.dumps(measure(nb, iters=iters, reps=reps)), flush=True)


if __name__ == "__main__":
    main()
