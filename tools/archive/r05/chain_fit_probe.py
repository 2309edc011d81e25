"""Where the chain family's default fit (tol = 1e-6, max_iter = 100; config 5's shape,
fp32, central differences, B = 2048, T = 100) spends its iterations: per iteration the
trajectories still running and their line searches' mean and max trials (fit history),
for the reference's 2Dof_arm and the coupled test chain.

    PYTHONPATH=.:ilqr.jl_amd python tools/archive/r05/chain_fit_probe.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
for p in (ROOT, os.path.join(ROOT, "ilqr.jl_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ilqr_amd.chain import ChainSolver, coupled_2dof_problem, rbd_2dof_problem, rbd_initial_states  # noqa: E402


def main():
    B, T = 2048, 100
    for name, pr in (("rbd_2dof", rbd_2dof_problem(1)), ("coupled", coupled_2dof_problem(1))):
        s = ChainSolver(pr, T, B, dtype=torch.float32, linearization="fd")
        u = torch.zeros((B, T, pr.nu), dtype=torch.float32, device="cuda")
        x = s.rollout(torch.from_numpy(rbd_initial_states(B, 2)).to("cuda", torch.float32), u)
        r = s.fit(x, u, max_iter=100, tol=1e-6, history=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = s.fit(x, u, max_iter=100, tol=1e-6, history=True)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        tr = r.history["trials"].cpu().numpy()  # (max_iter, B)
        rows = []
        for i in range(tr.shape[0]):
            live = tr[i] > 0
            if not live.any():
                break
            rows.append([i + 1, int(live.sum()), round(float(tr[i][live].mean()), 2), int(tr[i].max())])
        s.close()
        print(json.dumps({"chain": name, "fit_ms": ms, "iters_mean": float(r.iters.double().mean()),
                          "per_iteration[it, running, mean_trials, max_trials]": rows}), flush=True)


if __name__ == "__main__":
    main()
