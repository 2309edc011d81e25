"""Where a native RBD-script iteration goes (ilqr_floating_*, B = 1, T = 1000): the
line search's accepted trial per iteration (fit history) and the median wall time of
each stage called alone — linearize, backward, forward (its trials) — plus a T-step
rollout through the one-step dynamics launch.

    PYTHONPATH=.:ilqr.jl_amd python tools/archive/r05/floating_probe.py [iters] [B]
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

from ilqr_amd import _lib  # noqa: E402
from ilqr_amd.floating import FloatingSolver, rbd_example_problem, rbd_initial_state  # noqa: E402


def timed(f, reps=5):
    f()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = f()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts)), out


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    T = 1000
    s = FloatingSolver(rbd_example_problem(), T, nb)
    x0 = np.tile(rbd_initial_state(), (nb, 1))
    x0t = torch.from_numpy(x0).cuda()
    u = torch.zeros(nb, T, 8, dtype=torch.float64, device="cuda")
    t_roll, x = timed(lambda: s.rollout(x0t, u), reps=3)
    r = s.fit(x, u, options=_lib.default_options(max_iter=iters, tol=-1.0), history=True)
    trials = r.history["trials"][:, 0].cpu().tolist()
    # the stages at the iterate after `iters` iterations (a typical late iteration)
    xk, uk = r.x, r.u
    t_lin, _ = timed(lambda: s.linearize(xk, uk))
    t_bw, (d, K, _) = timed(lambda: s.backward(xk, uk))
    pc = torch.full((nb,), float(r.cost[0]) * 10, dtype=torch.float64, device="cuda")
    t_fw, fo = timed(lambda: s.forward(xk, uk, d, K, pc))
    o = _lib.default_options()
    o.alpha0 = o.alpha0 * 0.5 ** 5
    t_fw5, fo5 = timed(lambda: s.forward(xk, uk, d, K, torch.full_like(pc, float(r.cost[0])), options=o))
    print(json.dumps({"B": nb, "T": T, "fit_trials_per_iteration": trials,
                      "ms": {"rollout_T_steps": t_roll, "linearize": t_lin, "backward": t_bw,
                             "forward_trial1": t_fw, "forward_from_cost": t_fw5},
                      "forward_trials": [int(fo[3][0]), int(fo5[3][0])]}), flush=True)
    s.close()


if __name__ == "__main__":
    main()
