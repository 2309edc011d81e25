"""Where a fit iteration of the reference's RBD caller goes (nx = 16, nu = 8, T = 1000,
B = 1: test/RBD_2_link_example/animate_RBD_2_link.jl:8,19-20,31) on the generic closure
path: derivative tiles (torch.func on the device), ilqr_backward_tiles (the wide HIP
kernel) and the forward_pass rollout of the closures (one accepted trial: the first
iteration's prev_cost is Inf), HIP-graph replay and eager. Wall times with a device
synchronise around each phase, medians over repetitions.

    PYTHONPATH=.:ilqr.jl_amd:tests python tools/archive/r05/rbd_fit_breakdown.py [B] [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
for p in (ROOT, os.path.join(ROOT, "ilqr.jl_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from closures import jet_ns, rbd_floating_arm, rbd_initial_state, torch_arr_ns  # noqa: E402
from ilqr_amd import _lib, api  # noqa: E402
from ilqr_amd import tiles as _tiles  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    T = 1000
    fj, _, _ = rbd_floating_arm(jet_ns())
    x = np.zeros((nb, T + 1, 16))
    x[:, 0] = rbd_initial_state()
    u = np.zeros((nb, T, 8))
    for t in range(T):
        x[:, t + 1] = fj(x[:, t], u[:, t])
    f, l, lf = rbd_floating_arm(torch_arr_ns())
    xb, ub = torch.from_numpy(x).cuda(), torch.from_numpy(u).cuda()
    xt = torch.zeros_like(xb)
    prev = torch.full((nb,), float("inf"), dtype=torch.float64, device=xb.device)
    times = {"derivative_tiles": [], "backward_tiles": [], "rollout_forward": [], "rollout_forward_eager": []}

    def timed(name, fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        times[name].append((time.perf_counter() - t0) * 1e3)
        return out

    with api._tiles_solver(xb, ub) as s:
        for _ in range(reps + 1):  # the first repetition warms torch.func and the caches
            tl = timed("derivative_tiles", lambda: _tiles.derivative_tiles(xb, ub, f, l, lf))
            d, K, _ = timed("backward_tiles", lambda: s.backward_tiles(tl))
            timed("rollout_forward", lambda: _tiles.rollout_forward(
                xb, ub, xt, d, K, prev, f, l, lf, _lib.default_options().max_trials))
            _tiles.ROLLOUT_GRAPHS = False
            timed("rollout_forward_eager", lambda: _tiles.rollout_forward(
                xb, ub, xt, d, K, prev, f, l, lf, _lib.default_options().max_trials))
            _tiles.ROLLOUT_GRAPHS = True
    med = {k: float(np.median(v[1:])) for k, v in times.items()}
    print(json.dumps({"B": nb, "T": T, "nx": 16, "nu": 8, "ms_median": med, "reps": reps}))


if __name__ == "__main__":
    main()
