"""The floating forward alone (ilqr_floating_forward, trial 1 accepted: one rollout per
trial lane) at several batch sizes, after 1 s of forwards: host-timed median of 15
calls. A forward's lanes run the same chain at every B, so any difference is the
launch's placement / clock. ILQR_LIB + tools/ab_lib.py runs it on another build.

    PYTHONPATH=.:ilqr.jl_amd python tools/archive/r05/floating_fw_batch_probe.py [B ...]
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

from ilqr_amd.floating import FloatingSolver, rbd_example_problem, rbd_initial_state  # noqa: E402


def main():
    batches = [int(v) for v in sys.argv[1:]] or [1, 16, 17, 64, 256, 1024]
    T = 1000
    for nb in batches:
        s = FloatingSolver(rbd_example_problem(), T, nb)
        x0 = torch.from_numpy(np.tile(rbd_initial_state(), (nb, 1))).cuda()
        u = torch.zeros(nb, T, 8, dtype=torch.float64, device="cuda")
        x = s.rollout(x0, u)
        d, K, _ = s.backward(x, u)
        pc = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
        t_end = time.perf_counter() + 1.0  # settle the clock: 1 s of forwards first
        while time.perf_counter() < t_end:
            s.forward(x, u, d, K, pc)
        ts = []
        for _ in range(15):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            s.forward(x, u, d, K, pc)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        s.close()
        print(json.dumps({"B": nb, "workgroups": (nb * 4 + 63) // 64, "forward_ms": float(np.median(ts)),
                          "min_ms": float(np.min(ts))}), flush=True)


if __name__ == "__main__":
    main()
