"""Where the floating forward's stage time goes, per wave role of workgroup 0: the trace
build (make -C ilqr.jl_amd/csrc tracevariant → lib/variants/libilqr_hip_fbtrace.so)
totals, per wave, the 100 MHz counter's ticks between barriers (work), at them (wait)
and in its sequence-word polls (poll, part of work), and the phases between FBT_MARKs
(mass: rotation, CRBA incl. the R₀ poll, Schur + store; main: bias, solve incl. the ū
poll, RK update + stores; the rest of work after the last mark). Printed per barrier, i.e. per RK4
stage, in ns, beside the forward's host time in the trace build. Not product code.

    python tools/fb_trace.py [B ...]
"""
import json
import os
import sys
import time
import ctypes as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
from ilqr_amd import _lib  # noqa: E402

LIB = os.path.join(ROOT, "ilqr.jl_amd", "lib", "variants", "libilqr_hip_fbtrace.so")
_lib._lib = _lib.load(LIB)
from ilqr_amd.floating import FloatingSolver, rbd_example_problem, rbd_initial_state  # noqa: E402

ROLES = {0: "mass (joint 1)", 3: "rotation (joint 0)", 1: "main (bias, solve, RK)", 2: "control (u, cost)"}


def main():
    lib = _lib._lib
    lib.ilqr_debug_fb_trace.argtypes = [C.POINTER(C.c_ulonglong)]
    buf = (C.c_ulonglong * 32)()
    T = 1000
    for nb in [int(v) for v in sys.argv[1:]] or [1, 64, 1024]:
        s = FloatingSolver(rbd_example_problem(), T, nb)
        x0 = np.tile(rbd_initial_state(), (nb, 1))
        x0[:, 8:] += 0.05 * np.random.default_rng(nb).standard_normal((nb, 8))
        x0 = torch.from_numpy(x0).cuda()
        u = torch.zeros(nb, T, 8, dtype=torch.float64, device="cuda")
        x = s.rollout(x0, u)
        d, K, _ = s.backward(x, u)
        pc = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
        for _ in range(3):
            s.forward(x, u, d, K, pc)
        torch.cuda.synchronize()
        assert lib.ilqr_debug_fb_trace(buf) == 0  # reset
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            s.forward(x, u, d, K, pc)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        assert lib.ilqr_debug_fb_trace(buf) == 0
        v = np.array(buf[:], dtype=np.float64).reshape(4, 8)
        rec = {"B": nb, "forward_ms_median": 1e3 * float(np.median(ts))}
        for r, name in ROLES.items():
            n = max(v[r, 3], 1.0)
            rec[name] = {"barriers": int(v[r, 3]), "work_ns": round(10 * v[r, 0] / n, 1),
                         "wait_ns": round(10 * v[r, 1] / n, 1), "poll_ns": round(10 * v[r, 2] / n, 1),
                         "phases_ns": [round(10 * w / n, 1) for w in v[r, 4:8]]}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
