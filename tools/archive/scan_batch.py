"""Backward / forward / iterate launch time against the batch size (nx=12 nu=4 T=100):
shows whether a pass is throughput-bound (time ∝ batch) or latency-bound (flat)."""
import argparse
import ctypes as C
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]

from ilqr_amd import _lib  # noqa: E402
from ilqr_amd.problems import quadrotor_batch  # noqa: E402
from ilqr_amd.solver import Solver, _ptr  # noqa: E402


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, nargs="+", default=[1024, 4096, 8192])
    ap.add_argument("--T", type=int, default=100)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    T = a.T
    print(f"{'batch':>6} {'backward_us':>12} {'iterate_us':>11} {'iter_noring_us':>15} {'bw_us/1k':>9}", flush=True)
    for B in a.batches:
        lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
        s = Solver(12, 4, T, B)
        s.set_problem(lq)
        s._bind_stream()
        x, u = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
        d = torch.empty((B, T, 4), dtype=torch.float64, device="cuda")
        K = torch.empty((B, T, 4, 12), dtype=torch.float64, device="cuda")
        xn, un = torch.empty_like(x), torch.empty_like(u)
        pc = torch.empty((B,), dtype=torch.float64, device="cuda")
        st = torch.zeros((B,), dtype=torch.int32, device="cuda")
        tr = torch.empty((B,), dtype=torch.int32, device="cuda")
        o = _lib.default_options(tol=-1.0)
        ob = _lib.default_options()

        def bw():
            s.lib.ilqr_backward(s.h, s._p(), C.byref(ob), _ptr(x), _ptr(u), _ptr(d), _ptr(K), None)

        def fw():
            s.lib.ilqr_forward(s.h, s._p(), C.byref(ob), _ptr(x), _ptr(u), None, _ptr(d), _ptr(K), None,
                               _ptr(xn), _ptr(un), _ptr(pc), _ptr(tr), None)

        def it():
            s.iterate(x, u, xn, un, None, st, trials=tr, options=o, new_cost=pc)

        t0 = time.time()
        while time.time() - t0 < 0.3:
            it()
        torch.cuda.synchronize()
        tb, ti = timed(bw, a.reps), timed(it, a.reps)
        s.set_schedule(ring_forward=False)
        tr_ = timed(it, a.reps)
        s.set_schedule()
        print(f"{B:6d} {tb:12.1f} {ti:11.1f} {tr_:15.1f} {tb / B * 1000:9.1f}", flush=True)
        s.close()


if __name__ == "__main__":
    main()
