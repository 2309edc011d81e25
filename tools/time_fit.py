"""Time ilqr_fit on the headline workload (nx=12 nu=4 T=100, batch 4096): ms per fit
iteration, pipelined schedule vs sequential launches, and a bitwise check that both
schedules return the same result. tol is disabled, so every trajectory runs all
max_iter iterations (the check asserts it)."""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]

from ilqr_amd import _lib  # noqa: E402
from ilqr_amd.problems import quadrotor_batch  # noqa: E402
from ilqr_amd.solver import Solver  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--T", type=int, default=100)
    ap.add_argument("--iters", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--warm", type=float, default=0.3, help="seconds of untimed warmup")
    a = ap.parse_args()
    B, T = a.batch, a.T
    lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
    s = Solver(12, 4, T, B)
    s.set_problem(lq)
    x, u = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
    t0 = time.time()
    while time.time() - t0 < a.warm:
        s.fit(x, u, max_iter=4, tol=-1.0)
    torch.cuda.synchronize()
    for M in a.iters:
        res = {}
        for pipe in (False, True):
            s.set_schedule(pipelined=pipe)
            r = s.fit(x, u, max_iter=M, tol=-1.0)
            torch.cuda.synchronize()
            assert (r.iters == M).all().item() and (r.status == _lib.TRAJ_MAX_ITER).all().item()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                s.fit(x, u, max_iter=M, tol=-1.0)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            res[pipe] = (ms, r)
            print(f"max_iter={M:3d} pipelined={int(pipe)}  {ms:8.3f} ms/fit  {ms / M * 1000:8.1f} us/iter"
                  f"  {M * 1000 / ms:8.1f} batched it/s", flush=True)
        ra, rb = res[False][1], res[True][1]
        same = all(torch.equal(getattr(ra, f), getattr(rb, f)) for f in ("x", "u", "cost", "iters", "status"))
        print(f"max_iter={M:3d} pipelined == sequential: {same}", flush=True)
    s.close()


if __name__ == "__main__":
    main()
