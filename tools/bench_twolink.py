"""Secondary benchmark: BASELINE config 2 — the 2-link arm (nx=4, nu=2, T=50),
batch 1024 random x₀, fp64, 1 GPU. Same step definition as bench.py (one
cold-start fit iteration over the batch: linearise + backward + forward with
line search), timed with HIP events on the handle's stream. Prints one JSON line.
Not the driver's headline (bench.py); see DESIGN.md §2-link.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]

from ilqr_amd import _lib  # noqa: E402
from ilqr_amd.problems import two_link_initial_states  # noqa: E402
from ilqr_amd.solver import Solver, _ptr  # noqa: E402


def timed(fn, n, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(n):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--T", type=int, default=50)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    B, T = args.batch, args.T
    dev = torch.device("cuda", 0)
    s = Solver(4, 2, T, B, kind=_lib.PROBLEM_TWO_LINK)
    x0 = two_link_initial_states(B)
    u = torch.zeros((B, T, 2), dtype=torch.float64, device=dev)
    x = s.rollout(torch.from_numpy(x0).to(dev), u)
    xn, un = torch.empty_like(x), torch.empty_like(u)
    pc = torch.empty((B,), dtype=torch.float64, device=dev)
    st = torch.zeros((B,), dtype=torch.int32, device=dev)
    trials = torch.empty((B,), dtype=torch.int32, device=dev)
    opts = _lib.default_options(tol=-1.0)
    stream = torch.cuda.current_stream(dev)
    s._bind_stream()

    def step():
        s.iterate(x, u, xn, un, None, st, trials=trials, options=opts, new_cost=pc)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ms_ev = timed(step, args.steps, stream)
    ms_wall = (time.perf_counter() - t0) * 1000.0 / args.steps
    ms = max(ms_ev, ms_wall)

    d = torch.empty((B, T, 2), dtype=torch.float64, device=dev)
    K = torch.empty((B, T, 2, 4), dtype=torch.float64, device=dev)
    o = _lib.default_options()
    bw = lambda: s.lib.ilqr_backward(s.h, s._p(), C.byref(o), _ptr(x), _ptr(u), _ptr(d), _ptr(K), None)
    bw()
    bw_ms = timed(bw, args.steps, stream)
    pinf = torch.full((B,), float("inf"), dtype=torch.float64, device=dev)
    nc = torch.empty_like(pinf)
    fw = lambda: s.lib.ilqr_forward(s.h, s._p(), C.byref(o), _ptr(x), _ptr(u), None, _ptr(d), _ptr(K),
                                    _ptr(pinf), _ptr(xn), _ptr(un), _ptr(nc), None, None)
    fw()
    fw_ms = timed(fw, args.steps, stream)

    out = {
        "metric": "batched iLQR iterations/sec (fwd+bwd pass), 2-link arm nx=4 nu=2 T=50, batch=1024",
        "value": 1000.0 / ms, "unit": "batched iterations/s (batch=1024)", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
        "dtype": "f64", "data": "synthetic: x0 = default_rng(b).random(4), u0 = 0, rollout",
        "config": {"workload": "2-link arm fit iteration (cold start)", "T": T, "batch": B},
        "backward_ms": bw_ms, "forward_ms": fw_ms, "event_ms": ms_ev, "wall_ms": ms_wall,
        "traj_iters_per_s": B * 1000.0 / ms,
        "mean_trials": float(trials.double().mean()), "all_ok": bool((st == 0).all()),
        "cpu_baseline": None,
    }
    if not args.no_cpu:
        try:
            from oracle import cref
            out["cpu_baseline"] = cref.twolink_cpu_baseline(x.cpu().numpy(), u.cpu().numpy(), B,
                                                            args.cpu_budget)
        except Exception as e:
            out["cpu_baseline"] = {"error": repr(e)}
    print(json.dumps(out), flush=True)
    s.close()


if __name__ == "__main__":
    main()
