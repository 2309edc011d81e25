"""Secondary benchmark: BASELINE config 2 — the 2-link arm (nx=4, nu=1 as the config
states: f(x, [u₁, 0]); --nu 2 for the reference's own shape; T=50), batch 1024 random
x₀, fp64, 1 GPU. Step:
one cold-start fit iteration over the batch (linearise + backward + forward with
line search), timed with HIP events on the handle's stream. Prints one JSON line with
a roofline object per kernel (algorithmic FLOPs of the reference's formulas,
tools/flops.py, against the FP64 peak). Not the driver's headline (bench.py); see
DESIGN.md §2-link.
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
from tools import flops as FL  # noqa: E402

FP64_PEAK_TFLOPS = 78.6


def timed(fn, n, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(n):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def measure(B=1024, T=50, NU=1, steps=200, warmup=500, device=0, cpu_budget=None):
    """Config 2's fit-iteration rate and per-kernel roofline (one dict; bench.py's
    secondary_configs calls this after its headline, outside the headline's timed region)."""
    dev = torch.device("cuda", device)
    s = Solver(4, NU, T, B, device=device, kind=_lib.PROBLEM_TWO_LINK)
    x0 = two_link_initial_states(B)
    u = torch.zeros((B, T, NU), dtype=torch.float64, device=dev)
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

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ms_ev = timed(step, steps, stream)
    ms_wall = (time.perf_counter() - t0) * 1000.0 / steps
    ms = max(ms_ev, ms_wall)

    d = torch.empty((B, T, NU), dtype=torch.float64, device=dev)
    K = torch.empty((B, T, NU, 4), dtype=torch.float64, device=dev)
    o = _lib.default_options()
    bw = lambda: s.lib.ilqr_backward(s.h, s._p(), C.byref(o), _ptr(x), _ptr(u), _ptr(d), _ptr(K), None)
    bw()
    bw_ms = timed(bw, steps, stream)
    pinf = torch.full((B,), float("inf"), dtype=torch.float64, device=dev)
    nc = torch.empty_like(pinf)
    fw = lambda: s.lib.ilqr_forward(s.h, s._p(), C.byref(o), _ptr(x), _ptr(u), None, _ptr(d), _ptr(K),
                                    _ptr(pinf), _ptr(xn), _ptr(un), _ptr(nc), None, None)
    fw()
    fw_ms = timed(fw, steps, stream)

    # algorithmic FLOPs (tools/flops.py): linearise = dual RK4 over 4+NU directions,
    # backward = the Riccati step count, forward = one trial (1 on a cold start)
    f_rk4 = FL.twolink_dynamics_flops(NU)
    lin_fl = f_rk4 * FL.dual_factor(4 + NU) * T * B
    ric_fl = FL.riccati_flops_per_step(4, NU) * T * B
    fw_fl = FL.forward_flops_per_step(4, NU, f_rk4) * T * B
    roof = {"bound": "latency (the forward is one dependent RK4 chain per trajectory; B = 1024 fills 64 of 1024 SIMDs)",
            "unit": "TFLOP/s", "peak": FP64_PEAK_TFLOPS,
            "backward": {"kernels": "tl_linearize + tl_backward (4 trajectories per wave, 4x4x4 f64 MFMA)",
                         "avg_launch_ms": bw_ms, "algorithmic_flops": lin_fl + ric_fl,
                         "achieved": (lin_fl + ric_fl) / (bw_ms * 1e-3) / 1e12},
            "forward": {"kernel": "tl_forward (4 line-search candidate lanes per trajectory, branch-free rk4_roll)", "avg_launch_ms": fw_ms,
                        "algorithmic_flops": fw_fl, "achieved": fw_fl / (fw_ms * 1e-3) / 1e12},
            "flops_note": f"RK4 of the reference's formulas = {f_rk4} flop (tools/flops.py); dual factor "
                          f"1+2·ND; Riccati per SURVEY §8d"}
    for k in ("backward", "forward"):
        roof[k]["frac"] = roof[k]["achieved"] / FP64_PEAK_TFLOPS
    roof["achieved"] = roof["forward"]["achieved"]
    roof["frac"] = roof["forward"]["frac"]
    # the forward's real bound: T dependent RK4 steps per trajectory, so its time is
    # T × the latency of one step (one wave's instruction stream), whatever the batch
    roof["forward"]["step_latency_ns"] = fw_ms * 1e6 / T
    roof["forward"]["lanes_busy_frac"] = min(1.0, 4 * B / (1024 * 64))
    out = {
        "metric": f"batched iLQR iterations/sec (fwd+bwd pass), 2-link arm nx=4 nu={NU} T={T}, batch={B}",
        "value": 1000.0 / ms, "unit": f"batched iterations/s (batch={B})", "n_gpus": 1,
        "steps": steps, "warmup": warmup, "ms_per_step": ms, "higher_is_better": True,
        "dtype": "f64", "data": "synthetic: x0 = default_rng(b).random(4), u0 = 0, rollout",
        "config": {"workload": "2-link arm fit iteration (cold start)", "T": T, "batch": B, "nu": NU,
                   "variant": "reference shape" if NU == 2 else "f(x, [u1, 0]), build-defined, not reference-pinned"},
        "backward_ms": bw_ms, "forward_ms": fw_ms, "event_ms": ms_ev, "wall_ms": ms_wall,
        "roofline": roof,
        "traj_iters_per_s": B * 1000.0 / ms,
        "mean_trials": float(trials.double().mean()), "all_ok": bool((st == 0).all()),
        "cpu_baseline": None,
    }
    if cpu_budget:
        try:
            from oracle import cref
            out["cpu_baseline"] = cref.twolink_cpu_baseline(x.cpu().numpy(), u.cpu().numpy(), B, cpu_budget)
        except Exception as e:
            out["cpu_baseline"] = {"error": repr(e)}
    s.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--T", type=int, default=50)
    ap.add_argument("--nu", type=int, default=1, choices=[1, 2],
                    help="1 = BASELINE config 2 as stated (f(x, [u1, 0])); 2 = the reference's shape")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    out = measure(args.batch, args.T, args.nu, args.steps, args.warmup,
                  cpu_budget=None if args.no_cpu else args.cpu_budget)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
