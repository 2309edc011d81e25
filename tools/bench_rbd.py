"""Secondary benchmark: BASELINE config 5 — the RBD example (RigidBodyDynamics-style
dynamics of test/urdf/2Dof_arm.urdf, fixed base: nx = 4, nu = 1 as the config states, or
--nu 2), T = 100,
batch 2048 random x₀, fp32, linearised on the device by central finite differences
(BASELINE's wording) or dual numbers (the reference's ForwardDiff). Same step as
bench.py: one cold-start fit iteration over the batch (linearise + backward +
forward with line search), timed with HIP events on torch's current stream.
Prints one JSON line per linearisation. The CPU baseline is the C restatement
(oracle/ilqr_ref.c, fp64, OpenMP) on a bounded sample — a port, not the reference.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]

from ilqr_amd import _lib  # noqa: E402
from ilqr_amd.chain import ChainSolver, rbd_2dof_problem, rbd_initial_states  # noqa: E402
from tools import flops as FL  # noqa: E402

PEAK_TFLOPS = {"f32": 157.3, "f64": 78.6}   # MI355X vector FP32 / FP64 (spec; MI355X_MICROARCH.md)


def timed(fn, n, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(n):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def cpu_baseline(pr, x, u, budget_s):
    """The C restatement of the chain family (oracle/ilqr_ref.c: oracle_chain_iterate,
    fp64, central differences, OpenMP over trajectories) on a bounded sample: one
    cold-start iteration per trajectory."""
    from oracle import cref
    visible = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    threads = min(visible, int(share)) if share and share.isdigit() and int(share) > 0 else visible
    n = 16
    while True:
        idx = np.arange(n) % x.shape[0]
        t0 = time.perf_counter()
        cref.chain_iterate(pr, x[idx], u[idx], nthreads=threads)
        el = time.perf_counter() - t0
        if el > budget_s / 2 or n >= 1 << 15:
            break
        n *= 2
    return {"value": n / el, "unit": "trajectory-iterations/s", "cores": threads, "kind": "port",
            "sample": f"{n} trajectories x 1 cold-start iteration (C restatement oracle/ilqr_ref.c "
                      f"oracle_chain_iterate, fp64, central differences, OpenMP {threads} threads, -O3), "
                      f"{el:.2f} s"}


def measure(lin="fd", B=2048, T=100, nu=1, dtype="f32", steps=100, warmup=100, device=0,
            dynamics="auto", cpu_budget=None, base=None, problem=None):
    """Config 5's fit-iteration rate and per-kernel roofline for one linearisation (one
    dict; bench.py's secondary_configs calls this after its headline, outside the
    headline's timed region)."""
    dt = torch.float32 if dtype == "f32" else torch.float64
    dev = torch.device("cuda", device)
    # problem: another chain (the coupled 2-joint test chain: q-dependent M and bias, which
    # the reference's 2Dof_arm.urdf parses without — constant M, zero bias)
    pr = rbd_2dof_problem(nu) if problem is None else problem
    x0 = rbd_initial_states(B, 2)
    s = ChainSolver(pr, T, B, dtype=dt, linearization=lin, device=device)
    s.set_dynamics(dynamics)
    u = torch.zeros((B, T, pr.nu), dtype=dt, device=dev)
    x = s.rollout(torch.from_numpy(x0).to(dev, dt), u)
    xn, un = torch.empty_like(x), torch.empty_like(u)
    pc = torch.empty((B,), dtype=dt, device=dev)
    st = torch.zeros((B,), dtype=torch.int32, device=dev)
    trials = torch.empty((B,), dtype=torch.int32, device=dev)
    opts = _lib.default_options(tol=-1.0)
    stream = torch.cuda.current_stream(dev)
    s._bind()

    def step():
        s.iterate(x, u, xn, un, None, st, pc, trials=trials, options=opts)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ms_ev = timed(step, steps, stream)
    ms = max(ms_ev, (time.perf_counter() - t0) * 1000.0 / steps)
    ok = bool((st == 0).all().item())
    # per-kernel times and the roofline object (algorithmic FLOPs, tools/flops.py)
    d = torch.empty((B, T, pr.nu), dtype=dt, device=dev)
    K = torch.empty((B, T, pr.nu, pr.nx), dtype=dt, device=dev)
    A = torch.empty((B, T, pr.nx, pr.nx), dtype=dt, device=dev)
    Bm = torch.empty((B, T, pr.nx, pr.nu), dtype=dt, device=dev)
    o = _lib.default_options()
    import ctypes as C
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    lin_fn = lambda: s.lib.ilqr_chain_linearize(s.h, P(x), P(u), P(A), P(Bm))  # noqa: E731
    bw = lambda: s.lib.ilqr_chain_backward(s.h, C.byref(o), P(x), P(u), P(d), P(K), None)  # noqa: E731
    pinf = torch.full((B,), float("inf"), dtype=dt, device=dev)
    nc = torch.empty_like(pinf)
    fw = lambda: s.lib.ilqr_chain_forward(s.h, C.byref(o), P(x), P(u), None, P(d), P(K), P(pinf),  # noqa: E731
                                          P(xn), P(un), P(nc), None, None)
    for fn in (lin_fn, bw, fw):
        fn()
    lin_ms = timed(lin_fn, steps, stream)
    bw_ms = timed(bw, steps, stream)   # ilqr_chain_backward = linearise + Riccati
    fw_ms = timed(fw, steps, stream)
    nd = pr.nx + pr.nu
    # algorithmic FLOPs of the evaluator that runs: the closed form's own count
    # (pricing it on the recursion's 16x larger count put the linearisation above peak)
    f_ref = FL.chain_dynamics_flops(pr)
    f_rk4 = FL.chain_closed_form_flops(pr.nu) if s.dynamics_mode == "closed_form" else f_ref
    lin_fl = (f_rk4 * FL.dual_factor(nd) if lin == "dual" else 2 * nd * f_rk4 + nd * pr.nx) * T * B
    ric_fl = FL.riccati_flops_per_step(pr.nx, pr.nu) * T * B
    fw_fl = FL.forward_flops_per_step(pr.nx, pr.nu, f_rk4) * T * B
    peak = PEAK_TFLOPS[dtype]
    kern = {"linearize": (lin_ms, lin_fl), "riccati": (max(bw_ms - lin_ms, 1e-6), ric_fl),
            "forward": (fw_ms, fw_fl)}
    roof = {"bound": ("forward latency/issue (a dependent RK4 chain per trajectory, 4 candidate lanes each, "
                      "closed-form dynamics)"
                      if s.dynamics_mode == "closed_form" else
                      "forward latency/issue (16 lanes per trajectory)") + ", linearisation VALU issue",
            "unit": "TFLOP/s", "peak": peak, "peak_dtype": dtype,
            "flops_note": (f"RK4 of the closed form = {f_rk4} flop; of the restated RBD recursion "
                           f"(the reference's RigidBodyDynamics.jl calls) = {f_ref} flop (tools/flops.py)"
                           if f_rk4 != f_ref else
                           f"RK4 of the restated RBD formulas = {f_rk4} flop (tools/flops.py)")}
    for k, (ms_k, fl) in kern.items():
        roof[k] = {"avg_launch_ms": ms_k, "algorithmic_flops": fl,
                   "achieved": fl / (ms_k * 1e-3) / 1e12, "frac": fl / (ms_k * 1e-3) / 1e12 / peak}
    roof["achieved"], roof["frac"] = roof["forward"]["achieved"], roof["forward"]["frac"]
    # the forward's real bound: T dependent RK4 steps per trajectory (4 line-search
    # candidate lanes each: 4B of the chip's 65,536 lanes), so its time is T × the
    # latency of one step — the FLOP fraction is small by construction
    roof["forward"]["step_latency_ns"] = fw_ms * 1e6 / T
    roof["forward"]["lanes_busy_frac"] = min(1.0, 4 * B / (1024 * 64))
    res = {"metric": f"batched iLQR iterations/sec (fwd+bwd pass), RBD 2-DoF arm fixed base, "
                     f"nx=4 nu={pr.nu} T={T}",
           "value": 1000.0 / ms, "unit": f"batched iterations/s (batch={B})", "n_gpus": 1,
           "steps": steps, "warmup": warmup, "ms_per_step": ms,
           "higher_is_better": True, "dtype": dtype, "data": "synthetic x0 ~ U(-1,1)",
           "config": {"workload": "BASELINE config 5 (RBD_2_link_example, fixed base)",
                      "batch": B, "T": T, "linearization": lin, "dynamics": s.dynamics_mode,
                      "closed_form_check": s.closed_form_error},
           "traj_iters_per_s": B * 1000.0 / ms,
           "mean_line_search_trials": float(trials.double().mean().item()), "all_ok": ok,
           "roofline": roof,
           "cpu_baseline": None}
    if cpu_budget:
        if base is None:
            xs = x[: min(B, 256)].double().cpu().numpy()
            us = u[: min(B, 256)].double().cpu().numpy()
            base = cpu_baseline(pr, xs, us, cpu_budget)
            base["value"] = base["value"] / B  # trajectory-iterations/s → batched it/s
            base["unit"] = f"batched iterations/s (batch={B})"
        res["cpu_baseline"] = base
    res["fit"] = fit_timing(s, x, u)
    s.close()
    return res


def fit_timing(s, x, u, n=40):
    """ChainSolver.fit end to end (synchronous, wall clock, median of n): the 3-iteration
    fit from cold (tol disabled) and the reference's default call (tol = 1e-6,
    max_iter = 100)."""
    out = {}
    for name, kw in (("fit3", dict(max_iter=3, tol=-1.0)), ("fit_default", dict(max_iter=100, tol=1e-6))):
        for _ in range(5):
            r = s.fit(x, u, **kw)
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            r = s.fit(x, u, **kw)
            ts.append(time.perf_counter() - t0)
        ms = float(np.median(ts)) * 1e3
        it = float(r.iters.double().mean().item())
        out[name] = {"median_ms": ms, "mean_iterations": it, "batched_it_per_s": it * 1e3 / ms}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--T", type=int, default=100)
    ap.add_argument("--nu", type=int, default=1, choices=[1, 2],
                    help="1 = BASELINE config 5 as stated; 2 = both joints actuated")
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    ap.add_argument("--lin", default="fd,dual")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dynamics", default="auto", choices=["auto", "rnea", "closed_form"],
                    help="the chain handle's dynamics evaluator (ilqr_chain_set_dynamics)")
    args = ap.parse_args()
    base = None
    for lin in args.lin.split(","):
        res = measure(lin, args.batch, args.T, args.nu, args.dtype, args.steps, args.warmup,
                      dynamics=args.dynamics, cpu_budget=None if args.no_cpu else args.cpu_budget, base=base)
        base = res["cpu_baseline"]
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
