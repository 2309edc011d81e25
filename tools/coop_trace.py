"""Timeline of the cooperative line search in the headline's at-floor iterations, from the
trace build (ILQR_COOP_TRACE: `make -C ilqr.jl_amd/csrc tracevariant`):

    ILQR_LIB=ilqr.jl_amd/lib/variants/libilqr_hip_trace.so python tools/coop_trace.py

Runs the bench's chained iterations from cold (ilqr_iterate, prev_cost in place, as
tools/tail_probe.py) and, for each launch that published searches, prints: when the waves
finished their own trajectories, how many grabs ran, a grab's pass time and a finaliser's
time (µs, 100 MHz real-time counter), when the last wave left, and the grabs of the
deepest searches. Not product code."""
import ctypes as C
import os
import sys
from collections import defaultdict

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]
from ilqr_amd import _lib  # noqa: E402
from ilqr_amd.problems import quadrotor_batch  # noqa: E402
from ilqr_amd.solver import Solver  # noqa: E402

path = os.environ.get("ILQR_LIB", os.path.join(ROOT, "ilqr.jl_amd", "lib", "variants", "libilqr_hip_trace.so"))
_lib._lib = _lib.load(path)
lib = _lib._lib
lib.ilqr_debug_trace.restype = C.c_int
lib.ilqr_debug_trace.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
MAXR = 262144
buf = (C.c_ulonglong * (4 * MAXR))()

B, T, N = 4096, 100, int(os.environ.get("ITERS", 5))
lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
s = Solver(12, 4, T, B)
s.set_problem(lq)
s._bind_stream()
o = _lib.default_options(tol=-1.0)


def summarise(recs, it):
    if not recs:
        print(f"iteration {it}: no searches")
        return
    own = [r for r in recs if r[0] == 1]
    grabs = [r for r in recs if r[0] == 2]
    leaves = [r for r in recs if r[0] == 3]
    t00 = min(r[6] for r in own) if own else min(r[6] for r in grabs)
    us = lambda t: (t - t00) / 100.0  # noqa: E731 (100 MHz → µs)
    ownt = np.array([us(r[6]) for r in own])
    pass_us = np.array([(r[7] - r[6]) / 100.0 for r in grabs])
    fin = [r for r in grabs if r[5]]
    fin_us = np.array([(r[8] - r[7]) / 100.0 for r in fin])
    ends = [us(r[8]) for r in grabs] + [us(r[6]) for r in leaves]
    per = defaultdict(list)
    for r in grabs:
        per[r[2]].append(r)
    print(f"iteration {it}: {len(own)} waves entered the search (own done: first {ownt.min():.1f} p50 "
          f"{np.median(ownt):.1f} max {ownt.max():.1f} µs after the first); {len(per)} searches, {len(grabs)} grabs; "
          f"pass p50 {np.median(pass_us):.1f} p90 {np.percentile(pass_us, 90):.1f} max {pass_us.max():.1f} µs; "
          f"{len(fin)} finalised, finaliser p50 {np.median(fin_us) if len(fin) else 0:.1f} max "
          f"{fin_us.max() if len(fin) else 0:.1f} µs; last end {max(ends):.1f} µs", flush=True)
    grabs_per = np.array([len(v) for v in per.values()])
    print(f"  grabs per search: p50 {np.median(grabs_per):.0f} p90 {np.percentile(grabs_per, 90):.0f} "
          f"max {grabs_per.max()}; finalised at (µs) p50 "
          f"{np.median([us(r[8]) for r in fin]) if fin else 0:.1f} p90 "
          f"{np.percentile([us(r[8]) for r in fin], 90) if fin else 0:.1f}", flush=True)
    deep = sorted(per.items(), key=lambda kv: -max(r[4] for r in kv[1]))[:4]
    for b, rs in deep:
        rs = sorted(rs, key=lambda r: r[6])
        print(f"  traj {b}: lim {max(r[4] for r in rs)}, grabs " + ", ".join(
            f"j{r[3]}:{us(r[6]):.0f}-{us(r[7]):.0f}" + (f"+fin-{us(r[8]):.0f}" if r[5] else "") for r in rs),
            flush=True)


xi, ui = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
xn, un = torch.empty_like(xi), torch.empty_like(ui)
pc = torch.empty(B, dtype=torch.float64, device="cuda")
st = torch.zeros(B, dtype=torch.int32, device="cuda")
tr = torch.zeros(B, dtype=torch.int32, device="cuda")
lib.ilqr_debug_trace(buf, 0)  # reset
for it in range(N):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    s.iterate(xi, ui, xn, un, None if it == 0 else pc, st, trials=tr, options=o, new_cost=pc)
    e1.record()
    torch.cuda.synchronize()
    n = lib.ilqr_debug_trace(buf, MAXR)
    a = np.frombuffer(buf, dtype=np.uint64, count=4 * n).reshape(n, 4) if n > 0 else np.zeros((0, 4), np.uint64)
    recs = [(int(w & 15), int((w >> 4) & 15), int((w >> 24) & 0xFFFFFF), int((w >> 8) & 255), int((w >> 16) & 255),
             int((w >> 4) & 15), int(t0), int(t1), int(t2)) for w, t0, t1, t2 in a]
    # (kind, fin, id, j0, lim, fin, t0, t1, t2)
    print(f"iteration {it + 1}: {e0.elapsed_time(e1) * 1000:.1f} µs, mean trials {tr.double().mean().item():.3f}",
          flush=True)
    summarise(recs, it + 1)
    keep = st != _lib.TRAJ_OK
    xn[keep] = xi[keep]
    un[keep] = ui[keep]
    tr.zero_()
    xi, xn, ui, un = xn, xi, un, ui
