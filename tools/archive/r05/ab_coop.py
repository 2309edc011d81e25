"""A/B of the fused iteration's line-search schedules (cooperative vs sequential) on
the headline batch: one cold iteration (ilqr_iterate) and the 5-iteration fit."""
import sys, os, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]
from ilqr_amd import _lib
from ilqr_amd.problems import quadrotor_batch
from ilqr_amd.solver import Solver

B, T = int(os.environ.get("B", 4096)), 100
lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
s = Solver(12, 4, T, B)
s.set_problem(lq)
s._bind_stream()
x, u = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
xn, un = torch.empty_like(x), torch.empty_like(u)
pc = torch.empty(B, dtype=torch.float64, device="cuda")
st = torch.zeros(B, dtype=torch.int32, device="cuda")
o1 = _lib.default_options(tol=-1.0)

def cold(n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        s.iterate(x, u, xn, un, None, st, options=o1, new_cost=pc)
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000

def fit(n_iter, reps=20):
    ts = []
    for _ in range(reps + 3):
        t0 = time.perf_counter()
        s.fit(x, u, max_iter=n_iter, tol=-1.0)
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts[3:])) * 1000

t_end = time.time() + 1.0
while time.time() < t_end:
    cold(10)
for rnd in range(2):
    for seq in (True, False):
        s.set_schedule(sequential_search=seq)
        c = cold(200)
        f3, f5 = fit(3), fit(5)
        print(f"{'sequential' if seq else 'coop':10s} cold iteration {c:7.1f} us  fit3 {f3:.3f} ms ({3000/f3:.0f} it/s)  "
              f"fit5 {f5:.3f} ms ({5000/f5:.0f} it/s)", flush=True)
