"""Median time of the headline's 3-iteration fit (B = 4096, T = 100, tol disabled) for the
product library or, with ILQR_LIB, another build — an A/B of the fit driver's own costs
(launches, gather, call status)."""
import os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]
from ilqr_amd import _lib
if os.environ.get("ILQR_LIB"):
    _lib._lib = _lib.load(os.environ["ILQR_LIB"])
from ilqr_amd.problems import quadrotor_batch
from ilqr_amd.solver import Solver

B, T = 4096, 100
lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
s = Solver(12, 4, T, B)
s.set_problem(lq)
x, u = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
t_end = time.time() + 1.0
while time.time() < t_end:
    s.fit(x, u, max_iter=3, tol=-1.0)
ts = []
for _ in range(300):
    t0 = time.perf_counter()
    r = s.fit(x, u, max_iter=3, tol=-1.0)
    ts.append(time.perf_counter() - t0)
print(f"{os.path.basename(os.environ.get('ILQR_LIB', 'product'))} ILQR_GATHER_WG="
      f"{os.environ.get('ILQR_GATHER_WG', '-')}: 3-iteration fit median "
      f"{np.median(ts) * 1e3:.4f} ms (p10 {np.percentile(ts, 10) * 1e3:.4f}), call status {r.call_status}", flush=True)
