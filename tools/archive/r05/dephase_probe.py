"""Timing of the fused iteration launch (fit's first iteration, repeated on the same
inputs: prev_cost = Inf, every trajectory accepts trial 1) with the product build and
the two timing-only phase-mix builds of tools/archive/r05/dephase_probe.sh, each in its own process
on one box: `python tools/archive/r05/dephase_probe.py [lib.so]`."""
import ctypes as C
import os
import sys
import time

import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path[:0] = [R, os.path.join(R, "ilqr.jl_amd")]
from ilqr_amd import _lib  # noqa: E402
from ilqr_amd.problems import quadrotor_batch  # noqa: E402
from ilqr_amd.solver import Solver  # noqa: E402

LIB = sys.argv[1] if len(sys.argv) > 1 else None
if LIB:
    _lib._lib = _lib.load(LIB)
B, T = 4096, 100
lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
s = Solver(12, 4, T, B)
s.set_problem(lq)
s._bind_stream()
x, u = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
xn, un = torch.empty_like(x), torch.empty_like(u)
pc = torch.empty((B,), dtype=torch.float64, device="cuda")
st = torch.zeros((B,), dtype=torch.int32, device="cuda")
o1 = _lib.default_options(tol=-1.0)


def it():
    s.iterate(x, u, xn, un, None, st, options=o1, new_cost=pc)


for _ in range(20):
    it()
torch.cuda.synchronize()
res = []
for rep in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        it()
    e1.record()
    torch.cuda.synchronize()
    res.append(e0.elapsed_time(e1) / 200 * 1000)
print(f"{os.path.basename(LIB) if LIB else 'product'}: fused launch {min(res):.1f}-{max(res):.1f} us "
      f"(5 x 200 launches); cost[0..2] {pc[:3].tolist()}", flush=True)
