"""The headline's 5-iteration fit (SURVEY §8(d) protocol) in a loop, for a kernel trace:
each fit's launches in order (rocprofv3 --kernel-trace), so the per-iteration kernel
durations of the at-floor iterations 4-5 can be read off."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]
from ilqr_amd.problems import quadrotor_batch
from ilqr_amd.solver import Solver

B, T = int(os.environ.get("B", 4096)), 100
N = int(os.environ.get("FITS", 10))
lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
s = Solver(12, 4, T, B)
s.set_problem(lq)
x, u = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
for _ in range(N):
    r = s.fit(x, u, max_iter=5, tol=-1.0)
torch.cuda.synchronize()
print("fits", N, "status counts", torch.bincount(r.status.long()).tolist(), flush=True)
