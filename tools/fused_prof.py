"""rocprof target: 3-iteration fits, split then fused schedule (tools/fused_probe.py)."""
import os, sys, ctypes as C
import torch
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "ilqr.jl_amd")]
from ilqr_amd import _lib
from ilqr_amd.problems import quadrotor_batch
from ilqr_amd.solver import Solver, _ptr
B, T = 4096, 100
lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
s = Solver(12, 4, T, B); s.set_problem(lq); s._bind_stream()
x, u = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
xo, uo = torch.empty_like(x), torch.empty_like(u)
o3 = _lib.default_options(max_iter=3, tol=-1.0)
for fused in (False, True):
    s.set_schedule(backward="block", fused=fused)
    for _ in range(100):
        s.lib.ilqr_fit(s.h, s._p(), C.byref(o3), _ptr(x), _ptr(u), None, _ptr(xo), _ptr(uo), None, None, None)
torch.cuda.synchronize()
