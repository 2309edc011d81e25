"""Iteration time with the two-launch and the fused (ILQR_SCHED_FUSED) schedule."""
import os, sys, time, ctypes as C
import torch
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "ilqr.jl_amd")]
from ilqr_amd import _lib
from ilqr_amd.problems import quadrotor_batch
from ilqr_amd.solver import Solver, _ptr
LIBS = [a for a in sys.argv[1:] if a.endswith(".so")]
if LIBS:  # an alternate build of libilqr_hip.so (tools/archive/fw_alt.sh, tools/archive/fw_ab4.sh)
    _lib._lib = _lib.load(LIBS[0])
    print("library:", LIBS[0])

B, T = 4096, 100
lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
s = Solver(12, 4, T, B); s.set_problem(lq); s._bind_stream()
x, u = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
xn, un = torch.empty_like(x), torch.empty_like(u)
pc = torch.empty((B,), dtype=torch.float64, device="cuda")
st = torch.zeros((B,), dtype=torch.int32, device="cuda")
xo, uo = torch.empty_like(x), torch.empty_like(u)
o1 = _lib.default_options(tol=-1.0)
o3 = _lib.default_options(max_iter=3, tol=-1.0)
d = torch.empty((B, T, 4), dtype=torch.float64, device="cuda"); K = torch.empty((B, T, 4, 12), dtype=torch.float64, device="cuda")
def bw(): s.lib.ilqr_backward(s.h, s._p(), C.byref(o1), _ptr(x), _ptr(u), _ptr(d), _ptr(K), None)
def it(): s.iterate(x, u, xn, un, None, st, options=o1, new_cost=pc)
def fit(): s.lib.ilqr_fit(s.h, s._p(), C.byref(o3), _ptr(x), _ptr(u), None, _ptr(xo), _ptr(uo), None, None, None)
for rep in range(3):
    for fused in (False, True):
        s.set_schedule(backward="block", fused=fused)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5: it()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); [it() for _ in range(200)]; e1.record(); torch.cuda.synchronize()
        ms_it = e0.elapsed_time(e1) / 200
        t0 = time.perf_counter(); [fit() for _ in range(60)]; torch.cuda.synchronize()
        ms_fit = (time.perf_counter() - t0) * 1000 / 60 / 3
        e0.record(); [bw() for _ in range(200)]; e1.record(); torch.cuda.synchronize()
        ms_bw = e0.elapsed_time(e1) / 200
        print(f"fused={fused!s:5}  iterate {ms_it*1000:7.1f} us   fit(3) {ms_fit*1000:7.1f} us/iteration   backward {ms_bw*1000:6.1f} us", flush=True)
