"""Forward-pass time against batch (is the ring forward HBM- or latency-bound?)."""
import os, sys, ctypes as C
import torch
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "ilqr.jl_amd")]
from ilqr_amd import _lib
from ilqr_amd.problems import quadrotor_batch
from ilqr_amd.solver import Solver, _ptr

MFMA = "mfma" in sys.argv[1:]  # the forward's MFMA form (ILQR_SCHED_FORWARD_MFMA)
LIBS = [a for a in sys.argv[1:] if a.endswith(".so")]
if LIBS:  # an alternate build of libilqr_hip.so (tools/archive/fw_alt.sh)
    _lib._lib = _lib.load(LIBS[0])
    print("library:", LIBS[0])

for B in (256, 1024, 2048, 4096, 8192):
    lq, x0, u0 = quadrotor_batch(B, T=100, seed0=0)
    s = Solver(12, 4, 100, B); s.set_problem(lq); s._bind_stream(); s.set_schedule(forward_mfma=MFMA)
    x, u = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
    d = torch.empty((B, 100, 4), dtype=torch.float64, device="cuda"); K = torch.empty((B, 100, 4, 12), dtype=torch.float64, device="cuda")
    o = _lib.default_options()
    s.lib.ilqr_backward(s.h, s._p(), C.byref(o), _ptr(x), _ptr(u), _ptr(d), _ptr(K), None)
    pinf = torch.full((B,), float("inf"), dtype=torch.float64, device="cuda")
    xn, un, nc = torch.empty_like(x), torch.empty_like(u), torch.empty_like(pinf)
    fw = lambda: s.lib.ilqr_forward(s.h, s._p(), C.byref(o), _ptr(x), _ptr(u), None, _ptr(d), _ptr(K), _ptr(pinf), _ptr(xn), _ptr(un), _ptr(nc), None, None)
    bw = lambda: s.lib.ilqr_backward(s.h, s._p(), C.byref(o), _ptr(x), _ptr(u), _ptr(d), _ptr(K), None)
    for name, fn in (("forward", fw), ("backward", bw)):
        for _ in range(200): fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); [fn() for _ in range(100)]; e1.record(); torch.cuda.synchronize()
        print(f"B={B:5d} {name:8s} {e0.elapsed_time(e1) * 10:8.2f} us", flush=True)
    s.close()
