"""Timeline of the cooperative line search in one 5-iteration headline fit, from a
temporary instrumented build (device trace records: 1 = wave done with its own work,
2 = wave entering/leaving the search, 3 = one evaluated quad of trials with its
finalisation; s_memrealtime ticks) read back through ilqr_debug_trace. The product
library has no such export: this probe runs only against that build."""
import ctypes as C
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]
from ilqr_amd import _lib
from ilqr_amd.problems import quadrotor_batch
from ilqr_amd.solver import Solver

B, T = 4096, 100
lib = _lib.load(os.path.join(ROOT, "ilqr.jl_amd", "lib", "libilqr_hip_trace.so"))
_lib._lib = lib  # the Solver below binds the instrumented build
lib.ilqr_debug_trace.restype = C.c_int
lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
s = Solver(12, 4, T, B)
s.set_problem(lq)
x, u = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
buf = np.zeros((262144, 4), dtype=np.uint64)
for k in range(3):
    torch.cuda.synchronize()
    lib.ilqr_debug_trace(buf.ctypes.data_as(C.c_void_p), 262144)  # reset
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = s.fit(x, u, max_iter=5, tol=-1.0)
    e1.record()
    torch.cuda.synchronize()
    n = lib.ilqr_debug_trace(buf.ctypes.data_as(C.c_void_p), 262144)
    print(f"fit {k}: {e0.elapsed_time(e1):.3f} ms, {n} trace records", flush=True)
np.save(os.path.join(ROOT, "gpurun_out", "coop_trace.npy"), buf[:n])
