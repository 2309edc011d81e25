"""Host CPU time held by the end-of-fit wait, one library per
process: `python tools/archive/r05/spin_probe.py [lib.so]`. Per case, median wall ms per fit and
the host CPU ms the calling process used per fit (getrusage: every thread, including
ilqr_multi's shard threads):
  headline  the 3-iteration LQ fit from cold (12×4, T=100, B=4096) — must stay fast;
  config5   ChainSolver.fit with the reference's default options (tol 1e-6) — 9-39 ms;
  multi8    ilqr_multi_fit_resident with 8 shards of 512 on device 0 (a thread each)."""
import ctypes as C
import os
import resource
import sys
import time

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path[:0] = [R, os.path.join(R, "ilqr.jl_amd")]
from ilqr_amd import _lib  # noqa: E402

LIB = sys.argv[1] if len(sys.argv) > 1 else None
if LIB:
    _lib._lib = _lib.load(LIB)
from ilqr_amd.chain import ChainSolver  # noqa: E402
from ilqr_amd.multi import MultiSolver  # noqa: E402
from ilqr_amd.problems import quadrotor_batch  # noqa: E402
from ilqr_amd.solver import Solver, _ptr  # noqa: E402
from ilqr_amd.chain import rbd_2dof_problem, rbd_initial_states  # noqa: E402


def cpu_s():
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


def timed(fn, n):
    for _ in range(3):
        fn()
    walls, cpus = [], []
    for _ in range(n):
        c0, t0 = cpu_s(), time.perf_counter()
        fn()
        walls.append(time.perf_counter() - t0)
        cpus.append(cpu_s() - c0)
    return float(np.median(walls)) * 1e3, float(np.median(cpus)) * 1e3


out = {}
B, T = 4096, 100
lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
s = Solver(12, 4, T, B)
s.set_problem(lq)
s._bind_stream()
x, u = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
xo, uo = torch.empty_like(x), torch.empty_like(u)
o3 = _lib.default_options(max_iter=3, tol=-1.0)
out["headline"] = timed(lambda: s.lib.ilqr_fit(s.h, s._p(), C.byref(o3), _ptr(x), _ptr(u), None, _ptr(xo),
                                               _ptr(uo), None, None, None), 200)
pr = rbd_2dof_problem(1)
cs = ChainSolver(pr, 100, 2048, dtype=torch.float32, linearization="fd", device=0)
xc0 = rbd_initial_states(2048, 2)
uc = torch.zeros((2048, 100, pr.nu), dtype=torch.float32, device="cuda")
xc = cs.rollout(torch.from_numpy(xc0).to("cuda", torch.float32), uc)
out["config5"] = timed(lambda: cs.fit(xc, uc, max_iter=100, tol=1e-6), 20)
ms = MultiSolver([0] * 8, 12, 4, T, B)
ms.set_problem(lq)
ms.load(x0, u0)
out["multi8"] = timed(lambda: ms.fit_resident(max_iter=3, tol=-1.0), 40)
name = os.path.basename(LIB) if LIB else "product"
print(name + ": " + "  ".join(f"{k} wall {w:.3f} ms cpu {c:.3f} ms" for k, (w, c) in out.items()), flush=True)
