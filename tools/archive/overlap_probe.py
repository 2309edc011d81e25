"""Does a second set of trajectories per SIMD overlap the fused iteration's phases?
Times one cold ilqr_iterate (the fused lq_iter_fused4 launch) at B = 4096 (one wave per
SIMD) and B = 8192, for the product library and, with ILQR_LIB, a build whose forward
ring is 4 slots deep (PIPE_R = 4, PF = 3: 78 KB of LDS per 4-wave workgroup, so two
workgroups fit a CU and B = 8192 runs two waves per SIMD — one wave's HBM-bound forward
beside the other's issue-bound backward)."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]
from ilqr_amd import _lib
if os.environ.get("ILQR_LIB"):
    _lib._lib = _lib.load(os.environ["ILQR_LIB"])
from ilqr_amd.problems import quadrotor_batch
from ilqr_amd.solver import Solver

T = 100
for B in (4096, 8192):
    lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
    s = Solver(12, 4, T, B)
    s.set_problem(lq)
    s._bind_stream()
    x, u = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
    xn, un = torch.empty_like(x), torch.empty_like(u)
    pc = torch.empty(B, dtype=torch.float64, device="cuda")
    st = torch.zeros(B, dtype=torch.int32, device="cuda")
    o = _lib.default_options(tol=-1.0)
    for _ in range(300):
        s.iterate(x, u, xn, un, None, st, options=o, new_cost=pc)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        s.iterate(x, u, xn, un, None, st, options=o, new_cost=pc)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 200 * 1000
    print(f"{os.path.basename(os.environ.get('ILQR_LIB', 'product'))}: B = {B}: {us:.1f} us per fused iteration, "
          f"{us / (B / 4096):.1f} us per 4096 trajectories", flush=True)
    s.close()
