"""Per-trajectory record of the headline's chained iterations (ilqr_iterate from cold, as
tools/tail_probe.py): the cost before and after each iteration and its trial count, saved
for the question whether an iteration's relative cost decrease predicts a line search in
the next (the at-floor iterations 4-6). Not product code.

    python tools/floor_probe.py gpurun_out/floor.npz
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]
from ilqr_amd import _lib  # noqa: E402
from ilqr_amd.problems import quadrotor_batch  # noqa: E402
from ilqr_amd.solver import Solver  # noqa: E402

B, T, N = 4096, 100, int(os.environ.get("ITERS", 7))
lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
s = Solver(12, 4, T, B)
s.set_problem(lq)
s._bind_stream()
o = _lib.default_options(tol=-1.0)
xi, ui = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
xn, un = torch.empty_like(xi), torch.empty_like(ui)
pc = torch.full((B,), float("inf"), dtype=torch.float64, device="cuda")
st = torch.zeros(B, dtype=torch.int32, device="cuda")
tr = torch.zeros(B, dtype=torch.int32, device="cuda")
before, after, trials, status = [], [], [], []
for it in range(N):
    before.append(pc.cpu().numpy().copy())
    s.iterate(xi, ui, xn, un, None if it == 0 else pc, st, trials=tr, options=o, new_cost=pc)
    torch.cuda.synchronize()
    after.append(pc.cpu().numpy().copy())
    trials.append(tr.cpu().numpy().copy())
    status.append(st.cpu().numpy().copy())
    keep = st != _lib.TRAJ_OK
    xn[keep] = xi[keep]
    un[keep] = ui[keep]
    tr.zero_()
    xi, xn, ui, un = xn, xi, un, ui
np.savez(sys.argv[1], before=np.array(before), after=np.array(after), trials=np.array(trials), status=np.array(status))
for it in range(N):
    t = trials[it]
    print(f"iteration {it + 1}: searches {(t > 1).sum()}, exhausted {(status[it] == _lib.TRAJ_LS_EXHAUSTED).sum()}",
          flush=True)
