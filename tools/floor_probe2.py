"""Trial 1's cost excess over the cost to beat, (J(α=1) − J_prev) / J_prev, at each
at-floor iteration of the headline's chained fit (ilqr_iterate from cold, as
tools/tail_probe.py), beside the trial count that iteration's line search then needed: is
a deep search (trials ≥ 18, or the 64-trial cap) recognisable when it is published?
Trial 1's cost comes from the same iteration run once more with no cost to beat (every
trajectory accepts trial 1). Not product code.

    python tools/floor_probe2.py gpurun_out/floor2.npz
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

B, T, N = 4096, 100, int(os.environ.get("ITERS", 6))
lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
s = Solver(12, 4, T, B)
s.set_problem(lq)
s._bind_stream()
o = _lib.default_options(tol=-1.0)
xi, ui = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
xn, un = torch.empty_like(xi), torch.empty_like(ui)
xp, up = torch.empty_like(xi), torch.empty_like(ui)
pc = torch.full((B,), float("inf"), dtype=torch.float64, device="cuda")
st = torch.zeros(B, dtype=torch.int32, device="cuda")
tr = torch.zeros(B, dtype=torch.int32, device="cuda")
rec = {}
for it in range(N):
    if it >= 3:
        # trial 1 of this iteration for every open trajectory: no cost to beat
        c1 = torch.full((B,), float("nan"), dtype=torch.float64, device="cuda")
        st1 = st.clone()
        tr1 = torch.zeros_like(tr)
        s.iterate(xi, ui, xp, up, None, st1, trials=tr1, options=o, new_cost=c1)
        torch.cuda.synchronize()
        rec[f"c1_{it + 1}"] = c1.cpu().numpy()
        rec[f"prev_{it + 1}"] = pc.cpu().numpy().copy()
        rec[f"open_{it + 1}"] = (st == _lib.TRAJ_OK).cpu().numpy()
    s.iterate(xi, ui, xn, un, None if it == 0 else pc, st, trials=tr, options=o, new_cost=pc)
    torch.cuda.synchronize()
    rec[f"trials_{it + 1}"] = tr.cpu().numpy().copy()
    rec[f"status_{it + 1}"] = st.cpu().numpy().copy()
    keep = st != _lib.TRAJ_OK
    xn[keep] = xi[keep]
    un[keep] = ui[keep]
    tr.zero_()
    xi, xn, ui, un = xn, xi, un, ui
np.savez(sys.argv[1], **rec)
for it in range(4, N + 1):
    t, c1, p, op = rec[f"trials_{it}"], rec[f"c1_{it}"], rec[f"prev_{it}"], rec[f"open_{it}"]
    ex = (c1 - p) / np.abs(p)
    for name, m in (("accepted at 1", op & (t == 1)), ("trials 2-17", op & (t > 1) & (t < 18)),
                    ("trials 18+", op & (t >= 18))):
        q = np.percentile(ex[m], [0, 10, 50, 90, 100]) if m.sum() else []
        print(f"iteration {it} {name}: n={m.sum()} excess pcts", ["%.2e" % v for v in q], flush=True)
