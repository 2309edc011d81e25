"""Per-iteration time of the headline fit's chained iterations (ilqr_iterate, prev_cost
in place, exhausted trajectories keeping their iterate as fit does), cooperative vs
sequential line search, with the trial statistics of each iteration."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]
from ilqr_amd import _lib
from ilqr_amd.problems import quadrotor_batch
from ilqr_amd.solver import Solver
if os.environ.get("ILQR_LIB"):  # A/B against another build of the library
    _lib._lib = _lib.load(os.environ["ILQR_LIB"])

B, T, N = 4096, 100, int(os.environ.get("ITERS", 6))
lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
s = Solver(12, 4, T, B)
s.set_problem(lq)
s._bind_stream()
o = _lib.default_options(tol=-1.0, max_trials=int(os.environ.get("MAXT", 64)))

def run(seq, reps=5):
    s.set_schedule(sequential_search=seq)
    times = np.zeros((reps, N))
    for r in range(reps):
        xi, ui = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
        xn, un = torch.empty_like(xi), torch.empty_like(ui)
        pc = torch.empty(B, dtype=torch.float64, device="cuda")
        st = torch.zeros(B, dtype=torch.int32, device="cuda")
        tr = torch.zeros(B, dtype=torch.int32, device="cuda")
        stats = []
        for it in range(N):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            s.iterate(xi, ui, xn, un, None if it == 0 else pc, st, trials=tr, options=o, new_cost=pc)
            e1.record()
            torch.cuda.synchronize()
            times[r, it] = e0.elapsed_time(e1) * 1000
            t = tr.cpu().numpy(); stn = st.cpu().numpy()
            ran = t > 0
            srch = t[t > 1]
            q = np.percentile(srch, [50, 90, 100]).astype(int).tolist() if srch.size else []
            stats.append((int((t > 1).sum()), int((stn == _lib.TRAJ_LS_EXHAUSTED).sum()), float(t.mean()), q))
            keep = st != _lib.TRAJ_OK
            xn[keep] = xi[keep]; un[keep] = ui[keep]
            tr.zero_()
            xi, xn, ui, un = xn, xi, un, ui
    med = np.median(times, 0)
    print(("sequential" if seq else "coop      "), " ".join(f"{v:7.1f}" for v in med), "us | total",
          f"{med.sum():.0f}", flush=True)
    return stats

MODES = os.environ.get("MODES", "seq,coop").split(",")
for _ in range(2):
    if "seq" in MODES:
        st = run(True)
    if "coop" in MODES:
        st = run(False)
print("per iteration (searches past trial 1, exhausted so far, mean trials, trials p50/p90/max of the searches):", st)
