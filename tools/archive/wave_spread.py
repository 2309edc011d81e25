"""Per-wave timing of the fused iteration kernel in the headline fit (B = 4096, T = 100),
from the instrumented build (tools/archive/ablation/build_trace_lib.sh
tools/archive/ablation/wave_start_trace.patch): every wave records its start (with its hardware
slot: HW_ID, XCC_ID) and the end of its own work (backward + forward), s_memrealtime
ticks (100 MHz). Question: is the spread of the waves' finishing times (the launch's
ramp-down) the same waves every launch (placement: XCD, CU) or random — only the latter
would a persistent multi-iteration kernel recover."""
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
_lib._lib = lib
lib.ilqr_debug_trace.restype = C.c_int
lq, x0, u0 = quadrotor_batch(B, T=T, seed0=0)
s = Solver(12, 4, T, B)
s.set_problem(lq)
x, u = torch.from_numpy(x0).cuda(), torch.from_numpy(u0).cuda()
buf = np.zeros((262144, 4), dtype=np.uint64)
for _ in range(200):          # clock run-in
    s.fit(x, u, max_iter=4, tol=-1.0)
torch.cuda.synchronize()
lib.ilqr_debug_trace(buf.ctypes.data_as(C.c_void_p), 262144)   # reset
recs = []
for k in range(10):
    s.fit(x, u, max_iter=4, tol=-1.0)   # launches 2-4 carry the search: traced
    torch.cuda.synchronize()
    n = lib.ilqr_debug_trace(buf.ctypes.data_as(C.c_void_p), 262144)
    recs.append(buf[:n].copy())
R = np.concatenate(recs)
typ = (R[:, 0] & 15).astype(int)
wid = ((R[:, 0] >> 24) & 0xFFFFFF).astype(int)
gen = ((R[:, 0] >> 48) & 0xFFFF).astype(int)
t = R[:, 1].astype(np.int64)
gens = sorted(set(gen[typ == 4].tolist()))
print(f"{len(gens)} traced launches")
dur_all, done_rel_all = [], []
xcc_of, hw_of = {}, {}
for g in gens:
    st = {w: (tt, r2, r3) for w, tt, r2, r3 in zip(wid[(typ == 4) & (gen == g)], t[(typ == 4) & (gen == g)],
                                                   R[(typ == 4) & (gen == g), 2], R[(typ == 4) & (gen == g), 3])}
    dn = dict(zip(wid[(typ == 1) & (gen == g)], t[(typ == 1) & (gen == g)]))
    ws = sorted(set(st) & set(dn))
    t0 = min(st[w][0] for w in ws)
    starts = np.array([st[w][0] - t0 for w in ws]) / 100.0     # µs
    dones = np.array([dn[w] - t0 for w in ws]) / 100.0
    dur = dones - starts
    for w in ws:
        xcc_of[w] = int(st[w][2]) & 15
        hw_of[w] = int(st[w][1])
    dur_all.append(dict(zip(ws, dur)))
    done_rel_all.append(dict(zip(ws, dones)))
    print(f"gen {g}: {len(ws)} waves; start spread {starts.max():.1f} µs; done first {dones.min():.1f} "
          f"p10 {np.percentile(dones, 10):.1f} p50 {np.median(dones):.1f} p90 {np.percentile(dones, 90):.1f} "
          f"max {dones.max():.1f}; wave duration p10 {np.percentile(dur, 10):.1f} p50 {np.median(dur):.1f} "
          f"p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f} µs")
ws = sorted(set.intersection(*[set(d) for d in dur_all]))
M = np.array([[d[w] for w in ws] for d in dur_all])        # launches × waves
D = np.array([[d[w] for w in ws] for d in done_rel_all])
print(f"mean over launches of the last wave's finish: {D.max(1).mean():.1f} µs; "
      f"max over waves of each wave's mean finish: {D.mean(0).max():.1f} µs; "
      f"mean finish {D.mean():.1f} µs")
c = np.corrcoef(M)
print(f"wave-duration correlation between launches: mean off-diagonal {c[~np.eye(len(c), dtype=bool)].mean():.2f}")
# placement: by XCC
xcc = np.array([xcc_of[w] for w in ws])
for k in sorted(set(xcc.tolist())):
    print(f"  XCC {k}: {int((xcc == k).sum())} waves, mean duration {M[:, xcc == k].mean():.1f} µs, "
          f"mean finish {D[:, xcc == k].mean():.1f} µs")
# a persistent kernel's bound: each wave runs its launches back to back
seq = M.sum(0)
print(f"sum over {len(M)} launches: per-launch max-finish total {D.max(1).sum():.1f} µs vs "
      f"max over waves of summed durations {seq.max():.1f} µs (+ start spread)")
np.savez(os.path.join(ROOT, "gpurun_out", "wave_spread.npz"), wid=np.array(ws), dur=M, done=D,
         hw_id=np.array([hw_of[w] for w in ws]), xcc=xcc)
