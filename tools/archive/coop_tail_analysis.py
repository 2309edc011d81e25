"""Critical path of the cooperative line search in the headline's 5-iteration fit, from
the instrumented build (tools/archive/ablation/build_trace_lib.sh
tools/archive/ablation/wave_start_trace.patch): per launch, the waves' start and own-work-done
times, and for every published trajectory its publication (its wave's own-work-done),
each quad of trials handed out (start, end of the pass, end of its finalisation) and
the last wave's exit. Times in µs from the launch's first wave start."""
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
for _ in range(50):
    s.fit(x, u, max_iter=5, tol=-1.0)
torch.cuda.synchronize()
lib.ilqr_debug_trace(buf.ctypes.data_as(C.c_void_p), 262144)
R = None
for k in range(3):
    s.fit(x, u, max_iter=5, tol=-1.0)
    torch.cuda.synchronize()
    n = lib.ilqr_debug_trace(buf.ctypes.data_as(C.c_void_p), 262144)
    R = buf[:n].copy()   # keep the last fit
typ = (R[:, 0] & 15).astype(int)
fin = ((R[:, 0] >> 4) & 15).astype(int)
j0 = ((R[:, 0] >> 8) & 255).astype(int)
lim = ((R[:, 0] >> 16) & 255).astype(int)
ident = ((R[:, 0] >> 24) & 0xFFFFFF).astype(int)
gen = ((R[:, 0] >> 48) & 0xFFFF).astype(int)
t0, t1, t2 = (R[:, i].astype(np.int64) for i in (1, 2, 3))
for g in sorted(set(gen.tolist())):
    m = gen == g
    st = {w: t for w, t in zip(ident[m & (typ == 4)], t0[m & (typ == 4)])}
    if not st:
        continue
    base = min(st.values())
    us = lambda t: (t - base) / 100.0  # noqa: E731
    done = {w: t for w, t in zip(ident[m & (typ == 1)], t0[m & (typ == 1)])}
    leave = t1[m & (typ == 2)]
    dn = np.array([us(t) for t in done.values()])
    last = max(dn.max(), us(leave.max()) if len(leave) else 0)
    q = m & (typ == 3)
    trajs = sorted(set(ident[q].tolist()))
    print(f"gen {g}: {len(st)} waves; own done first {dn.min():.1f} p50 {np.median(dn):.1f} max {dn.max():.1f}; "
          f"last exit {last:.1f} µs; {len(trajs)} searches, {int(q.sum())} quads")
    if not trajs:
        continue
    rows = []
    for b in trajs:
        k = q & (ident == b)
        pub = us(done.get(b // 4, base))
        qs = sorted(zip(j0[k], us(t0[k]), us(t1[k]), us(t2[k]), fin[k], lim[k]))
        f = [r for r in qs if r[4]]
        fe = f[0][3] if f else float("nan")
        rows.append((b, pub, len(qs), qs[0][1], max(r[2] for r in qs), fe, f[0][5] if f else -1))
    rows = np.array(rows, dtype=float)
    print(f"  publish p50 {np.median(rows[:, 1]):.1f} max {rows[:, 1].max():.1f}; first quad start − publish "
          f"p50 {np.median(rows[:, 3] - rows[:, 1]):.1f}; last pass end p50 {np.median(rows[:, 4]):.1f} "
          f"max {rows[:, 4].max():.1f}; finalised p50 {np.nanmedian(rows[:, 5]):.1f} max {np.nanmax(rows[:, 5]):.1f}")
    worst = rows[np.argsort(-np.nan_to_num(rows[:, 5], nan=1e9))[:5]]
    for r in worst:
        b = int(r[0])
        k = q & (ident == b)
        qs = sorted(zip(j0[k], us(t0[k]), us(t1[k]), us(t2[k]), fin[k]))
        print(f"  traj {b}: published {r[1]:.1f}, lim {int(r[6])}, quads " +
              ", ".join(f"j{a}:{s0:.0f}-{s1:.0f}" + (f"+fin-{s2:.0f}" if fn else "") for a, s0, s1, s2, fn in qs))
