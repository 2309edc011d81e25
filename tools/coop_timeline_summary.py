"""Reduce tools/coop_timeline.py's trace (gpurun_out/coop_trace.npy) to a per-launch
timeline of the cooperative line search (µs from the launch's first record; the
real-time counter runs at 100 MHz)."""
import collections
import sys

import numpy as np

TICK_US = 0.01
a = np.load(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/coop_trace.npy")
w0 = a[:, 0]
typ, fin = (w0 & 15).astype(int), ((w0 >> 4) & 15).astype(int)
j0, lim = ((w0 >> 8) & 255).astype(int), ((w0 >> 16) & 255).astype(int)
ident, gen = ((w0 >> 24) & 0xFFFFFF).astype(int), ((w0 >> 48) & 0xFFFF).astype(int)
t0, t1, t2 = a[:, 1].astype(np.int64), a[:, 2].astype(np.int64), a[:, 3].astype(np.int64)
for g in sorted(set(gen.tolist())):
    m = gen == g
    base = t0[m].min()
    us = lambda t: (t - base) * TICK_US
    st = us(t0[m & (typ == 1)])
    ins, outs = us(t0[m & (typ == 2)]), us(t1[m & (typ == 2)])
    print(f"gen {g}: own work done {st.min():6.1f}..{st.max():6.1f} us (p50 {np.median(st):6.1f}); "
          f"left the search p50 {np.median(outs):6.1f} p90 {np.percentile(outs, 90):6.1f} max {outs.max():6.1f}")
    q = m & ((typ == 3) | (typ == 4))
    if q.any():
        qs, qe, qf = us(t0[q]), us(t1[q]), us(t2[q])
        d = qe - qs
        wd = typ[q] == 4
        if wd.any():
            print(f"   wide passes {wd.sum()}: pass p50 {np.median(d[wd]):5.1f} max {d[wd].max():5.1f} us, start p50 {np.median(qs[wd]):6.1f}")
        fz = fin[q] == 1
        print(f"   quads {q.sum()}: start {qs.min():6.1f}..{qs.max():6.1f}; pass p50 {np.median(d):5.1f} p90 "
              f"{np.percentile(d, 90):5.1f} max {d.max():5.1f} us; finalised {fz.sum()}, finalise p50 "
              f"{np.median(qf[fz] - qe[fz]) if fz.any() else 0:5.1f} us, last end {qf.max():6.1f}")
        edges = np.arange(0, qf.max() + 25, 25)
        busy = [int(((qs < b1) & (qf > b0_)).sum()) for b0_, b1 in zip(edges[:-1], edges[1:])]
        active = [int(((ins < b1) & (outs > b0_)).sum()) for b0_, b1 in zip(edges[:-1], edges[1:])]
        print("   per 25 us: quads in flight " + " ".join(map(str, busy)))
        print("              waves in search " + " ".join(map(str, active)))
        per_b = collections.defaultdict(list)
        for b, s0, e0, f0, jj, ll, ff in zip(ident[q], qs, qe, qf, j0[q], lim[q], fin[q]):
            per_b[int(b)].append((s0, e0, f0, jj, ll, ff))
        deep = sorted(per_b.items(), key=lambda kv: -len(kv[1]))[:3]
        for b, recs in deep:
            recs.sort()
            print(f"   trajectory {b}: {len(recs)} quads, j0 {[r[3] for r in recs]}, starts "
                  f"{[round(r[0]) for r in recs]}, ends {[round(r[2]) for r in recs]}, lim {recs[-1][4]}")
