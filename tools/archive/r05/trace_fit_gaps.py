"""Summarise a rocprofv3 --kernel-trace of bench.py: the fused iteration kernel's durations
inside the timed region's fits (runs of 3 launches between gathers) against the
back-to-back launch sections after it (runs of > 10), and the per-fit timeline — the
gather and flags kernels and the host turnaround gap before the next fit's first launch.

    python tools/archive/r05/trace_fit_gaps.py gpurun_out/prof/run_kernel_trace.csv
"""
import csv
import sys

import numpy as np


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    runs, cur = [], []
    for r in rows:
        if "lq_iter_fused4" in r["Kernel_Name"]:
            cur.append(r)
        elif cur:
            runs.append(cur)
            cur = []
    if cur:
        runs.append(cur)

    def dur(run):
        return np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in run])
    fits = [dur(r) for r in runs if len(r) == 3]
    if fits:
        f = np.stack(fits)
        print(f"fits (runs of 3 launches): {len(fits)}; fused µs per position {f.mean(0).round(1).tolist()}, "
              f"median {np.median(f):.1f}")
    for r in runs:
        if len(r) > 10:
            d = dur(r)
            print(f"back-to-back section: {len(r)} launches, fused µs mean {d.mean():.1f}, first 5 "
                  f"{d[:5].round(1).tolist()}, last 5 {d[-5:].round(1).tolist()}")
    # per-fit tail: gather, flags, and the gap to the next fused launch
    gaps, gath, flags = [], [], []
    for i, r in enumerate(rows[:-1]):
        if "gather_wg_kernel" in r["Kernel_Name"] and "lq_iter_fused4" in rows[i + 1]["Kernel_Name"]:
            g = (int(rows[i + 1]["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1000
            if g < 200:
                gaps.append(g)
                flags.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
                p = rows[i - 1]
                gath.append((int(r["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1000)  # gap after the last fused
            continue
        if "gather_flags_kernel" in r["Kernel_Name"] and "lq_iter_fused4" in rows[i + 1]["Kernel_Name"]:
            g = (int(rows[i + 1]["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1000
            if g < 200:   # inside a run of fits (not a section boundary)
                gaps.append(g)
                flags.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
                p = rows[i - 1]
                if "gather_kernel" in p["Kernel_Name"]:
                    gath.append((int(p["End_Timestamp"]) - int(p["Start_Timestamp"])) / 1000)
    if gaps and any("gather_wg_kernel" in r["Kernel_Name"] for r in rows):
        print(f"per fit (one-launch gather): gap after the last fused launch {np.median(gath):.1f} µs, "
              f"gather_wg {np.median(flags):.1f} µs, host turnaround {np.median(gaps):.1f} µs "
              f"(median over {len(gaps)} fits)")
    elif gaps:
        print(f"per fit: gather {np.median(gath):.1f} µs, flags {np.median(flags):.1f} µs, host turnaround "
              f"{np.median(gaps):.1f} µs (median over {len(gaps)} fits)")


if __name__ == "__main__":
    main(sys.argv[1])
