"""Summarise a rocprofv3 PMC pass of MFMA counters for bench.py's kernels into
profiles/mfma_<tag>.json (north_star: MFMA utilisation against the gfx950 peak).

Run on the GPU box (one pass, no trace domains):
  rocprofv3 --pmc MfmaUtil MfmaFlopsF64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU GRBM_GUI_ACTIVE \
      --kernel-trace --output-format csv -d gpurun_out/pmc_mfma -o run -- python bench.py --steps 5 --warmup 1 --no-cpu
  python profiles/collect_mfma.py gpurun_out/pmc_mfma profiles/mfma_r02.json

MfmaUtil = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE · SIMDs) in %, MfmaFlopsF64 =
SQ_INSTS_VALU_MFMA_MOPS_F64 · 512 (rocprofv3's derived counters). Per-dispatch values
averaged per kernel; the kernel-trace durations give the achieved MFMA TFLOP/s.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KEYS = (("lq_iter_fused4", "fused"), ("lq_iter_backward4", "backward"), ("lq_backward4", "backward_api"),
        ("lq_iter_forward", "forward"), ("lq_forward", "forward_api"))


def key_of(name):
    for pat, k in KEYS:
        if pat in name:
            return k
    return None


def main(d, out):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = key_of(r["Kernel_Name"])
            if k:
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = key_of(r["Kernel_Name"])
            if k:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    res = {"source": "rocprofv3 --pmc MfmaUtil MfmaFlopsF64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU GRBM_GUI_ACTIVE, "
                     "python bench.py --steps 5 --warmup 1 --no-cpu", "peak_fp64_tflops": 78.6}
    for k, cs in vals.items():
        e = {c: sum(v) / len(v) for c, v in cs.items()}
        if dur.get(k):
            t = sorted(dur[k])[len(dur[k]) // 2]
            e["median_duration_s"] = t
            if "MfmaFlopsF64" in e:
                e["mfma_tflops"] = e["MfmaFlopsF64"] / t / 1e12
                e["mfma_frac_of_peak"] = e["mfma_tflops"] / 78.6
            if "GRBM_GUI_ACTIVE" in e:
                e["effective_clock_ghz"] = e["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
        res[k] = e
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:3])
