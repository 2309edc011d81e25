"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; one counter set per pass)
for the backward / forward kernels of bench.py into profiles/pmc_<tag>.json.

Run on the GPU box (see tools/gpu_round.sh `pmc`):
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 5 --warmup 1 --no-cpu
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 5 --warmup 1 --no-cpu
  python profiles/collect_pmc.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/pmc_r01.json

Units: FETCH_SIZE / WRITE_SIZE are KiB per dispatch. Correction per
MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reads exactly half the bytes of
a wide (16 B/lane) coalesced streaming read, so the read side is doubled;
WRITE_SIZE is exact for 16-B streaming stores. Our kernels mix 8-B and 16-B
accesses, so the corrected figure is an estimate (both raw and corrected are kept).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def read(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"]
            key = ("backward" if "lq_iter_backward" in name else
                   "forward" if "lq_iter_forward" in name else
                   "fused" if "lq_iter_fused" in name else
                   "backward_api" if "lq_backward" in name else None)
            if key:
                vals[key].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items() if v}


def main(fetch_dir, write_dir, out):
    fetch = read(fetch_dir, "FETCH_SIZE")
    write = read(write_dir, "WRITE_SIZE")
    res = {"batch": 4096, "T": 100, "units": "bytes per launch",
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, python bench.py"}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, 0.0) * 1024
        w = write.get(k, 0.0) * 1024
        res[k] = {"fetch_raw": f, "write": w, "fetch_x2": 2 * f, "hbm_bytes_corrected": 2 * f + w,
                  "hbm_bytes_raw": f + w}
    be = res.get("backward") or res.get("backward_api")
    if be:
        res["hbm_bytes_per_backward_launch"] = be["hbm_bytes_corrected"]
    if res.get("fused"):
        res["hbm_bytes_per_fused_launch"] = res["fused"]["hbm_bytes_corrected"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
