"""HBM traffic of the tiles backward kernels (row f3) from two rocprofv3 PMC passes over
tools/bench_tiles.py (B = 4096, T = 100), beside each kernel's algorithmic bytes.

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/tp_fetch -o run -- python tools/bench_tiles.py
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/tp_write -o run -- python tools/bench_tiles.py
  python tools/archive/r05/pmc_tiles.py gpurun_out/tp_fetch gpurun_out/tp_write profiles/pmc_tiles_r05.json

FETCH_SIZE / WRITE_SIZE are KiB per dispatch. The tiles kernels read with 8-byte loads
(global_load_dwordx2), not the 16-byte streaming reads MI355X_MICROARCH.md's ×2 read
correction is stated for, so both the raw and the doubled read figure are kept.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def algorithmic_bytes(nx, nu, B=4096, T=100):
    # tools/bench_tiles.py's count: the nine tiles in, d and K out, terminal tiles in
    per_step = 8 * (nx * nx + nx * nu + nx + nu + nx * nx + nu * nx + nu * nu)
    return B * T * per_step + B * T * 8 * (nu * nx + nu) + B * 8 * (nx + nx * nx)


def read(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"]
            if "tiles_backward_wide_kernel" in name:
                key = "wide"
            else:
                m = re.search(r"tiles_backward_kernel<(\d+), (\d+)>", name)
                if not m:
                    continue
                key = f"narrow_{m.group(1)}x{m.group(2)}"
            vals[key].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}


def main(fetch_dir, write_dir, out):
    fetch, write = read(fetch_dir, "FETCH_SIZE"), read(write_dir, "WRITE_SIZE")
    shapes = {"narrow_12x4": (12, 4), "wide": (16, 8), "narrow_4x1": (4, 1)}
    res = {"B": 4096, "T": 100, "units": "bytes per launch",
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, python tools/bench_tiles.py"}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, (0.0, 0))[0] * 1024
        w = write.get(k, (0.0, 0))[0] * 1024
        alg = algorithmic_bytes(*shapes[k]) if k in shapes else None
        res[k] = {"launches": fetch.get(k, (0, 0))[1], "fetch_raw": f, "write": w, "hbm_bytes_raw": f + w,
                  "hbm_bytes_fetch_x2": 2 * f + w, "algorithmic_bytes": alg,
                  "raw_over_algorithmic": (f + w) / alg if alg else None}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
