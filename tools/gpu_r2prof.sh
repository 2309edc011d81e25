#!/bin/bash
# round-2 profiles: kernel-trace stats of bench.py, PMC HBM passes, 2-link and chain
# kernel-trace stats. Each step has its own limit; a crash-class exit stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2p
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/r2p/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "gpurun_out/r2p/$name.log"; exit $rc; fi
}
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2p/prof -o run --output-format csv -- python bench.py --no-cpu
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r2p/pmc_fetch -o run -- python bench.py --steps 5 --warmup 1 --settle 0 --no-cpu
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r2p/pmc_write -o run -- python bench.py --steps 5 --warmup 1 --settle 0 --no-cpu
python profiles/collect_pmc.py gpurun_out/r2p/pmc_fetch gpurun_out/r2p/pmc_write gpurun_out/r2p/pmc_r02.json > gpurun_out/r2p/pmc_summary.log 2>&1
step prof_tl 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2p/prof_tl -o run --output-format csv -- python tools/bench_twolink.py --nu 1 --steps 50 --warmup 20 --no-cpu
step prof_rbd 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2p/prof_rbd -o run --output-format csv -- python tools/bench_rbd.py --steps 20 --warmup 5 --no-cpu
find gpurun_out/r2p -name "*kernel_stats.csv" | head
tail -c 1500 gpurun_out/r2p/prof.log
