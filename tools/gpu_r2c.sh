#!/bin/bash
# round-2 GPU session: the whole GPU suite, smoke, bench, config-2 and config-5 benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2c
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r2c/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error" gpurun_out/r2c/pytest_gpu.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2c/smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 300 python bench.py > gpurun_out/r2c/bench.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_twolink.py > gpurun_out/r2c/bench_twolink.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_rbd.py > gpurun_out/r2c/bench_rbd.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r2c/bench*.log | cut -c1-400
