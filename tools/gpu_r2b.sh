#!/bin/bash
# round-2 GPU session: the whole GPU suite, smoke, bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2b
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r2b/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error" gpurun_out/r2b/pytest_gpu.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2b/smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 300 python bench.py > gpurun_out/r2b/bench.log 2>&1; echo "bench rc=$?"
tail -c 5000 gpurun_out/r2b/bench.log
