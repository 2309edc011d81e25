#!/bin/bash
# round-2 GPU session: new parity tests, full GPU suite, bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2a
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_chain.py tests/test_gpu_twolink.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r2a/pytest_new.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/r2a/bench.log 2>&1; echo "bench rc=$?"
tail -c 4000 gpurun_out/r2a/bench.log
grep -E "passed|failed|FAILED|Error" gpurun_out/r2a/pytest_new.log | tail -30
