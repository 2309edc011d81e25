#!/bin/bash
# cost_functions.jl session: the simple-cost GPU tests, the chain suite (regressions),
# config-5 bench (the closed-form forward now carries the task-cost pointer)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cf
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cost_functions.py tests/test_gpu_chain.py -v --timeout 200 --timeout-method thread > gpurun_out/cf/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error" gpurun_out/cf/pytest.log | tail -40
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_rbd.py --no-cpu > gpurun_out/cf/bench_rbd.log 2>&1
echo "bench rc=$?"
grep -h "^{" gpurun_out/cf/bench_rbd*.log | cut -c1-330
