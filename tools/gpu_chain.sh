#!/bin/bash
# chain session: the chain GPU tests (both evaluators), config-5 bench in both modes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ch
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -v --timeout 200 --timeout-method thread > gpurun_out/ch/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error" gpurun_out/ch/pytest.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_rbd.py --no-cpu > gpurun_out/ch/bench_rbd.log 2>&1 && \
timeout -k 10 300 python tools/bench_rbd.py --no-cpu --dynamics rnea > gpurun_out/ch/bench_rbd_rnea.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ch/prof -o run --output-format csv -- python tools/bench_rbd.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ch/prof.log 2>&1
echo "bench rc=$?"
grep -h "^{" gpurun_out/ch/bench_rbd*.log | cut -c1-330
