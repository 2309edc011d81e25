#!/bin/bash
# 2-link forward session: probe variants, the 2-link GPU tests, the config-2 bench (nu 1, 2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tl
export TMPDIR=/tmp
for v in s0_p2 s1_p2 s1_p4; do
  timeout -k 10 60 tools/tl_fw_probe_$v >> gpurun_out/tl/probe.log 2>&1 || { echo "probe $v failed"; exit 1; }
done
timeout -k 10 120 tools/tl_fw_probe_s1_p2 65536 50 >> gpurun_out/tl/probe.log 2>&1 || { echo "probe wide failed"; exit 1; }
cat gpurun_out/tl/probe.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_twolink.py -v --timeout 200 --timeout-method thread > gpurun_out/tl/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error" gpurun_out/tl/pytest.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/bench_twolink.py --nu 1 --no-cpu > gpurun_out/tl/bench_nu1.log 2>&1 && \
timeout -k 10 200 python tools/bench_twolink.py --nu 2 --no-cpu > gpurun_out/tl/bench_nu2.log 2>&1; echo "bench rc=$?"
tail -c 3000 gpurun_out/tl/bench_nu1.log; tail -c 3000 gpurun_out/tl/bench_nu2.log
