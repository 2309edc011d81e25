cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r2a
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_chain.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2a/pytest_new.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python bench.py > gpurun_out/r2a/bench.log 2>&1; echo "bench rc=$?"
tail -c 3000 gpurun_out/r2a/bench.log
grep -E "passed|failed|FAILED|Error" gpurun_out/r2a/pytest_new.log | tail -20
