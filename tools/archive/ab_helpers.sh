#!/bin/bash
# A/B of the helper-wave build against the product library (one box). The helper library
# is built here first: apply tools/archive/ablation/coop_helpers.patch in a copy of the tree, compile
# ilqr_bw4.hip and ilqr_lq.hip with -DILQR_COOP_HELPERS=1 and link them with the product
# objects into ilqr.jl_amd/lib/libilqr_hip_helpers.so.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
H=$PWD/ilqr.jl_amd/lib/libilqr_hip_helpers.so
PT=$(python -c "import pytest,os;print(os.path.join(os.path.dirname(pytest.__file__),'__main__.py'))")
ILQR_LIB=$H timeout -k 10 300 python -u tools/ab_lib.py $PT tests/test_gpu_line_search.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/hl_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/hl_pytest.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
  MODES=coop timeout -k 10 200 python tools/tail_probe.py > gpurun_out/hl_tail_base_$i.log 2>&1 || exit 1; echo base; grep coop gpurun_out/hl_tail_base_$i.log
  ILQR_LIB=$H MODES=coop timeout -k 10 200 python tools/tail_probe.py > gpurun_out/hl_tail_help_$i.log 2>&1 || exit 1; echo helpers; grep coop gpurun_out/hl_tail_help_$i.log
done
for i in 1 2; do
  timeout -k 10 200 python tools/ab_lib.py bench.py --no-cpu > gpurun_out/hl_bench_base_$i.log 2>&1 || exit 1
  ILQR_LIB=$H timeout -k 10 200 python tools/ab_lib.py bench.py --no-cpu > gpurun_out/hl_bench_help_$i.log 2>&1 || exit 1
  for L in base help; do python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; c=d['co_headline']; print(sys.argv[2], round(d['value'],1), c['value'] if isinstance(c,dict) else c)" gpurun_out/hl_bench_${L}_$i.log $L; done
done
