export TMPDIR=/tmp
# Archived (round 6): the scratch experiments behind profiles/r06/coop_*; the variant
# libraries it names (qreg, scr1024, nodeep) were built by hand and are gone.
V=ilqr.jl_amd/lib/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_line_search.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ls_deep.log 2>&1 || exit 1
ILQR_LIB=$V/libilqr_hip_trace.so timeout -k 10 120 python tools/coop_trace.py > gpurun_out/ct_deep.log 2>&1 || exit 1
ILQR_LIB=$V/libilqr_hip_nodeep_trace.so timeout -k 10 120 python tools/coop_trace.py > gpurun_out/ct_nodeep.log 2>&1 || exit 1
for i in 1 2; do
  ILQR_LIB=$V/libilqr_hip_nodeep.so MODES=coop timeout -k 10 120 python tools/tail_probe.py > gpurun_out/tp_nodeep_$i.log 2>&1 || exit 1
  MODES=coop timeout -k 10 120 python tools/tail_probe.py > gpurun_out/tp_deep_$i.log 2>&1 || exit 1
done
echo done
