timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_line_search.py tests/test_gpu_configs.py tests/test_gpu_headline.py > gpurun_out/ls_r05d.log 2>&1 || { tail -20 gpurun_out/ls_r05d.log; exit 1; }
tail -1 gpurun_out/ls_r05d.log
bash tools/archive/r05/ab_acc_r05.sh > gpurun_out/ab_cand1_r05.log 2>&1; cat gpurun_out/ab_cand1_r05.log
