#!/bin/bash
# One GPU session: tests, smoke, bench, kernel-trace profile, diagnostics. Each GPU
# step has its own time limit; a crash-class exit (fault/abort/segv/timeout) stops.
# The A/B steps (vanishab, headab, chainab, tlab) compare the product library with
# ilqr.jl_amd/lib/variants/libilqr_hip_prev.so — the previous commit's build, made on the
# CPU before the call:
#   git archive HEAD ilqr.jl_amd/csrc include | tar -x -C /tmp/prev &&
#   make -C /tmp/prev/ilqr.jl_amd/csrc ../lib/libilqr_hip.so &&
#   cp /tmp/prev/ilqr.jl_amd/lib/libilqr_hip.so ilqr.jl_amd/lib/variants/libilqr_hip_prev.so
# (chainab names it libilqr_hip_prevchain.so); spread and tail5 need the instrumented
# build of tools/archive/ablation/build_trace_lib.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for WHAT in "$@"; do
case $WHAT in
  test) step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
        step smoke 180 python -c "import __graft_entry__ as g; g.smoke()" ;;
  bench) step bench 300 python bench.py ;;
  hist) step pytest_hist 400 python -u -m pytest tests/test_gpu_history.py -m gpu -x -v --timeout 200 --timeout-method thread ;;
  ab) step ab 200 python tools/archive/r05/ab_coop.py ;;
  multi) step pytest_multi 400 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -v --timeout 200 --timeout-method thread
         step bench_multi 300 python tools/bench_multi.py ;;
  ls) step pytest_ls 400 python -u -m pytest tests/test_gpu_line_search.py -m gpu -x -v --timeout 200 --timeout-method thread ;;
  cfg) step pytest_cfg 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -s --timeout 200 --timeout-method thread ;;
  smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
  prof) step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 50 --warmup 300 --no-cpu --no-secondary ;;
  ablate) step ablate 120 ./tools/archive/ablate_bw ;;
  dist2) ILQR_DIST_BACKEND=gloo step dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu ;;
  pmc) step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 5 --warmup 1 --no-cpu --no-secondary
       step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 5 --warmup 1 --no-cpu --no-secondary
       python profiles/collect_pmc.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc.json > gpurun_out/pmc_summary.log 2>&1 ;;
  mfma) step pmc_mfma 300 rocprofv3 --pmc MfmaUtil MfmaFlopsF64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_mfma -o run -- python bench.py --steps 5 --warmup 1 --no-cpu --no-secondary
        python profiles/collect_mfma.py gpurun_out/pmc_mfma gpurun_out/mfma.json > gpurun_out/mfma_summary.log 2>&1 ;;
  tl) step pytest_twolink 600 python -m pytest tests/test_gpu_twolink.py -x -q ;;
  tiles) step pytest_tiles 600 python -m pytest tests/test_gpu_tiles.py -x -q ;;
  tlbench) step bench_twolink 300 python tools/bench_twolink.py ;;
  tlprof) step rocprof_twolink 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tl -o run --output-format csv -- python tools/bench_twolink.py --steps 20 --warmup 2 --no-cpu ;;
  chain) step pytest_chain 600 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 120 --timeout-method thread ;;
  rbdbench) step bench_rbd 300 python tools/bench_rbd.py ;;
  rbdprof) step rocprof_rbd 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rbd -o run --output-format csv -- python tools/bench_rbd.py --steps 20 --warmup 5 --no-cpu ;;
  fit5) step tail_probe 200 python tools/tail_probe.py
        step rocprof_fit5 200 rocprofv3 --kernel-trace -d gpurun_out/prof_fit5 -o run --output-format csv -- python tools/archive/r05/fit5_trace.py ;;
  tailcap) MODES=coop MAXT=16 step tail_cap16 200 python tools/tail_probe.py
           MODES=coop MAXT=32 step tail_cap32 200 python tools/tail_probe.py
           MODES=coop MAXT=64 step tail_cap64 200 python tools/tail_probe.py ;;
  ubench) step ubench 120 ./tools/archive/ubench_f64 ;;
  ilp) step tl_ilp 120 ./tools/archive/tl_ilp_probe ;;
  waitab) for i in 1 2; do
            ILQR_FIT_WAIT=sync step bench_wait_sync_$i 300 python bench.py --no-cpu --no-secondary
            step bench_wait_spin_$i 300 python bench.py --no-cpu --no-secondary
          done
          for f in gpurun_out/bench_wait_*.log; do python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[1], round(d['value'],1), round(d['fit_timing']['median_fit_ms']*1000,1), round(d['roofline']['avg_launch_ms']*1000,1))" $f; done ;;
  waitab20) for i in 1 2 3; do
              ILQR_FIT_WAIT=sync step bench20_sync_$i 300 python bench.py --steps 20 --no-cpu --no-secondary
              step bench20_spin_$i 300 python bench.py --steps 20 --no-cpu --no-secondary
            done
            step bench100_spin 300 python bench.py --steps 100 --no-cpu --no-secondary
            for f in gpurun_out/bench20_*.log gpurun_out/bench100_spin.log; do python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[1], round(d['value'],1), 'ms_per_step', round(d['ms_per_step']*1000,2), 'event_us', round(d['iteration']['event_ms']*1000,2), 'traffic', d['roofline']['traffic'])" $f; done > gpurun_out/wait20_ab.log; cat gpurun_out/wait20_ab.log ;;
  w16ab) for i in 1 2; do
           for v in w4 w16; do
             ILQR_LIB=ilqr.jl_amd/lib/variants/libilqr_hip_$v.so step bench_${v}_$i 300 python tools/ab_lib.py bench.py --no-cpu --no-secondary
           done
           step bench_prod_$i 300 python bench.py --no-cpu --no-secondary
         done
         for f in gpurun_out/bench_w4_*.log gpurun_out/bench_w16_*.log gpurun_out/bench_prod_*.log; do python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[1], 'value', round(d['value'],1), 'co_headline', round(d['co_headline']['value'],1), 'fit5_ms', round(d['co_headline']['ms_per_fit'],4), 'dflt', round(d['fit_default_options']['batched_it_per_s'],1), 'status5', d['fit_5_iterations']['trajectory_status_counts'])" $f; done > gpurun_out/w16_ab.log; cat gpurun_out/w16_ab.log ;;
  tailab) for i in 1 2; do
            for v in w4 w16; do
              ILQR_LIB=ilqr.jl_amd/lib/variants/libilqr_hip_$v.so MODES=coop step tail_${v}_$i 200 python tools/tail_probe.py
            done
            MODES=coop step tail_prod_$i 200 python tools/tail_probe.py
          done
          grep -H "coop" gpurun_out/tail_*_[12].log > gpurun_out/tail_ab.log; cat gpurun_out/tail_ab.log ;;
  gatherab) for i in 1 2 3; do for wg in 0 1 4 16; do
              ILQR_GATHER_WG=$wg step ab_fit_wg${wg}_$i 120 python tools/archive/r05/ab_fit.py
            done; done
            grep -h "fit median" gpurun_out/ab_fit_wg*.log > gpurun_out/gather_ab.log; cat gpurun_out/gather_ab.log ;;
  gathertrace) for wg in 0 4; do
                 ILQR_GATHER_WG=$wg step trace_wg$wg 200 rocprofv3 --kernel-trace -d gpurun_out/trace_wg$wg -o run --output-format csv -- python tools/archive/r05/ab_fit.py
                 python tools/archive/r05/trace_fit_gaps.py gpurun_out/trace_wg$wg/run_kernel_trace.csv > gpurun_out/trace_fit_gaps_wg$wg.txt 2>&1
               done ;;
  spread) step wave_spread 200 python tools/archive/wave_spread.py ;;
  chainab) for i in 1 2; do
             ILQR_LIB=ilqr.jl_amd/lib/variants/libilqr_hip_prevchain.so step rbd_prev_$i 200 python tools/ab_lib.py tools/bench_rbd.py --lin fd --no-cpu --steps 50 --warmup 50
             step rbd_new_$i 200 python tools/bench_rbd.py --lin fd --no-cpu --steps 50 --warmup 50
           done
           for f in gpurun_out/rbd_prev_*.log gpurun_out/rbd_new_*.log; do python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; f=d['fit']; print(sys.argv[1], round(d['value'],1), 'fit3', round(f['fit3']['median_ms'],4), 'default', round(f['fit_default']['median_ms'],4), round(f['fit_default']['mean_iterations'],2))" $f; done > gpurun_out/chain_fit_ab.log; cat gpurun_out/chain_fit_ab.log ;;
  vanishab) for i in 1 2; do
              ILQR_LIB=ilqr.jl_amd/lib/variants/libilqr_hip_prev.so MODES=coop step tail_prev_$i 200 python tools/tail_probe.py
              MODES=coop step tail_new_$i 200 python tools/tail_probe.py
            done
            grep -h "coop \|per iteration" gpurun_out/tail_prev_*.log gpurun_out/tail_new_*.log > gpurun_out/vanish_ab.log; cat gpurun_out/vanish_ab.log ;;
  tail5) step coop_tail 200 python tools/archive/coop_tail_analysis.py ;;
  headab) for i in 1 2; do
            ILQR_LIB=ilqr.jl_amd/lib/variants/libilqr_hip_prev.so step ab_fit_prev_$i 120 python tools/archive/r05/ab_fit.py
            step ab_fit_new_$i 120 python tools/archive/r05/ab_fit.py
          done
          grep -h "fit median" gpurun_out/ab_fit_prev_*.log gpurun_out/ab_fit_new_*.log > gpurun_out/head_ab.log; cat gpurun_out/head_ab.log ;;
  tlab) for i in 1 2; do
          ILQR_LIB=ilqr.jl_amd/lib/variants/libilqr_hip_prev.so step tl_prev_$i 200 python tools/ab_lib.py tools/bench_twolink.py --no-cpu
          step tl_new_$i 200 python tools/bench_twolink.py --no-cpu
        done
        for f in gpurun_out/tl_prev_*.log gpurun_out/tl_new_*.log; do python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']; print(sys.argv[1], round(d['value'],1), {k: round(v['avg_launch_ms']*1000,2) for k,v in r.items() if isinstance(v, dict) and 'avg_launch_ms' in v})" $f; done > gpurun_out/tl_ab.log; cat gpurun_out/tl_ab.log ;;
  floating) step pytest_floating 400 python -u -m pytest tests/test_gpu_floating.py -m gpu -x -v --timeout 300 --timeout-method thread
            step bench_floating 300 python tools/bench_floating.py 5 2 1 256 1024
            step rocprof_floating 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fb -o run --output-format csv -- python tools/bench_floating.py 3 1 1 ;;
  fbab) for i in 1 2; do
          ILQR_LIB=ilqr.jl_amd/lib/variants/libilqr_hip_nola.so step fb_nola_$i 200 python tools/ab_lib.py tools/floating_fw_ab.py gpurun_out/fb_nola.npz 1 4 16 64 1024
          step fb_la_$i 200 python tools/floating_fw_ab.py gpurun_out/fb_la.npz 1 4 16 64 1024
        done
        python tools/floating_fw_ab.py --compare gpurun_out/fb_nola.npz gpurun_out/fb_la.npz > gpurun_out/fb_bits.log 2>&1
        grep -H "forward_ms\|bit_equal" gpurun_out/fb_nola_*.log gpurun_out/fb_la_*.log gpurun_out/fb_bits.log > gpurun_out/fb_ab.log; cat gpurun_out/fb_ab.log ;;
  fdeepab) for i in 1 2; do
             ILQR_LIB=ilqr.jl_amd/lib/variants/libilqr_hip_fshallow.so MODES=coop step tail_fshallow_$i 200 python tools/tail_probe.py
             MODES=coop step tail_prod_$i 200 python tools/tail_probe.py
           done
           for i in 1 2; do
             ILQR_LIB=ilqr.jl_amd/lib/variants/libilqr_hip_fshallow.so step bench_fshallow_$i 300 python tools/ab_lib.py bench.py --no-cpu --no-secondary
             step bench_prod_$i 300 python bench.py --no-cpu --no-secondary
           done
           grep -H "coop" gpurun_out/tail_fshallow_*.log gpurun_out/tail_prod_*.log > gpurun_out/fdeep_ab.log
           for f in gpurun_out/bench_fshallow_*.log gpurun_out/bench_prod_*.log; do python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[1], 'value', round(d['value'],1), 'co_headline', round(d['co_headline']['value'],1), 'fit5_ms', round(d['co_headline']['ms_per_fit'],4), 'dflt', round(d['fit_default_options']['batched_it_per_s'],1))" $f; done >> gpurun_out/fdeep_ab.log; cat gpurun_out/fdeep_ab.log ;;
  fbprev) ILQR_LIB=ilqr.jl_amd/lib/variants/libilqr_hip_prev.so step fbp_prev 200 python tools/ab_lib.py tools/floating_fw_ab.py gpurun_out/fbp_prev.npz 1 9 70 1024
          step fbp_new 200 python tools/floating_fw_ab.py gpurun_out/fbp_new.npz 1 9 70 1024
          python tools/floating_fw_ab.py --compare gpurun_out/fbp_prev.npz gpurun_out/fbp_new.npz > gpurun_out/fbp_bits.log 2>&1
          grep -H "forward_ms\|bit_equal" gpurun_out/fbp_prev.log gpurun_out/fbp_new.log gpurun_out/fbp_bits.log > gpurun_out/fbp_ab.log; cat gpurun_out/fbp_ab.log ;;
  tilesab) for i in 1 2; do
            for v in prev new; do
              L=""; [ $v = prev ] && L=ilqr.jl_amd/lib/variants/libilqr_hip_prev.so
              ILQR_LIB=$L TILES_SAVE=gpurun_out/tl_$v step tiles_${v}_1k_$i 200 python tools/ab_lib.py tools/bench_tiles.py 1 1000
              ILQR_LIB=$L TILES_SAVE=gpurun_out/tl_$v step tiles_${v}_4k_$i 200 python tools/ab_lib.py tools/bench_tiles.py 4096 100
            done
          done
          for f in gpurun_out/tl_prev_*.npz; do python tools/floating_fw_ab.py --compare $f ${f/tl_prev/tl_new}; done > gpurun_out/tiles_bits.log 2>&1
          grep -H '"nx"' gpurun_out/tiles_*_[12].log | sed 's/"algorithmic_bytes.*us_per_step/us_per_step/' > gpurun_out/tiles_ab.log; cat gpurun_out/tiles_ab.log gpurun_out/tiles_bits.log | cut -c1-200 ;;
  fbcandfit) for i in 1 2; do
               for c in ${CANDS:-4 16}; do
                 ILQR_FB_CAND=$c step fbfit_c${c}_$i 300 python tools/bench_floating.py 5 2 ${FBB:-256 1024}
               done
             done
             grep -H ms_per_iteration gpurun_out/fbfit_c*.log | sed 's/"workload[^,]*,//' > gpurun_out/fbfit_cand.log; cat gpurun_out/fbfit_cand.log | cut -c1-220 ;;
  fbcand) for c in 4 16 64; do
            ILQR_FB_CAND=$c step fbc_la_c$c 200 python tools/floating_fw_ab.py gpurun_out/fbc_la_c$c.npz 1 64
          done
          grep -H "forward_ms" gpurun_out/fbc_*.log > gpurun_out/fb_cand.log; cat gpurun_out/fb_cand.log ;;
  gtest) step pytest_gather 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_line_search.py tests/test_gpu_multi.py -m gpu -x -q --timeout 120 --timeout-method thread ;;
esac
done
