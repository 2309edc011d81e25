# A/B of the forward's DPP dot accumulators (round 5): the product build against
# tools/fwalt/libilqr_hip_base.so (the previous commit), the bench without CPU
# baseline / secondary configs, alternated twice on one box.
set -o pipefail
for rep in 1 2; do
  for lib in "" tools/fwalt/libilqr_hip_base.so; do
    out=gpurun_out/ab_acc_${rep}_$(basename "${lib:-product}").json
    ILQR_LIB=$lib timeout -k 10 200 python -u tools/ab_lib.py bench.py --no-cpu --no-secondary --steps 100 > "$out" 2>/dev/null || exit 1
    python -c "import json,sys; d=json.loads([l for l in open('$out') if l.startswith('{')][-1]); print('${lib:-product}', round(d['value']), 'co', round(d['co_headline']['value']), 'fused_us', round(d['roofline']['avg_launch_ms']*1000,1), 'fw_us', round(d['forward_kernel']['avg_launch_ms']*1000,1), 'all_ok', d['iteration']['all_ok'], 'trials', [round(t,3) for t in d['fit_5_iterations']['line_search_trials_per_iteration']], 'fit5 status', d['fit_5_iterations']['trajectory_status_counts'])"
  done
done
