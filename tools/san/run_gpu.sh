#!/bin/bash
# Host sanitizer runs on a GPU box (prebuilt here by tools/san/run_cpu.sh; device code is
# not instrumented): the ABI driver's GPU paths — fit_ex with history, iterate, the
# multi-device host path and resident calls with their per-shard host threads — under
# ASan+UBSan and under TSan. Each step under its own time limit; stops on a crash-class
# exit. Logs into gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
run() {  # run <name> <cmd...>
  local name=$1; shift
  timeout -k 10 240 "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  return $rc
}
# the HIP runtime is not instrumented: its allocations are not leaks of ours. No
# quarantine: freed device buffers sit in it, and its recycling during the HIP runtime's
# exit-time teardown CHECK-fails in the sanitizer's device allocator
# (dev_runtime_unloaded_) after every check has passed (profiles/r05/san_address_gpu_final_r05.log);
# the CPU run (run_cpu.sh) keeps the quarantine for the host paths.
ASAN_OPTIONS=detect_leaks=0:quarantine_size_mb=0 run san_address ./ilqr.jl_amd/lib/san_address/abi_driver &&
TSAN_OPTIONS="suppressions=tools/san/tsan.supp" run san_thread ./ilqr.jl_amd/lib/san_thread/abi_driver
