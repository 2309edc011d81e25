#!/bin/bash
# A/B of tools/archive/bw_alt.sh builds on the GPU box (timing only): fused_probe per library,
# two passes in alternating order
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for pass in 1 2; do
  for n in "$@"; do
    echo "=== $n (pass $pass)"
    timeout -k 10 120 python -u tools/archive/fused_probe.py tools/fwalt/libilqr_hip_$n.so || exit $?
  done
done
