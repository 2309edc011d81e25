#!/bin/bash
# A/B of whole-library builds on the GPU box (timing only): runs <cmd> with the product
# library, then with each tools/fwalt/libilqr_hip_<name>.so copied over it, twice.
#   tools/archive/gpu_libab.sh "<cmd>" <name>...
set -o pipefail
cd "$(dirname "$0")/.."
CMD=$1; shift
LIB=ilqr.jl_amd/lib/libilqr_hip.so
cp $LIB /tmp/libilqr_hip_product.so
for pass in 1 2; do
  echo "=== product (pass $pass)"; cp /tmp/libilqr_hip_product.so $LIB
  timeout -k 10 200 $CMD || exit $?
  for n in "$@"; do
    echo "=== $n (pass $pass)"; cp tools/fwalt/libilqr_hip_$n.so $LIB
    timeout -k 10 200 $CMD || exit $?
  done
done
cp /tmp/libilqr_hip_product.so $LIB
