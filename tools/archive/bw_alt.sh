#!/bin/bash
# (Round 3: the -DILQR_* switches below exist only in the restored tree: run this from
# the directory tools/archive/ablation/restore_tree.sh makes.)
# Alternate builds of the backward file (ilqr_bw4.hip) for A/B timing with
# tools/archive/fused_probe.py <lib>: tools/fwalt/libilqr_hip_<name>.so
#   base: the product flags
#   mu0:  μ added in the factorisation (ILQR_BW4_MU_IN_H=0; the product folds it into H)
set -e
cd "$(dirname "$0")/.."
make -C ilqr.jl_amd/csrc > /dev/null
mkdir -p tools/fwalt
O=ilqr.jl_amd/lib/obj
build() {  # build <name> <flags...>
  local n=$1; shift
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 "$@" \
    -c ilqr.jl_amd/csrc/ilqr_bw4.hip -o tools/fwalt/bw4_$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/fwalt/libilqr_hip_$n.so $O/ilqr_lq.hip.o tools/fwalt/bw4_$n.o \
    $O/ilqr_twolink.hip.o $O/ilqr_tiles.hip.o $O/ilqr_chain.hip.o $O/ilqr_abi.cpp.o $O/ilqr_multi.cpp.o -lpthread
}
if [ $# -gt 0 ]; then build "$@"; exit 0; fi
build base
build mu0 -DILQR_BW4_MU_IN_H=0
