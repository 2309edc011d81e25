#!/bin/bash
# (Round 3: the -DILQR_* switches below exist only in the restored tree: run this from
# the directory tools/archive/ablation/restore_tree.sh makes.)
# Ablation build: the fused iteration and the ring forward without the K δx product
# (ILQR_FW_ABLATE=4, wrong results; timing only) -> tools/fwalt/libilqr_hip_ab$AB.so
set -e
AB=${1:-4}
cd "$(dirname "$0")/.."
make -C ilqr.jl_amd/csrc > /dev/null
mkdir -p tools/fwalt
O=ilqr.jl_amd/lib/obj
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -DILQR_FW_ABLATE=$AB"
/opt/rocm/bin/hipcc $F -c ilqr.jl_amd/csrc/ilqr_lq.hip -o tools/fwalt/lq_ab$AB.o &
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-mfma-vgpr-form=1 -c ilqr.jl_amd/csrc/ilqr_bw4.hip -o tools/fwalt/bw4_ab$AB.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/fwalt/libilqr_hip_ab$AB.so tools/fwalt/lq_ab$AB.o tools/fwalt/bw4_ab$AB.o \
  $O/ilqr_twolink.hip.o $O/ilqr_tiles.hip.o $O/ilqr_chain.hip.o $O/ilqr_abi.cpp.o $O/ilqr_multi.cpp.o -lpthread
