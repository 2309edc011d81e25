#!/bin/bash
# (Round 3: the -DILQR_* switches below exist only in the restored tree: run this from
# the directory tools/archive/ablation/restore_tree.sh makes.)
# Alternate builds of libilqr_hip.so with flags on BOTH files that hold the ring
# forward (ilqr_lq.hip: the split schedule's forward; ilqr_bw4.hip: the fused
# iteration), for A/B timing with tools/archive/fused_probe.py <lib> / tools/archive/gpu_bwab.sh:
#   tools/archive/fw_alt.sh <name> <flags...>   ->  tools/fwalt/libilqr_hip_<name>.so
# e.g. -DILQR_FW_ST_AUX=2 (nt result stores), -DILQR_FW_LD_NT=1 (nt slot loads),
# -DILQR_FW_ABLATE=<bits> (timing-only ablations), -DILQR_FW_LDS_BCAST=1.
set -e
cd "$(dirname "$0")/.."
make -C ilqr.jl_amd/csrc > /dev/null
mkdir -p tools/fwalt
O=ilqr.jl_amd/lib/obj
n=$1; shift
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950"
/opt/rocm/bin/hipcc $F "$@" -c ilqr.jl_amd/csrc/ilqr_lq.hip -o tools/fwalt/lq_$n.o &
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-mfma-vgpr-form=1 "$@" -c ilqr.jl_amd/csrc/ilqr_bw4.hip -o tools/fwalt/bw4_$n.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/fwalt/libilqr_hip_$n.so tools/fwalt/lq_$n.o tools/fwalt/bw4_$n.o \
  $O/ilqr_twolink.hip.o $O/ilqr_tiles.hip.o $O/ilqr_chain.hip.o $O/ilqr_abi.cpp.o $O/ilqr_multi.cpp.o -lpthread
