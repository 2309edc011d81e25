#!/bin/bash
# Alternate builds of libilqr_hip.so for tools/fw_scan.py <lib>: the standalone ring
# forward on one-wave workgroups (ILQR_FW_WAVES=1) and forward ablations
# (ILQR_FW_ABLATE bits: 1 no cost row, 2 no x̄ stores), the DPP row broadcasts
# (ILQR_FW_LDS_BCAST=0); the product objects otherwise.
set -e
cd "$(dirname "$0")/.."
make -C ilqr.jl_amd/csrc > /dev/null
mkdir -p tools/fwalt
O=ilqr.jl_amd/lib/obj
build() {  # build <name> <flags...>
  local n=$1; shift
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c ilqr.jl_amd/csrc/ilqr_lq.hip -o tools/fwalt/ilqr_lq_$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/fwalt/libilqr_hip_$n.so tools/fwalt/ilqr_lq_$n.o \
    $O/ilqr_bw4.hip.o $O/ilqr_twolink.hip.o $O/ilqr_tiles.hip.o $O/ilqr_chain.hip.o $O/ilqr_abi.cpp.o $O/ilqr_multi.cpp.o -lpthread
}
build w1 -DILQR_FW_WAVES=1 &
build lds -DILQR_FW_LDS_BCAST=1 &
build ab1 -DILQR_FW_ABLATE=1 &
build ab2 -DILQR_FW_ABLATE=2 &
build ab3 -DILQR_FW_ABLATE=3 &
wait
