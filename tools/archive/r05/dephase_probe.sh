#!/bin/bash
# Timing-only builds of the fused iteration with half of the waves in the other phase
# order (ILQR_FUSED_DEPHASE_PROBE, ilqr_bw4.hip): tools/fwalt/libilqr_hip_dephase{1,2,3,4}.so,
# timed against the product by tools/archive/r05/dephase_probe.py (round 5).
set -e
cd "$(dirname "$0")/../../.."
make -C ilqr.jl_amd/csrc > /dev/null
mkdir -p tools/fwalt
O=ilqr.jl_amd/lib/obj
for v in 1 2 3 4; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 \
    -DILQR_FUSED_DEPHASE_PROBE=$v -c ilqr.jl_amd/csrc/ilqr_bw4.hip -o tools/fwalt/bw4_dephase$v.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/fwalt/libilqr_hip_dephase$v.so \
    $O/ilqr_lq.hip.o tools/fwalt/bw4_dephase$v.o $O/ilqr_twolink.hip.o $O/ilqr_tiles.hip.o \
    $O/ilqr_chain.hip.o $O/ilqr_abi.cpp.o $O/ilqr_multi.cpp.o -lpthread
done
