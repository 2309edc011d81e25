#!/bin/bash
# Builds tools/archive/tl_ilp_probe (run on the CPU; the binary travels to the GPU box).
cd "$(dirname "$0")" && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 \
  -Wno-unused-function tl_ilp_probe.hip -o tl_ilp_probe
