#!/bin/bash
# (Round 3: the -DILQR_* switches below exist only in the restored tree: run this from
# the directory tools/archive/ablation/restore_tree.sh makes.)
# Builds tools/archive/tl_fw_probe.hip in its variants into tools/tl_fw_probe_<variant>:
# s = rollout RK4 (ILQR_TL_RK4_SHIFT), p = prefetch depth (ILQR_FW_GROUP_PF).
# Run on the CPU; the binaries travel to the GPU box.
set -e
cd "$(dirname "$0")"
for v in "0 2" "1 2" "1 4"; do
  set -- $v
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 \
    -DILQR_TL_RK4_SHIFT=$1 -DILQR_FW_GROUP_PF=$2 -Wno-unused-function tl_fw_probe.hip \
    -o tl_fw_probe_s$1_p$2 &
done
wait
