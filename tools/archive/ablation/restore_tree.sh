#!/bin/bash
# Copy the sources (ilqr.jl_amd/csrc, include, tools) into DIR and apply
# restore_alternates.patch there: the tree the round-1/2 A/B scripts and probes were
# written against (tools/archive/bw_alt.sh, fw_alt.sh, fw_ab4.sh, tl_fw_probe.sh, ablate_bw.hip,
# bw4_probe.hip, bw8_probe.hip, tl_fw_probe.hip: their -DILQR_* switches and ABL bits).
# Run those scripts from DIR. The product tree holds one path per kernel.
set -euo pipefail
DIR=${1:?usage: restore_tree.sh DIR}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p "$DIR/ilqr.jl_amd"
cp -r "$ROOT/ilqr.jl_amd/csrc" "$DIR/ilqr.jl_amd/"
cp -r "$ROOT/include" "$ROOT/tools" "$DIR/"
(cd "$DIR" && patch -p1 --fuzz=3 --no-backup-if-mismatch -s < "$ROOT/tools/archive/ablation/restore_alternates.patch")
echo "restored tree in $DIR"
