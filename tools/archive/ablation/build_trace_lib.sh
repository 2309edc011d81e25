#!/bin/bash
# Build ilqr.jl_amd/lib/libilqr_hip_trace.so: the product sources with coop_trace.patch
# applied (device timestamps of the cooperative line search, read back by
# ilqr_debug_trace) for tools/archive/coop_timeline.py. Optional extra patches (e.g.
# coop_wide_pass.patch, coop_ranked_stop.patch) are applied first.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
TMP=$(mktemp -d)
mkdir -p "$TMP/ilqr.jl_amd"
cp -r "$ROOT/ilqr.jl_amd/csrc" "$TMP/ilqr.jl_amd/"
cp -r "$ROOT/include" "$TMP/"
for p in "$@"; do (cd "$TMP" && patch -p1 --fuzz=3 -s --no-backup-if-mismatch < "$p"); done
(cd "$TMP" && patch -p1 --fuzz=3 -s --no-backup-if-mismatch < "$ROOT/tools/archive/ablation/coop_trace.patch")
make -j8 -C "$TMP/ilqr.jl_amd/csrc" > /dev/null
cp "$TMP/ilqr.jl_amd/lib/libilqr_hip.so" "$ROOT/ilqr.jl_amd/lib/libilqr_hip_trace.so"
rm -rf "$TMP"
echo "built ilqr.jl_amd/lib/libilqr_hip_trace.so"
