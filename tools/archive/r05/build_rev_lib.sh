#!/bin/bash
# Build libilqr_hip.so of another git revision for an A/B on one box:
#   tools/archive/r05/build_rev_lib.sh <rev> <name>  →  tools/fwalt/libilqr_hip_<name>.so
set -e
cd "$(dirname "$0")/../../.."
rev=$1; name=$2
tmp=$(mktemp -d)
git archive "$rev" ilqr.jl_amd/csrc include | tar -x -C "$tmp"
make -s -C "$tmp/ilqr.jl_amd/csrc" -j8 ../lib/libilqr_hip.so
mkdir -p tools/fwalt
cp "$tmp/ilqr.jl_amd/lib/libilqr_hip.so" "tools/fwalt/libilqr_hip_$name.so"
rm -rf "$tmp"
echo "tools/fwalt/libilqr_hip_$name.so"
