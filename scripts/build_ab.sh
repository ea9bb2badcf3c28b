#!/usr/bin/env bash
# Build a tools/*.hip tuner against the sources of a git revision (A/B on the same box):
#   scripts/build_ab.sh tools/tune_f1.hip HEAD tools/tune_f1_old [extra hipcc flags...]
# The revision's shortseq_amd/csrc + include are exported to a scratch tree; the tool's own file is
# taken from the working tree (its relative includes then resolve to the revision's sources).
set -euo pipefail
cd "$(dirname "$0")/.."
tool=$1 rev=$2 out=$3; shift 3
tmp=$(mktemp -d)
git archive "$rev" shortseq_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$tmp/tools"
cp "$tool" "$tmp/tools/"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -I "$tmp/include" "$@" "$tmp/tools/$(basename "$tool")" -o "$out"
rm -rf "$tmp"
