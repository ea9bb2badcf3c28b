#!/usr/bin/env bash
# Build the HIP C-ABI library of a git revision into shortseq_amd/lib/libshortseq_amd_<tag>.so for a
# same-box A/B with `scripts/gpu.sh libab` (which swaps it with the working tree's build):
#   scripts/build_lib_rev.sh HEAD~1 old
set -euo pipefail
cd "$(dirname "$0")/.."
rev=$1 tag=$2
tmp=$(mktemp -d)
git archive "$rev" shortseq_amd/csrc include | tar -x -C "$tmp"
srcs=$(python3 -c "import sys; sys.path.insert(0, '.'); from shortseq_amd.build import HIP_SOURCES; print(' '.join(HIP_SOURCES))")
args=()
for f in $srcs; do args+=("$tmp/shortseq_amd/csrc/$f"); done
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -mllvm -amdgpu-mfma-vgpr-form=1 \
    -Xarch_host -mbmi2 -Xarch_host -mpopcnt -I "$tmp/include" "${args[@]}" -o "shortseq_amd/lib/libshortseq_amd_$tag.so"
rm -rf "$tmp"
