#!/usr/bin/env bash
# Build the HIP C-ABI library from the WORKING TREE with one source replaced by a given file, into
# shortseq_amd/lib/libshortseq_amd_<tag>.so (a variant kept outside the tree, for `gpu.sh libab`):
#   scripts/build_lib_file.sh new2 ss_counter.hip /tmp/isa/new2.hip
set -euo pipefail
cd "$(dirname "$0")/.."
tag=$1 f=$2 src=$3
tmp=$(mktemp -d)
mkdir -p "$tmp/shortseq_amd"
cp -r shortseq_amd/csrc "$tmp/shortseq_amd/" && cp -r include "$tmp/"
cp "$src" "$tmp/shortseq_amd/csrc/$f"
srcs=$(python3 -c "import sys; sys.path.insert(0, '.'); from shortseq_amd.build import HIP_SOURCES; print(' '.join(HIP_SOURCES))")
args=()
for s in $srcs; do args+=("$tmp/shortseq_amd/csrc/$s"); done
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -mllvm -amdgpu-mfma-vgpr-form=1 \
    -Xarch_host -mbmi2 -Xarch_host -mpopcnt -I "$tmp/include" "${args[@]}" -o "shortseq_amd/lib/libshortseq_amd_$tag.so"
rm -rf "$tmp"
