#!/usr/bin/env bash
# Build the HIP C-ABI library from the WORKING TREE with some sources taken from a git revision, into
# shortseq_amd/lib/libshortseq_amd_<tag>.so (same-box A/B of one change among several, `gpu.sh libab`):
#   scripts/build_lib_mix.sh vq HEAD:ss_codec.hip        (working tree, but ss_codec.hip of HEAD)
set -euo pipefail
cd "$(dirname "$0")/.."
tag=$1; shift
tmp=$(mktemp -d)
mkdir -p "$tmp/shortseq_amd"
cp -r shortseq_amd/csrc "$tmp/shortseq_amd/" && cp -r include "$tmp/"
for spec in "$@"; do
  rev=${spec%%:*} f=${spec#*:}
  git show "$rev:shortseq_amd/csrc/$f" > "$tmp/shortseq_amd/csrc/$f"
done
srcs=$(python3 -c "import sys; sys.path.insert(0, '.'); from shortseq_amd.build import HIP_SOURCES; print(' '.join(HIP_SOURCES))")
args=()
for f in $srcs; do args+=("$tmp/shortseq_amd/csrc/$f"); done
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -mllvm -amdgpu-mfma-vgpr-form=1 \
    -Xarch_host -mbmi2 -Xarch_host -mpopcnt -I "$tmp/include" "${args[@]}" -o "shortseq_amd/lib/libshortseq_amd_$tag.so"
rm -rf "$tmp"
