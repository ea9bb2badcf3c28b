#!/usr/bin/env bash
# Build the HIP C-ABI library from the WORKING TREE with sed edits applied to one source, into
# shortseq_amd/lib/libshortseq_amd_<tag>.so (a one-knob variant for `gpu.sh libab`):
#   scripts/build_lib_sed.sh fp15 ss_ingest.hip 's/2 \* need_all + 2/need_all + need_all \/ 2 + 2/'
set -euo pipefail
cd "$(dirname "$0")/.."
tag=$1 f=$2; shift 2
tmp=$(mktemp -d)
mkdir -p "$tmp/shortseq_amd"
cp -r shortseq_amd/csrc "$tmp/shortseq_amd/" && cp -r include "$tmp/"
for e in "$@"; do sed -i "$e" "$tmp/shortseq_amd/csrc/$f"; done
if cmp -s "$tmp/shortseq_amd/csrc/$f" "shortseq_amd/csrc/$f"; then echo "sed changed nothing in $f" >&2; exit 1; fi
srcs=$(python3 -c "import sys; sys.path.insert(0, '.'); from shortseq_amd.build import HIP_SOURCES; print(' '.join(HIP_SOURCES))")
args=()
for s in $srcs; do args+=("$tmp/shortseq_amd/csrc/$s"); done
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -mllvm -amdgpu-mfma-vgpr-form=1 \
    -Xarch_host -mbmi2 -Xarch_host -mpopcnt -I "$tmp/include" "${args[@]}" -o "shortseq_amd/lib/libshortseq_amd_$tag.so"
rm -rf "$tmp"
