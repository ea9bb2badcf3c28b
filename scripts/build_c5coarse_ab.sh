#!/usr/bin/env bash
# tools/tune_c5coarse against a git revision's ss_counter.hip ("head") and the working tree's ("new"):
#   scripts/build_c5coarse_ab.sh [rev=HEAD]
set -euo pipefail
cd "$(dirname "$0")/.."
rev=${1:-HEAD}
tmp=$(mktemp -d)
mkdir -p "$tmp/shortseq_amd"
cp -r shortseq_amd/csrc "$tmp/shortseq_amd/csrc"
cp -r include "$tmp/include"
git show "$rev:shortseq_amd/csrc/ss_counter.hip" > "$tmp/shortseq_amd/csrc/head.hip"
cp shortseq_amd/csrc/ss_counter.hip "$tmp/shortseq_amd/csrc/new.hip"
for v in head new; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I include \
      -DSS_COUNTER_SRC="\"$tmp/shortseq_amd/csrc/$v.hip\"" -DSS_VARIANT="\"$v\"" tools/tune_c5coarse.hip \
      shortseq_amd/csrc/ss_codec.hip shortseq_amd/csrc/ss_runtime.hip -o tools/tune_c5coarse_$v &
done
wait
rm -rf "$tmp"
