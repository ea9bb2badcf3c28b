#!/usr/bin/env bash
# Build tools/tune_c5coarse against the production ss_counter.hip and three diagnostic copies of it
# (k_pf_coarse only; their tables are wrong on purpose):
#   nost  the coarse records' global stores cut out (a never-true guard keeps the work that feeds them)
#   l2ld  the tile loads served from the first 128k reads (4 MB: L2 / Infinity Cache, not HBM)
#   both  the two together
set -euo pipefail
cd "$(dirname "$0")/.."
src=shortseq_amd/csrc/ss_counter.hip
tmp=$(mktemp -d)
mkdir -p "$tmp/shortseq_amd"; cp -r shortseq_amd/csrc "$tmp/shortseq_amd/csrc"
cp -r include "$tmp/include"
st='s|((Rec12\*)w.akey)\[at\] = r;|if (r.klo == 0x9E3779B9u \&\& r.khi == 0x7F4A7C15u) ((Rec12*)w.akey)[at] = r;|'
ld='s|min(r0, n - 1) \* stride16|(min(r0, n - 1) \& 0x1FFFFull) * stride16|; s|min(r0 + 32, n - 1) \* stride16|(min(r0 + 32, n - 1) \& 0x1FFFFull) * stride16|'
cp $src "$tmp/shortseq_amd/csrc/prod.hip"
sed "$st" $src > "$tmp/shortseq_amd/csrc/nost.hip"
sed "$ld" $src > "$tmp/shortseq_amd/csrc/l2ld.hip"
sed "$st; $ld" $src > "$tmp/shortseq_amd/csrc/both.hip"
for v in nost l2ld both; do cmp -s $src "$tmp/shortseq_amd/csrc/$v.hip" && { echo "sed changed nothing for $v"; exit 1; }; done
for v in prod nost l2ld both; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I include \
      -DSS_COUNTER_SRC="\"$tmp/shortseq_amd/csrc/$v.hip\"" -DSS_VARIANT="\"$v\"" tools/tune_c5coarse.hip \
      shortseq_amd/csrc/ss_codec.hip shortseq_amd/csrc/ss_runtime.hip -o tools/tune_c5coarse_$v &
done
wait
rm -rf "$tmp"
ls -la tools/tune_c5coarse_*
