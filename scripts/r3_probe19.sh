#!/usr/bin/env bash
# F1 staging run size (kTileCap) sweep, alternating builds on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in 2048 1024 1280 1536 2048 1024 1280 1536; do
  timeout -k 10 60 tools/tune_f1_cap$v 30 > gpurun_out/f1_cap$v.log 2>&1 || { cat gpurun_out/f1_cap$v.log; exit 1; }
  echo "cap $v: $(grep -E 'OK|MISMATCH' gpurun_out/f1_cap$v.log | head -1 | grep -o 'offsets+lens [A-Z]*') $(grep 'round 2' gpurun_out/f1_cap$v.log)"
done
