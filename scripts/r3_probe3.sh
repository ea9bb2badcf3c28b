#!/usr/bin/env bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2; do for v in cap new4; do echo "== f1 $v round $r"; timeout -k 10 120 tools/tune_f1_$v 30 || exit 1; done; done > gpurun_out/f1_probe3.log 2>&1
grep -E "==|round 2" gpurun_out/f1_probe3.log
timeout -k 10 200 tools/tune_ham3 30 > gpurun_out/ham3_x3.log 2>&1 || exit 1
cat gpurun_out/ham3_x3.log
