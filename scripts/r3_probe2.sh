#!/usr/bin/env bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in cap new2 new3 u4 u16; do
    echo "== f1 $v round $r"
    timeout -k 10 120 tools/tune_f1_$v 30 || exit 1
  done
done > gpurun_out/f1_probe2.log 2>&1
cat gpurun_out/f1_probe2.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/f1prof -o run --output-format csv -- tools/tune_f1_new3 20 > gpurun_out/f1prof.log 2>&1 || exit 1
cat gpurun_out/f1prof/*/run_kernel_stats.csv | cut -d, -f1-4 | head -20
timeout -k 10 200 tools/tune_ham3 30 > gpurun_out/ham3_x4.log 2>&1 || exit 1
cat gpurun_out/ham3_x4.log
