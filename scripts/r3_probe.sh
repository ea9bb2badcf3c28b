#!/usr/bin/env bash
# GPU probes: F1 one-pass index old / new / fixed-slot variants, C5 stream overlap and grid oversubscription
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in old new cap; do
    echo "== f1 $v round $r"
    timeout -k 10 120 tools/tune_f1_$v 30 || exit 1
  done
done > gpurun_out/f1_probe.log 2>&1
cat gpurun_out/f1_probe.log
timeout -k 10 200 tools/tune_c5pipe 125000000 8 > gpurun_out/c5pipe2.log 2>&1 || exit 1
cat gpurun_out/c5pipe2.log
timeout -k 10 200 tools/tune_ham3 30 > gpurun_out/ham3_glds.log 2>&1 || exit 1
cat gpurun_out/ham3_glds.log
