#!/usr/bin/env bash
# Ablation timings of the C5 insert (tools/tune_counter_<v> built by scripts/build_tune_counter.sh
# with the measurement-only SS_PF_STOP / SS_PF_WRITE / SS_FS_WRITE / SS_PF_DET knobs), uniform 2^24,
# interleaved rounds on one box.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for v in "$@"; do
    echo -n "$v $rep: "
    timeout -k 10 120 tools/tune_counter_$v 125000000 15 24 0 || exit 1
  done
done 2>&1 | tee gpurun_out/ab/ablate.log
echo DONE
