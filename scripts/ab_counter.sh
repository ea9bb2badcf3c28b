#!/usr/bin/env bash
# A/B the counter tuner binaries tools/tune_counter_<v> given as arguments, same box, interleaved:
# uniform 2^24 and Zipf 1.1 2^24 (and 2^20 uniform), 3 rounds.  Prints one line per run.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for rep in 1 2 3; do
  for cfg in "24 0" "24 1.1" "20 0"; do
    for v in "$@"; do
      echo -n "$v $rep: "
      timeout -k 10 120 tools/tune_counter_$v 125000000 15 $cfg || exit 1
    done
  done
done 2>&1 | tee gpurun_out/ab/ab.log
echo DONE
