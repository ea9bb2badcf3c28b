#!/usr/bin/env bash
# A/B the counter tuner binaries given as arguments: rocprofv3 kernel-trace stats per binary, twice.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in "$@"; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/$v.$rep -o run --output-format csv -- tools/tune_counter_$v 125000000 15 > gpurun_out/ab/$v.$rep.log 2>&1 || exit 1
  done
done
echo DONE
