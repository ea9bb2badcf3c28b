#!/usr/bin/env bash
# Run one GPU step under its own time limit; stop the whole call on a fault/abort/timeout.
# usage: scripts/gpu_step.sh <seconds> <logname> <cmd...>
# exit codes 0 (ok) and 1 (test failures) let the caller continue; anything else ends the call.
set -u
secs=$1; name=$2; shift 2
mkdir -p gpurun_out
echo "=== $name: $*" >&2
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "=== $name rc=$rc" >&2
tail -n 25 "gpurun_out/$name.log" >&2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
  echo "=== $name: fatal rc=$rc, stopping" >&2
  exit 99
fi
exit 0
