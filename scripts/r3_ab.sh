#!/usr/bin/env bash
# same-box A/B of two builds of a tool (interleaved rounds), then optional GPU tests
# usage: scripts/r3_ab.sh <tool_old> <tool_new> <rounds> "<tool args>" [pytest selection...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
old=$1; new=$2; rounds=$3; args=$4; shift 4
for r in $(seq 1 "$rounds"); do
  for b in "$old" "$new"; do
    echo "== round $r $b" >> gpurun_out/ab.log
    timeout -k 10 120 $b $args >> gpurun_out/ab.log 2>&1 || { echo "$b rc=$?"; cat gpurun_out/ab.log; exit 1; }
  done
done
grep -v "^coarse" gpurun_out/ab.log
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/ab_pytest.log 2>&1
  rc=$?; tail -5 gpurun_out/ab_pytest.log; exit $rc
fi
