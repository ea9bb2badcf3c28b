#!/usr/bin/env bash
# same-box A/B of two builds of the HIP library through a python driver script (interleaved
# rounds; the in-tree library file is swapped between runs), then GPU tests on the new build
# usage: scripts/r3_libab.sh <rounds> "<python cmd>" [pytest selection...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rounds=$1; cmd=$2; shift 2
L=shortseq_amd/lib
cp $L/libshortseq_amd.so $L/libshortseq_amd_new.so
for r in $(seq 1 "$rounds"); do
  for v in old new; do
    cp $L/libshortseq_amd_$v.so $L/libshortseq_amd.so
    echo "== round $r $v: $(timeout -k 10 300 $cmd 2>&1 | tail -1)" | tee -a gpurun_out/libab.log
  done
done
cp $L/libshortseq_amd_new.so $L/libshortseq_amd.so
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/libab_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/libab_pytest.log; exit $rc
fi
