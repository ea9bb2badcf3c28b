#!/usr/bin/env bash
# class-table sizing hook + counter / ragged / drop-in parity
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_ragged.py tests/test_dropin_gpu.py tests/test_fastq.py "tests/test_gpu_parity.py::test_counter_insert_words" \
  "tests/test_gpu_parity.py::test_counter_multiword" "tests/test_gpu_parity.py::test_counter_multiword_bad_read" > gpurun_out/pytest_r3s.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_r3s.log | grep -E "undersized|FAIL|ERROR" ; tail -3 gpurun_out/pytest_r3s.log; exit $rc
