#!/usr/bin/env bash
# round-3 GPU step: the C5 stream-overlap probe, then the new GPU tests (each step time-limited)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 150 tools/tune_c5pipe 125000000 8 > gpurun_out/c5pipe.log 2>&1 || { echo "c5pipe rc=$?"; exit 1; }
cat gpurun_out/c5pipe.log
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_ragged.py tests/test_dropin_gpu.py "tests/test_fastq.py::test_fastq_gpu_table_growth_multiword" \
  "tests/test_fastq.py::test_fastq_gpu_table_growth" > gpurun_out/pytest_r3a.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_r3a.log
exit $rc
