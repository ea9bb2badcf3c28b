#!/usr/bin/env bash
# F2 engine profile (probe_f2 under rocprofv3 kernel stats) + the multi-word / ragged / drop-in GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-f2q}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag -o run --output-format csv -- python3 -u tools/probe_f2.py 4 > gpurun_out/$tag.log 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/$tag.log; exit 1; }
grep rep gpurun_out/$tag.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ragged.py tests/test_dropin_gpu.py tests/test_fastq.py tests/test_gpu_parity.py -k "multiword or words or ragged or dropin or fastq or growth" > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_pytest.log; exit $rc
