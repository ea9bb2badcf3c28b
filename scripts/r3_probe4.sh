#!/usr/bin/env bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 tools/tune_ham3 20 > gpurun_out/ham3_prod.log 2>&1 || exit 1
cat gpurun_out/ham3_prod.log | head -12
timeout -k 10 300 python -u tools/probe_ragged.py 5 > gpurun_out/ragged_probe.log 2>&1 || { cat gpurun_out/ragged_probe.log; exit 1; }
cat gpurun_out/ragged_probe.log
for v in cap new4; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/f1prof_$v -o run --output-format csv -- tools/tune_f1_$v 20 > gpurun_out/f1prof_$v.log 2>&1 || exit 1
  python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/f1prof_$v/**/run_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print('$v', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')
"
done
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_ragged.py tests/test_fastq.py > gpurun_out/pytest_r3d.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r3d.log; exit $rc
