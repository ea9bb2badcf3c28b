#!/usr/bin/env bash
# round-3 probe 7: F1 (nlpos at 62 VGPRs, wide place loads) vs the previous build, then FASTQ parity
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in new5 new11 new5 new11; do
  timeout -k 10 60 tools/tune_f1_$v 30 > gpurun_out/f1_$v.log 2>&1 || { cat gpurun_out/f1_$v.log; exit 1; }
  echo "$v: $(grep -E 'OK|MISMATCH' gpurun_out/f1_$v.log | head -1 | cut -c1-60) $(grep round gpurun_out/f1_$v.log | tr '\n' ' ')"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/f1prof_new11 -o run --output-format csv -- tools/tune_f1_new11 20 > gpurun_out/f1prof_new11.log 2>&1 || exit 1
python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/f1prof_new11/**/run_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print('new11', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')
"
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_fastq.py tests/test_dropin_gpu.py > gpurun_out/pytest_r3m.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r3m.log; exit $rc
