#!/usr/bin/env bash
# round-3 probe 6: length-class tables in the drop-in engine — parity first, then the f2 timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_ragged.py tests/test_dropin_gpu.py tests/test_fastq.py "tests/test_gpu_parity.py::test_counter_insert_words" \
  "tests/test_gpu_parity.py::test_counter_multiword" > gpurun_out/pytest_r3r.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_r3r.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_ragged.py 5 > gpurun_out/ragged_probe10.log 2>&1 || { cat gpurun_out/ragged_probe10.log; exit 1; }
cat gpurun_out/ragged_probe10.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/f2prof10 -o run --output-format csv -- python3 -u tools/probe_f2.py 4 > gpurun_out/f2prof10.log 2>&1 || { tail -20 gpurun_out/f2prof10.log; exit 1; }
grep "^rep" gpurun_out/f2prof10.log
python3 - <<'PY'
import csv, glob
rows = []
for f in glob.glob('gpurun_out/f2prof10/**/run_kernel_stats.csv', recursive=True):
    rows += list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print('kernel total ms over all reps', round(tot / 1e6, 2), 'launches', sum(int(r['Calls']) for r in rows))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:25]:
    print(r['Name'][:60], r['Calls'], round(float(r['TotalDurationNs']) / 1e6, 3), 'ms', round(float(r['AverageNs']) / 1e3, 2), 'us')
PY
