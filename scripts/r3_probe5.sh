#!/usr/bin/env bash
# round-3 probe 5: F1 read ceiling (tools/tune_nl), ragged encode (scratch-free loader), the f2
# engine's wall time vs its kernels (rocprofv3 kernel trace)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/tune_nl 1979711488 30 > gpurun_out/tune_nl.log 2>&1 || { cat gpurun_out/tune_nl.log; exit 1; }
cat gpurun_out/tune_nl.log
timeout -k 10 300 python -u tools/probe_ragged.py 5 > gpurun_out/ragged_probe5.log 2>&1 || { cat gpurun_out/ragged_probe5.log; exit 1; }
cat gpurun_out/ragged_probe5.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/f2prof -o run --output-format csv -- python3 -u tools/probe_f2.py 4 > gpurun_out/f2prof.log 2>&1 || { tail -20 gpurun_out/f2prof.log; exit 1; }
grep "^rep" gpurun_out/f2prof.log
python3 - <<'PY'
import csv, glob
rows = []
for f in glob.glob('gpurun_out/f2prof/**/run_kernel_stats.csv', recursive=True):
    rows += list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print('kernel total ms over all reps', round(tot / 1e6, 2), 'launches', sum(int(r['Calls']) for r in rows))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:25]:
    print(r['Name'][:60], r['Calls'], round(float(r['TotalDurationNs']) / 1e6, 3), 'ms', round(float(r['AverageNs']) / 1e3, 2), 'us')
PY
