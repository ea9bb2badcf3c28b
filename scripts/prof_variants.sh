#!/usr/bin/env bash
# Per-kernel times (rocprofv3 kernel trace) of tools/tune_counter_<v> builds, uniform 2^24.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pv
for v in "$@"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pv/$v -o run --output-format csv -- tools/tune_counter_$v 125000000 10 ${ULOG:-24} ${ZIPF:-0} > gpurun_out/pv/$v.log 2>&1 || exit 1
  f=$(find gpurun_out/pv/$v -name "*kernel_stats.csv" | head -1)
  echo "== $v: $(grep insert gpurun_out/pv/$v.log)"
  python3 tools/kstats.py "$f" > gpurun_out/pv/$v.txt
  sed -n 2,6p gpurun_out/pv/$v.txt
done
echo DONE
