#!/usr/bin/env bash
# same-box per-kernel A/B: rocprofv3 kernel stats of two builds of a tool, interleaved rounds
# usage: scripts/r3_abprof.sh <tool_old> <tool_new> <rounds> "<tool args>" <kernel-name-regex>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/abprof
export TMPDIR=/tmp
old=$1; new=$2; rounds=$3; args=$4; pat=$5
for r in $(seq 1 "$rounds"); do
  for b in "$old" "$new"; do
    d=gpurun_out/abprof/$(basename $b)_$r
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- $b $args > $d.log 2>&1 || { echo "$b rc=$?"; tail -5 $d.log; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    echo "== round $r $(basename $b): $(grep -v '^[WE]2' $d.log | grep -v '^coarse' | head -3 | tr '\n' ' ')"
    python3 - "$f" "$pat" <<'PY'
import csv, re, sys
for row in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], row["Name"]):
        print(f"   {float(row['AverageNs'])/1000:9.1f} us x{row['Calls']:>4}  {row['Name'][:90]}")
PY
  done
done
