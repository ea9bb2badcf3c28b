#!/usr/bin/env bash
# rocprofv3 kernel + HIP runtime API summary of one command (no counters):
#   scripts/prof_api.sh <name> -- <cmd...>      -> gpurun_out/profapi_<name>/ and the top API / kernel rows
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
name=$1; shift; [ "$1" = "--" ] && shift
d=gpurun_out/profapi_$name
mkdir -p $d
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace ${EXTRA:-} --stats -d $d -o run --output-format csv -- "$@" > $d.log 2>&1 || { echo "profapi $name rc=$?"; tail -20 $d.log; exit 1; }
grep -v '^[WE]2' $d.log | tail -12
python3 - "$d" <<'PY'
import csv, glob, sys
for kind in ("hip_api_stats", "kernel_stats", "memory_copy_stats"):
    rows = []
    for f in glob.glob(sys.argv[1] + f"/**/*{kind}.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    print(f"== {kind}")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
        print(f"   {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>6}  tot {float(r['TotalDurationNs'])/1e6:8.3f} ms  {r['Name'][:90]}")
PY
