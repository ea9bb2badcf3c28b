#!/usr/bin/env bash
# Many-process A/B of tools/tune_counter_<v> builds (process-to-process spread is ~±5 %: compare
# medians): ROUNDS rounds (default 6) of uniform 2^24 and Zipf 1.1 2^24, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
R=${ROUNDS:-6}
for rep in $(seq 1 $R); do
  for cfg in "24 0" "24 1.1"; do
    for v in "$@"; do
      echo -n "$v $rep: "
      timeout -k 10 120 tools/tune_counter_$v 125000000 15 $cfg || exit 1
    done
  done
done 2>&1 | tee gpurun_out/ab/many.log
python3 - <<'PY'
import re, statistics, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ab/many.log"):
    m = re.match(r"(\S+) \d+: U=2\^(\d+) zipf=([\d.]+): insert avg ([\d.]+)", l)
    if m: d[(m.group(1), m.group(2), m.group(3))].append(float(m.group(4)))
for k in sorted(d): print(k, "median %.3f  min %.3f  n %d" % (statistics.median(d[k]), min(d[k]), len(d[k])))
PY
