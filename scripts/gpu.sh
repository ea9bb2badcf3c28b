#!/usr/bin/env bash
# One parameterised entry point for the GPU calls used while tuning (replaces round 3's r3_* scripts).
# Every GPU step runs under its own time limit; a failing step ends the call (no retries).
#
#   scripts/gpu.sh pytest <secs> <pytest selection...>           -m gpu tests, log gpurun_out/pytest_<TAG>.log
#   scripts/gpu.sh ab <rounds> "<args>" <tool_a> <tool_b> ...    interleaved same-box runs of tuner binaries
#   scripts/gpu.sh abprof <rounds> "<args>" <regex> <tool>...    the same under rocprofv3 kernel stats (kernels ~ regex)
#   scripts/gpu.sh libab <rounds> "<python cmd>" [variants..]    in-tree libshortseq_amd.so ("new") vs
#                                                                libshortseq_amd_<v>.so (default: old new)
#   scripts/gpu.sh prof <name> <regex> -- <cmd...>               rocprofv3 kernel-trace summary of one command
#   scripts/gpu.sh pmc <name> "<counters>" -- <cmd...>           one rocprofv3 --pmc pass (kernel rows grouped)
#   scripts/gpu.sh full                                          whole GPU suite, then the default bench line
#   scripts/gpu.sh profall                                       bench + rocprof kernel stats + FETCH/WRITE passes
# TAG (env, default "x") names the logs. Steps can be chained in one call with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-x}
mode=$1; shift

stats() {  # stats <kernel_stats.csv dir> <regex>
  python3 - "$1" "$2" <<'PY'
import csv, glob, re, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if re.search(sys.argv[2], r["Name"]):
        print(f"   {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>5}  tot {float(r['TotalDurationNs'])/1e6:8.3f} ms  {r['Name'][:100]}")
PY
}

case $mode in
pytest)
  secs=$1; shift
  timeout -k 10 "$secs" python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; tail -15 gpurun_out/pytest_$TAG.log; exit $rc ;;
ab)
  rounds=$1; args=$2; shift 2
  for r in $(seq 1 "$rounds"); do
    for b in "$@"; do
      echo "== round $r $b" >> gpurun_out/ab_$TAG.log
      timeout -k 10 150 $b $args >> gpurun_out/ab_$TAG.log 2>&1 || { echo "$b rc=$?"; tail -20 gpurun_out/ab_$TAG.log; exit 1; }
    done
  done
  cat gpurun_out/ab_$TAG.log ;;
abprof)
  rounds=$1; args=$2; pat=$3; shift 3
  for r in $(seq 1 "$rounds"); do
    for b in "$@"; do
      d=gpurun_out/abprof_$TAG/$(basename $b)_$r
      mkdir -p $d
      timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- $b $args > $d.log 2>&1 || { echo "$b rc=$?"; tail -5 $d.log; exit 1; }
      echo "== round $r $(basename $b): $(grep -v '^[WE]2' $d.log | head -3 | tr '\n' ' ')"
      stats $d "$pat"
    done
  done ;;
libab)
  rounds=$1; cmd=$2; shift 2
  vs=${*:-old new}
  export SHORTSEQ_AMD_LENIENT_ABI=1
  L=shortseq_amd/lib
  cp $L/libshortseq_amd.so $L/libshortseq_amd_new.so
  # the real library goes back however the loop ends (a killed run left a variant installed)
  trap "cp $L/libshortseq_amd_new.so $L/libshortseq_amd.so" EXIT
  for r in $(seq 1 "$rounds"); do
    for v in $vs; do
      cp $L/libshortseq_amd_$v.so $L/libshortseq_amd.so
      echo "== round $r $v: $(timeout -k 10 300 $cmd 2>&1 | tail -1)" | tee -a gpurun_out/libab_$TAG.log
    done
  done
  cp $L/libshortseq_amd_new.so $L/libshortseq_amd.so ;;
libtest)      # libtest <variant> <secs> <pytest selection...>: the -m gpu tests against libshortseq_amd_<variant>.so
  v=$1; secs=$2; shift 2
  L=shortseq_amd/lib
  cp $L/libshortseq_amd.so $L/libshortseq_amd_new.so
  trap "cp $L/libshortseq_amd_new.so $L/libshortseq_amd.so" EXIT
  cp $L/libshortseq_amd_$v.so $L/libshortseq_amd.so
  timeout -k 10 "$secs" python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/pytest_${TAG}_$v.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_${TAG}_$v.log; exit $rc ;;
libprof)      # libprof <name> <regex> "<variants>" -- <cmd...>: rocprof kernel stats of cmd per library variant
  name=$1; pat=$2; vs=$3; shift 3; [ "$1" = "--" ] && shift
  L=shortseq_amd/lib
  cp $L/libshortseq_amd.so $L/libshortseq_amd_new.so
  trap "cp $L/libshortseq_amd_new.so $L/libshortseq_amd.so" EXIT
  for v in $vs; do
    cp $L/libshortseq_amd_$v.so $L/libshortseq_amd.so
    d=gpurun_out/prof_${name}_$v
    mkdir -p $d
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- "$@" > $d.log 2>&1 || { echo "libprof $v rc=$?"; tail -20 $d.log; exit 1; }
    echo "== $v: $(grep -v '^[WE]2' $d.log | tail -1)"
    stats $d "$pat"
  done ;;
prof)
  name=$1; pat=$2; shift 2; [ "$1" = "--" ] && shift
  d=gpurun_out/prof_$name
  mkdir -p $d
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- "$@" > $d.log 2>&1 || { echo "prof $name rc=$?"; tail -20 $d.log; exit 1; }
  grep -v '^[WE]2' $d.log | tail -8
  stats $d "$pat" ;;
pmc)
  name=$1; ctrs=$2; shift 2; [ "$1" = "--" ] && shift
  d=gpurun_out/pmc_$name
  mkdir -p $d
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $d -o run --output-format csv -- "$@" > $d.log 2>&1 || { echo "pmc $name rc=$?"; tail -5 $d.log; exit 1; }
  echo "pmc $name done" ;;
full)
  S=scripts/gpu_step.sh
  $S 700 pytest_gpu_$TAG python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
  $S 400 bench_$TAG python bench.py --steps 20 --warmup 5 || exit 1
  python - "$TAG" <<'PY'
import json, sys
tag = sys.argv[1]
line = [l for l in open(f"gpurun_out/bench_{tag}.log") if l.startswith("{")][-1]
print("JSON line bytes:", len(line))
print("extra keys:", list(json.loads(line).get("extra", {})))
PY
  echo ALLDONE ;;
profall)
  S=scripts/gpu_step.sh
  P=gpurun_out/prof_$TAG
  mkdir -p $P
  $S 300 bench_$TAG python bench.py --steps 20 --warmup 5 || exit 1
  $S 300 rocprof_stats rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline || exit 1
  $S 300 rocprof_fetch rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline || exit 1
  $S 300 rocprof_write rocprofv3 --pmc WRITE_SIZE -d $P/write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline || exit 1
  $S 300 rocprof_all rocprofv3 --kernel-trace --stats -d $P/all/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1
  $S 300 rocprof_all_fetch rocprofv3 --pmc FETCH_SIZE -d $P/all/fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit 1
  $S 300 rocprof_all_write rocprofv3 --pmc WRITE_SIZE -d $P/all/write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit 1
  echo ALLDONE ;;
*)
  echo "unknown mode $mode"; exit 2 ;;
esac
