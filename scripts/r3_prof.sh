#!/usr/bin/env bash
# One GPU call: the rocprofv3 kernel-trace summaries and PMC traffic passes of gpu_round.sh, without
# its test / bench steps (run those with r3_full.sh); output under gpurun_out/prof_<tag>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r3}
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
echo ALLDONE
