#!/usr/bin/env bash
# One GPU call: tests, tuning sweep, bench, rocprofv3 kernel-trace + PMC traffic passes.
# Each step has its own time limit; a fatal step (fault/abort/timeout) ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r1}
S=scripts/gpu_step.sh
$S 600 pytest_gpu python -m pytest tests -m gpu -q || exit 1
if [ -x tools/tune_kernels ] && [ "${TUNE:-0}" = 1 ]; then $S 400 tune_kernels tools/tune_kernels 20 || exit 1; fi
$S 400 bench python bench.py --steps 20 --warmup 5 || exit 1
P=gpurun_out/prof_$TAG
mkdir -p $P
# C2-only runs: the rocprof summary's k_encode_g16 average is the bench's roofline kernel
$S 400 rocprof_stats rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline || exit 1
$S 400 rocprof_fetch rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline || exit 1
$S 400 rocprof_write rocprofv3 --pmc WRITE_SIZE -d $P/write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline || exit 1
# all configs (C3/C4/C5 kernels)
$S 400 rocprof_all rocprofv3 --kernel-trace --stats -d $P/all/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1
$S 400 rocprof_all_fetch rocprofv3 --pmc FETCH_SIZE -d $P/all/fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit 1
$S 400 rocprof_all_write rocprofv3 --pmc WRITE_SIZE -d $P/all/write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit 1
echo ALLDONE
