#!/usr/bin/env bash
# kernel trace of the C5 counter step only
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/prof_${1:-c5}
mkdir -p $P
scripts/gpu_step.sh 400 prof_c5 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 tools/c5_only.py || exit 1
python3 tools/prof_summary.py $P | head -20
