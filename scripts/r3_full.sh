#!/usr/bin/env bash
# GPU call: the whole GPU suite on the current build, then the default bench (JSON line size checked)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
TAG=${1:-r3b}
$S 700 pytest_gpu_$TAG python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
$S 400 bench_$TAG python bench.py --steps 20 --warmup 5 || exit 1
python - "$TAG" <<'PY'
import json, sys
tag = sys.argv[1]
line = [l for l in open(f"gpurun_out/bench_{tag}.log") if l.startswith("{")][-1]
print("JSON line bytes:", len(line))
d = json.loads(line)
print("extra keys:", list(d.get("extra", {})))
PY
echo ALLDONE
