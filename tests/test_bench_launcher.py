"""bench.py's launcher contract on CPU: `--gpus N` with no WORLD_SIZE starts N
ranks itself (torch.distributed.run child, 127.0.0.1) and hands on rank 0's one JSON line with
n_gpus N; a WORLD_SIZE that disagrees with --gpus exits non-zero.  --dry-run does no GPU work (the
plumbing only); the same path with real GPU work runs on the box (tests/test_dist_gpu.py)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], env=env, cwd=REPO,
                          capture_output=True, text=True, timeout=240)


def test_bench_starts_ranks_without_launcher():
    p = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-run", "--reads-per-gpu", "1000"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["config"]["parallelism"] == "dp2"
    assert rec["value"] is None and "dry run" in rec["data"]


def test_bench_refuses_mismatched_world():
    p = _run(["--gpus", "4", "--steps", "1", "--warmup", "0", "--dry-run"],
             {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]
