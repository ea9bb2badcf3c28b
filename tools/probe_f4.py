#!/usr/bin/env python3
"""F4 timing alone: the bench's all-pairs case (100k x 12-nt UMIs, distance <= 1) plus larger L."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd._native import lib  # noqa: E402

dev = torch.device("cuda", 0)
if len(sys.argv) > 1 and sys.argv[1] == "quick":     # one case per method (rocprof kernel tables)
    # python tools/probe_f4.py quick [n L k]: pigeonhole and auto times on the last line (scripts/gpu.sh libab)
    n, L, k = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (100_000, 12, 1)
    res = []
    for m in ("tiles", "pigeonhole", "auto"):
        r = bench.bench_all_pairs(B, lib(), dev, n=n, L=L, k=k, method=m, reps=20)
        res.append(f"{m} {r['ms_per_step']:.4f} ms")
        print(res[-1], flush=True)
    print(" | ".join(res[1:]), flush=True)
    sys.exit(0)
for _ in range(2):
    print(bench.bench_all_pairs(B, lib(), dev), flush=True)
CASES = ((100_000, 12, 1), (200_000, 12, 1), (1_000_000, 12, 1), (100_000, 16, 2), (50_000, 32, 2),
         (200_000, 32, 3), (100_000, 8, 1), (20_000, 96, 4))
# multi-word reads (round 6: the pigeonhole form for L <= 128): python tools/probe_f4.py multiword
MULTI = ((100_000, 64, 2), (100_000, 96, 3), (100_000, 128, 4), (200_000, 100, 1), (1_000_000, 96, 2),
         (100_000, 40, 5))
for n, L, k in (MULTI if len(sys.argv) > 1 and sys.argv[1] == "multiword" else CASES):
    for m in (("tiles", "pigeonhole", "auto") if L <= 128 else ("tiles",)):
        if m == "tiles" and n > 200_000:
            continue
        r = bench.bench_all_pairs(B, lib(), dev, n=n, L=L, k=k, method=m, reps=5)
        print(n, L, k, m, f"{r['pairs_per_s'] / 1e12:.2f} T pairs/s", f"{r['ms_per_step']:.4f} ms",
              "hits", r["hits"], flush=True)
