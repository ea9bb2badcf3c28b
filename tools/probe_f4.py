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
for _ in range(2):
    print(bench.bench_all_pairs(B, lib(), dev), flush=True)
for n, L, k in ((200_000, 12, 1), (50_000, 32, 2), (20_000, 96, 4)):
    r = bench.bench_all_pairs(B, lib(), dev, n=n, L=L, k=k)
    print(n, L, k, f"{r['pairs_per_s'] / 1e12:.2f} T pairs/s", r["ms_per_step"], flush=True)
