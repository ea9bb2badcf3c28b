#!/usr/bin/env python3
"""Why does C5 run ~10 % faster inside bench.py than alone (same box, same build: round 6,
2.28 vs 2.52 ms, the coarse pass 0.99 vs 1.19 ms)?  One process, the same counter step
(bench.bench_counter: 125M x 32-nt reads, pool 2^24) measured
  fresh        right after start-up (as tools/c5_only.py)
  again        a second time in the same process (new table, new workspace)
  after_heat   after ~2 s of back-to-back C2 encodes (clocks / power state after sustained load)
  after_churn  after allocating and freeing 40 GB through torch's caching allocator (address layout)
  bench_order  after the C2 / C3 / C4 steps of bench.py (its actual order)

    python tools/probe_c5_env.py [steps=10]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd._native import lib  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)


def c5(tag):
    el, d, u, _chk, passes, _x = bench.bench_counter(B, lib(), dev, 0, 1, 125_000_000, 32, 1 << 24, steps, 3)
    pp = " ".join(f"{k} {v:.3f}" for k, v in passes.items())
    print(f"{tag:12s} C5 {el / steps * 1e3:.3f} ms/step, device {d:.3f} ms [{pp}]", flush=True)


c5("fresh")
c5("again")
a = B.synth_reads(100_000_000, 32, seed=1, device=dev)
w = torch.empty((100_000_000, 1), dtype=torch.int64, device=dev)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 2.0:
    for _ in range(50):
        B.encode(a, 32, out=w, check_errors=False)
    torch.cuda.synchronize()
del a, w
c5("after_heat")
blocks = [torch.empty(4 << 30, dtype=torch.uint8, device=dev) for _ in range(10)]
del blocks
c5("after_churn")
torch.cuda.empty_cache()
L, n = 32, 100_000_000
bench.bench_encode(B, lib(), dev, 0, 1, n, L, 20, 5)
bench.bench_encode_hamming(B, lib(), dev, 0, 1, n, 96, 20, 5)
bench.bench_roundtrip(B, lib(), dev, 0, 1, n // 2, 512, 10, 5)
c5("bench_order")
