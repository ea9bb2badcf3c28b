#!/usr/bin/env python3
"""Run only the C5 counter step (bench.py's bench_counter) for profiling."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd._native import lib  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
el, d, u = bench.bench_counter(B, lib(), dev, 0, 1, 125_000_000, 32, 1 << 24, 10, 3)
print(f"C5: {el / 10 * 1e3:.3f} ms/step wall, {d:.3f} ms device, unique {u}")

# A/B in the same process: lazy reset (fresh aggregate) vs an eager reset (memset + slice read)
from shortseq_amd.dist import ShardedCounter  # noqa: E402
ascii = B.synth_pool_reads(125_000_000, 32, 5, 77, 1 << 24, device=dev)
sc = ShardedCounter(1 << 25, device=dev)
t = sc.local
for name in ("lazy", "eager", "lazy", "eager"):
    def step():
        t.reset()
        if name == "eager":
            t.size()                 # flushes the pending reset: memset, then a non-fresh insert
        t.insert(ascii, 32, base_index=0, check_errors=False)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        step()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / 10:.3f} ms/step (device)", flush=True)
