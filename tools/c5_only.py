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
