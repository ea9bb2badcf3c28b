#!/usr/bin/env python3
"""Run only the C5 counter step (bench.py's bench_counter) for profiling.

    python3 tools/c5_only.py [U_log2=24] [zipf_s=0 (uniform)] [steps=10]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd._native import lib  # noqa: E402

ulog = int(sys.argv[1]) if len(sys.argv) > 1 else 24
zs = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
el, d, u, _chk, passes, _x = bench.bench_counter(B, lib(), dev, 0, 1, 125_000_000, 32, 1 << ulog, steps, 3, zipf=zs or None)
pp = " ".join(f"{k} {v:.3f}" for k, v in passes.items())
print(f"C5 U=2^{ulog} zipf={zs}: {el / steps * 1e3:.3f} ms/step wall, {d:.3f} ms device, unique {u} [{pp}]", flush=True)
