#!/usr/bin/env python3
"""C5 pass times without the parity check (for diagnostic library builds whose tables are wrong on
purpose, e.g. the coarse pass with its record stores or its loads cut out): the bench's counter step
(125M x 32-nt reads, pool 2^24 uniform), per-pass device ms from ss_counter_set_timing.

    python tools/probe_c5_diag.py [steps=10]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd.dist import ShardedCounter  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
n, L, U = 125_000_000, 32, 1 << 24
ascii = B.synth_pool_reads(n, L, 5, 77, U, device=dev)
sc = ShardedCounter(1 << 25, device=dev)


def step(_t):
    sc.count(ascii, L, base_index=0, check_errors=False)


el, tr = bench.timed_loop(step, steps, 3, 1)
sc.local.set_timing(True)
bench.timed_loop(step, max(2, steps // 2), 1, 1, on_timed_start=lambda: sc.local.pass_times())
p = sc.local.pass_times()
print(f"C5 {tr.region_ms / steps:.3f} ms/step  " + " ".join(f"{k} {v:.3f}" for k, v in p.items()), flush=True)
