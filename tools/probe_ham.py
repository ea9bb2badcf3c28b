#!/usr/bin/env python3
"""Time ss_hamming_ref (dense packed rows) for the SURVEY §8(d) C3' configs: HIP events over 20
launches after a 100-ms settle."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd._native import lib  # noqa: E402

dev = torch.device("cuda", 0)
L_ = lib()
s = torch.cuda.current_stream(dev).cuda_stream
for L, n in ((32, 100_000_000), (96, 100_000_000), (512, 50_000_000)):
    words = B.encode(B.synth_reads(n, L, seed=6, device=dev), L)
    ref = words[0].clone()
    out = torch.empty(n, dtype=torch.int32, device=dev)
    wpr = words.shape[1]
    f = lambda: L_.ss_hamming_ref(words.data_ptr(), n, L, wpr, ref.data_ptr(), out.data_ptr(), s)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.1:
        f()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    gbs = n * (8 * wpr + 4) / (ms * 1e-3) / 1e9
    print(f"L={L}: {ms:.4f} ms {gbs:.0f} GB/s frac {gbs / 8000:.3f}", flush=True)
    del words, out
