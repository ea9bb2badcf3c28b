#!/usr/bin/env python3
"""Time ss_hamming_ref (dense packed rows) for the SURVEY §8(d) C3' configs: HIP events over 20
launches after a 100-ms settle."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shortseq_amd._native as N  # noqa: E402
if os.environ.get("SS_PROBE_LIB"):   # A/B: a library variant built with other -D knobs
    N.LIB = os.environ["SS_PROBE_LIB"]
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
    print(f"{os.path.basename(N.LIB)} L={L}: {ms:.4f} ms {gbs:.0f} GB/s frac {gbs / 8000:.3f}", flush=True)
    del words, out

# C3: fused encode + hamming vs one read, 100M x 96 nt (ss_encode_hamming_ref)
L, n = 96, 100_000_000
ascii = B.synth_reads(n, L, seed=2, device=dev)
words = torch.empty((n, 3), dtype=torch.int64, device=dev)
ref = torch.zeros(3, dtype=torch.int64, device=dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
fb = B.first_bad_buffer(dev)
f = lambda: L_.ss_encode_hamming_ref(ascii.data_ptr(), n, L, L, words.data_ptr(), 3, ref.data_ptr(), out.data_ptr(),
                                     fb.data_ptr(), s)
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
gbs = n * 124 / (ms * 1e-3) / 1e9
print(f"{os.path.basename(N.LIB)} C3 fused L=96: {ms:.4f} ms {gbs:.0f} GB/s frac {gbs / 8000:.3f}", flush=True)
