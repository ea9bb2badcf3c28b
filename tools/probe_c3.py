#!/usr/bin/env python3
"""C3 (100M x 96-nt fused encode + hamming vs read 0) timing forms: one event pair around N
back-to-back fused calls vs a pair around each call (bench.py's kernel_ms_events)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd._native import lib  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
n, L = 100_000_000, 96
ascii = B.synth_reads(n, L, seed=2, i0=0, device=dev)
wpr = B.wpr_for(L)
words = torch.empty((n, wpr), dtype=torch.int64, device=dev)
dist_out = torch.empty(n, dtype=torch.int32, device=dev)
ref = torch.empty((1, wpr), dtype=torch.int64, device=dev)
fb = B.first_bad_buffer(dev)
s = torch.cuda.current_stream(dev).cuda_stream
Lb = lib()
assert Lb.ss_encode_fixed(ascii.data_ptr(), 1, L, L, ref.data_ptr(), wpr, fb.data_ptr(), s) == 0


def call():
    assert Lb.ss_encode_hamming_ref(ascii.data_ptr(), n, L, L, words.data_ptr(), wpr, ref.data_ptr(),
                                    dist_out.data_ptr(), fb.data_ptr(), s) == 0


for _ in range(5):
    call()
torch.cuda.synchronize()
for r in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        call()
    e1.record()
    torch.cuda.synchronize()
    batch_ms = e0.elapsed_time(e1) / 20
    pairs = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        call()
        b.record()
        pairs.append((a, b))
    torch.cuda.synchronize()
    each = sum(a.elapsed_time(b) for a, b in pairs) / 20
    print(f"C3 fused: {batch_ms:.4f} ms per call (20 back to back), {each:.4f} ms per call (a pair each)",
          flush=True)
