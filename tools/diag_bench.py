#!/usr/bin/env python3
"""Diagnose bench-vs-C++ timing gaps for the 32-nt encode: torch caching-allocator buffers vs raw
hipMalloc buffers, loop length, and launching on torch's current stream vs a fresh HIP stream."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd._native import lib  # noqa: E402

L, n = 32, 100_000_000
hip = C.CDLL("libamdhip64.so")
dev = torch.device("cuda", 0)
lb = lib()


def region(ap, wp, fp, stream, steps):
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        lb.ss_encode_fixed(ap, n, L, L, wp, 1, fp, stream)
    torch.cuda.synchronize()
    s0.record()
    for _ in range(steps):
        lb.ss_encode_fixed(ap, n, L, L, wp, 1, fp, stream)
    s1.record()
    torch.cuda.synchronize()
    return s0.elapsed_time(s1) / steps


ascii = B.synth_reads(n, L, seed=1, device=dev)
words = torch.empty((n, 1), dtype=torch.int64, device=dev)
fb = B.first_bad_buffer(dev)
st = torch.cuda.current_stream(dev).cuda_stream
for steps in (20, 100):
    ms = region(ascii.data_ptr(), words.data_ptr(), fb.data_ptr(), st, steps)
    print(f"torch buffers, torch stream, {steps} steps: {ms:.4f} ms  {4e9 / ms / 1e6:.1f} GB/s", flush=True)
# raw hipMalloc buffers
pa, pw = C.c_void_p(), C.c_void_p()
assert hip.hipMalloc(C.byref(pa), C.c_size_t(n * L)) == 0
assert hip.hipMalloc(C.byref(pw), C.c_size_t(n * 8)) == 0
assert hip.hipMemcpy(pa, C.c_void_p(ascii.data_ptr()), C.c_size_t(n * L), 3) == 0
for steps in (20, 100):
    ms = region(pa.value, pw.value, fb.data_ptr(), st, steps)
    print(f"hipMalloc buffers, torch stream, {steps} steps: {ms:.4f} ms  {4e9 / ms / 1e6:.1f} GB/s", flush=True)
s2 = torch.cuda.Stream(dev)
with torch.cuda.stream(s2):
    ms = region(ascii.data_ptr(), words.data_ptr(), fb.data_ptr(), s2.cuda_stream, 100)
    print(f"torch buffers, side stream, 100 steps: {ms:.4f} ms  {4e9 / ms / 1e6:.1f} GB/s", flush=True)
ms = region(ascii.data_ptr(), words.data_ptr(), fb.data_ptr(), st, 100)
print(f"torch buffers, torch stream, 100 steps (again): {ms:.4f} ms  {4e9 / ms / 1e6:.1f} GB/s", flush=True)
