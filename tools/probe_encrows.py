#!/usr/bin/env python3
"""k_encode_rows alone on the f2 batch (50M reads of 50-150 nt, S = 6): the library's internal
ss_encode_rows_impl called through ctypes, mean of `reps` launches timed with torch events (the
engine's other passes left out, so diagnostic builds that skip its fingerprint work still run).

    python3 tools/probe_encrows.py [reps=10]
"""
import ctypes as C
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd._native import lib  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    n, S = 50_000_000, 6
    blob, offs, lens = B.synth_ragged_pool_reads(n, 41, 42, 1 << 20, 50, 150, device=dev)
    out = torch.empty(n * S, dtype=torch.int64, device=dev)
    fps = torch.empty(n, dtype=torch.int64, device=dev)
    hll = torch.zeros(33 << 11, dtype=torch.int32, device=dev)
    fb = torch.full((1,), -1, dtype=torch.int64, device=dev)
    f = lib().ss_encode_rows_impl
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                  C.c_void_p, C.c_void_p]
    s = torch.cuda.current_stream(dev).cuda_stream
    args = (blob.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, S, out.data_ptr(), fps.data_ptr(), hll.data_ptr(),
            fb.data_ptr(), s)
    for _ in range(2):
        assert f(*args) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f(*args)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    moved = int(lens.sum().item()) + n * 12 + n * S * 8 + n * 8
    print(f"k_encode_rows: {ms:.3f} ms per launch, {moved / ms / 1e6:.0f} GB/s of algorithmic bytes", flush=True)


if __name__ == "__main__":
    main()
