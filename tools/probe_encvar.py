#!/usr/bin/env python3
"""ss_encode_var on the bench's F2 batch (50M ragged reads of 50-150 nt, wpr 5): median kernel time
over reps (events around each call) and a checksum of the words, on the last line (for
scripts/r3_libab.sh A/B runs of two library builds).

    python tools/probe_encvar.py [reps]
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd._native import check, lib  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    n = 50_000_000
    blob, offs, lens = B.synth_ragged_pool_reads(n, 41, 42, 1 << 20, 50, 150, device=dev)
    words = torch.empty((n, 5), dtype=torch.int64, device=dev)
    fb = B.first_bad_buffer(dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    L = lib()
    ts = []
    for r in range(reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        check(L.ss_encode_var(blob.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, words.data_ptr(), 5,
                              fb.data_ptr(), s), "encode_var")
        e1.record()
        torch.cuda.synchronize()
        if r >= 2:
            ts.append(e0.elapsed_time(e1))
    ts.sort()
    csum = int(words.view(-1)[::7].sum().item()) & 0xFFFFFFFFFFFF
    print(f"encode_var median {ts[len(ts) // 2]:.4f} ms  min {ts[0]:.4f}  bad {int(fb.item())}  csum {csum:x}",
          flush=True)


if __name__ == "__main__":
    main()
