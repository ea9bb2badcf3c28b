#!/usr/bin/env python3
"""F1 one-pass index time alone, no parity check (for diagnostic library builds whose outputs are
deliberately incomplete): median of `reps` ss_fastq_index_onepass calls over the bench's 1.98-GB
synthetic FASTQ, events around each call.

    python tools/probe_f1_raw.py [reps]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
from shortseq_amd._native import check, lib  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    L, m, n_rec = 100, 1 << 16, 8 << 20
    rng = np.random.default_rng(1)
    parts = []
    for i in range(m):
        seq = rng.choice(np.frombuffer(b"ACGT", np.uint8), L).tobytes()
        parts.append(b"@SYN:%08d:" % i + b"x" * int(rng.integers(8, 28)) + b"\n" + seq + b"\n+\n" + b"I" * L + b"\n")
    buf = torch.from_numpy(np.frombuffer(b"".join(parts), np.uint8).copy()).to(dev).repeat(n_rec // m)
    nbytes, nrec = buf.numel(), n_rec
    lb = lib()
    s = torch.cuda.current_stream(dev).cuda_stream
    ws1_bytes = int(lb.ss_fastq_onepass_ws_bytes(nbytes, nrec + 2))
    ws1 = torch.empty((ws1_bytes + 7) // 8, dtype=torch.int64, device=dev)
    cnt = torch.empty(3, dtype=torch.int64, device=dev)
    offs = torch.empty(nrec + 2, dtype=torch.int64, device=dev)
    lens = torch.empty(nrec + 2, dtype=torch.int32, device=dev)
    aux = torch.empty(nrec + 2, dtype=torch.int64, device=dev)
    ts = []
    for r in range(reps + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        check(lb.ss_fastq_index_onepass(buf.data_ptr(), nbytes, 0, 1, ws1.data_ptr(), ws1_bytes, offs.data_ptr(),
                                        lens.data_ptr(), aux.data_ptr(), nrec + 2, cnt.data_ptr(), s), "index1")
        e1.record()
        torch.cuda.synchronize()
        if r >= 3:
            ts.append(e0.elapsed_time(e1))
    ts.sort()
    print(f"onepass median {ts[len(ts) // 2]:.4f} ms  min {ts[0]:.4f}", flush=True)


if __name__ == "__main__":
    main()
