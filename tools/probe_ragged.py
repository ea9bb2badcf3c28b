#!/usr/bin/env python3
"""f2 probe: ss_encode_var and the device-fed drop-in engine on the bench's ragged workload (50M reads
of 50-150 nt over a 2^20-item pool), timed like bench.py's F2 line, with the digest check.

    python tools/probe_ragged.py [reps]
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import bench  # noqa: E402
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd._native import lib  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    t0 = time.time()
    r = bench.bench_ragged(B, lib(), dev, reps=reps)
    print(bench.json.dumps(bench.compact(r)), f"({time.time() - t0:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
