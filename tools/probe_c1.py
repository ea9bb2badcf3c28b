#!/usr/bin/env python3
"""Phase timings of ShortSeqCounter(list) on the GPU path (C1 config: 1M x 32-nt reads)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle  # noqa: E402
import shortseq_amd as sq  # noqa: E402
from shortseq_amd import ingest  # noqa: E402

n, L = 1_000_000, 32
a = oracle.gen_reads(11, 0, n, L)
reads = [a[i * L:(i + 1) * L].tobytes() for i in range(n)]
dev = torch.device("cuda", 0)
sq.ShortSeqCounter(reads[:100_000])
torch.cuda.synchronize()
for rep in range(2):
    t0 = time.perf_counter()
    lens = np.full(n, L, dtype=np.int64)
    gc = ingest.count_list(reads, lens, dev)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    groups, e = gc.finish()
    t2 = time.perf_counter()
    c = sq.ShortSeqCounter()
    t3 = time.perf_counter()
    full = sq.ShortSeqCounter(reads)
    t4 = time.perf_counter()
    print(f"count_list {1e3 * (t1 - t0):.1f} ms, finish (extract + D2H) {1e3 * (t2 - t1):.1f} ms, "
          f"full ShortSeqCounter {1e3 * (t4 - t3):.1f} ms", flush=True)
t0 = time.perf_counter()
d = {}
for r in reads:
    k = sq.pack(r)
    d[k] = d.get(k, 0) + 1
print(f"python dict of packs {1e3 * (time.perf_counter() - t0):.1f} ms")
