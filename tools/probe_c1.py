#!/usr/bin/env python3
"""Phase timings of ShortSeqCounter(list) on the GPU path (C1 config: 1M x 32-nt reads), all-unique
and 2^14-pool lists, beside the reference's own ShortSeqCounter (oracle/_ref) when it is present."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402
import shortseq_amd as sq  # noqa: E402
from shortseq_amd import ingest, _shortseq as S  # noqa: E402

n, L = 1_000_000, 32
dev = torch.device("cuda", 0)
a = oracle.gen_reads(11, 0, n, L)
uniq = [a[i * L:(i + 1) * L].tobytes() for i in range(n)]
pa = oracle.gen_pool_reads(12, 13, 1 << 14, 0, n, L)
pool = [pa[i * L:(i + 1) * L].tobytes() for i in range(n)]
sq.ShortSeqCounter(uniq[:100_000])
torch.cuda.synchronize()
ref = None
if oracle.ref_available():
    sys.path.insert(0, oracle.REF_DIR)
    import shortseq.counter as ref  # noqa: E402
for name, reads in (("unique", uniq), ("pool16k", pool)):
    for rep in range(3):
        lens = np.full(n, L, dtype=np.int64)
        t0 = time.perf_counter()
        gc = ingest.count_list(reads, lens, dev)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        res = gc.finish_ordered()
        t2 = time.perf_counter()

        class G:
            def finish_ordered(self):
                return res
        c = sq.ShortSeqCounter()
        S._fill_groups(c, G())
        t3 = time.perf_counter()
        c = None
        t4 = time.perf_counter()
        full = sq.ShortSeqCounter(reads)
        t5 = time.perf_counter()
        full = None
        tr = float("nan")
        if ref is not None:
            t6 = time.perf_counter()
            x = ref.ShortSeqCounter(reads)
            tr = 1e3 * (time.perf_counter() - t6)
            x = None
        print(f"{name}: count_list {1e3 * (t1 - t0):.1f} ms, finish_ordered {1e3 * (t2 - t1):.1f} ms, "
              f"fill {1e3 * (t3 - t2):.1f} ms | full ShortSeqCounter {1e3 * (t5 - t4):.1f} ms | "
              f"reference {tr:.1f} ms", flush=True)
