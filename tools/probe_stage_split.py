#!/usr/bin/env python3
"""C2 host-staged (32M x 32-nt pageable reads through ss_encode_host) by copy-thread count and
placement, with the stage split of each setting: every stager is created in the
same process, so the box, the input and the output are the same for all of them.

    python tools/probe_stage_split.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shortseq_amd.batch as B  # noqa: E402

dev = torch.device("cuda", 0)
n, L = 32_000_000, 32
host = B.synth_reads(n, L, seed=1, device=dev).cpu().numpy()
out = np.empty((n, 1), np.uint64)
for threads, pin in ((8, "1"), (8, "0"), (16, "1"), (16, "0"), (4, "1"), (12, "1")):
    os.environ["SHORTSEQ_STAGE_PIN"] = pin
    st = B.HostStager(dev, copy_threads=threads)
    st.encode(host, out=out)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        st.encode(host, out=out)
        ts.append(time.perf_counter() - t0)
    st.set_timing(True)
    st.stats()
    for _ in range(2):
        st.encode(host, out=out)
    sp = st.stats()
    st.close()
    stages = " ".join(f"{k} {v:.2f}" for k, v in sp.items() if isinstance(v, float))
    print(f"threads {threads:2d} pin {pin}: {np.median(ts) * 1e3:.2f} ms (min {min(ts) * 1e3:.2f})  [{stages}]  "
          f"affinity {sp['affinity_cpus']} numa {sp['gpu_numa_node']} pinned {sp['pinned_cpus']}", flush=True)
