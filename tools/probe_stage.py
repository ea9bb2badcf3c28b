#!/usr/bin/env python3
"""PCIe-inclusive encode/decode of host-resident batches (ss_encode_host / ss_decode_host):
pageable vs pinned buffers, chunk size, ring depth and staging threads."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shortseq_amd.batch as B  # noqa: E402

dev = torch.device("cuda", 0)
n, L = 32_000_000, 32
a_dev = B.synth_reads(n, L, seed=1, device=dev)
pageable = a_dev.cpu().numpy()
pinned_t = torch.empty(n * L, dtype=torch.uint8).pin_memory()
pinned_t.copy_(a_dev.reshape(-1).cpu())
pinned = pinned_t.numpy().reshape(n, L)
out_pin_t = torch.empty(n, dtype=torch.int64).pin_memory()
out_pin = out_pin_t.numpy().view(np.uint64).reshape(n, 1)
out_pg = np.empty((n, 1), np.uint64)
exp = B.encode(a_dev, L).cpu().numpy().view(np.uint64)
torch.cuda.synchronize()
print(f"host encode, {n} x {L} nt = {n * L / 1e9:.2f} GB in, {n * 8 / 1e9:.2f} GB out", flush=True)
for chunk in (16 << 20, 64 << 20, 256 << 20):
    for nslots in (2, 3, 4):
        for threads in (0, 4, 8, 16):
            if threads and chunk == (16 << 20) and nslots != 3:
                continue
            st = B.HostStager(dev, chunk_bytes=chunk, nslots=nslots, copy_threads=threads)
            for name, src, dst in (("pageable", pageable, out_pg), ("pinned", pinned, out_pin)):
                if name == "pinned" and threads not in (0,):
                    continue
                st.encode(src, out=dst)
                ts = []
                for _ in range(3):
                    t0 = time.perf_counter()
                    st.encode(src, out=dst)
                    ts.append(time.perf_counter() - t0)
                t = min(ts)
                assert np.array_equal(dst, exp)
                print(f"chunk {chunk >> 20:4d} MiB slots {nslots} threads {threads:2d} {name:8s}: "
                      f"{t * 1e3:7.1f} ms  {n * L / t / 1e9:6.1f} G nt/s  {n * (L + 8) / t / 1e9:5.1f} GB/s host<->dev",
                      flush=True)
            st.close()
st = B.HostStager(dev, chunk_bytes=64 << 20, nslots=3, copy_threads=8)
back = np.empty((n, L), np.uint8)
for name, w in (("pageable", out_pg),):
    st.decode(w, L, out=back)
    t0 = time.perf_counter()
    st.decode(w, L, out=back)
    t = time.perf_counter() - t0
    assert np.array_equal(back, pageable)
    print(f"host decode {name}: {t * 1e3:.1f} ms {n * L / t / 1e9:.1f} G nt/s", flush=True)
# H2D-only ceiling for reference
t0 = time.perf_counter()
for _ in range(3):
    a_dev.reshape(-1).copy_(pinned_t, non_blocking=True)
torch.cuda.synchronize()
t = (time.perf_counter() - t0) / 3
print(f"pinned H2D copy ceiling: {n * L / t / 1e9:.1f} GB/s", flush=True)
