#!/usr/bin/env python3
"""Cost of the C5 exchange-side kernels on one GPU: extract(n_parts=8) of a 125M-read table (pool
2^24) and the owner-side merge of as many (key, count, first) entries as one of 8 owners receives
(~ the table's unique keys: every rank holds most of the pool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shortseq_amd.batch as B  # noqa: E402


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


dev = torch.device("cuda", 0)
n, L, U = 125_000_000, 32, 1 << 24
ascii = B.synth_pool_reads(n, L, 5, 77, U, device=dev)
local = B.GpuCounter(1 << 25, device=dev)
local.insert(ascii, L)
del ascii
keys, lens, counts, first, parts = local.extract(n_parts=8)
m = int(parts.sum().item())
print("unique", m, "parts", parts.tolist(), flush=True)
print(f"extract(8): {t(lambda: local.extract(n_parts=8)):.3f} ms", flush=True)
owner = B.GpuCounter(1 << 25, device=dev)
k, c, f = keys[:m].contiguous(), counts[:m].contiguous(), first[:m].contiguous()


def merge():
    owner.reset()
    owner.merge(k, c, f, L)


print(f"merge {m} entries: {t(merge):.3f} ms (incl. 1-GB table reset)", flush=True)
print(f"reset only: {t(owner.reset):.3f} ms", flush=True)

# region-range protocol: extract_ranges(8) + owner 0 folding 7 runs of ~2.1M entries
keys, lens, counts, first, parts = local.extract_ranges(8)
torch.cuda.synchronize()
print(f"extract_ranges(8): {t(lambda: local.extract_ranges(8)):.3f} ms", flush=True)
p0 = int(parts[0].item())
k7 = keys[:p0].repeat(7)
c7 = counts[:p0].repeat(7)
f7 = first[:p0].repeat(7)
runs = [(i * p0, (i + 1) * p0) for i in range(7)]
dst = B.GpuCounter(1 << 25, device=dev)


def merge_runs():
    dst.reset()
    dst.merge_runs(k7, c7, f7, runs, 0, 8, L)


print(f"merge_runs 7 x {p0} entries into owner 0: {t(merge_runs):.3f} ms (incl. table reset)", flush=True)
dst.merge_runs(k7, c7, f7, runs, 0, 8, L)
assert not dst.overflowed()

# packed protocol: pack_ranges(8, skip=0) right after the insert (aggregate occupancy, one pass),
# then owner 0 folding 7 packed runs
local.reset()
ascii = B.synth_pool_reads(n, L, 5, 77, U, device=dev)
local.insert(ascii, L)
del ascii


def pack():
    return local.pack_ranges(8, skip=0, first_base=0)


torch.cuda.synchronize()
rec, pparts = pack()
torch.cuda.synchronize()
print(f"pack_ranges(8, skip 0) after the insert: {t(pack, reps=1):.3f} ms (occupancy from the aggregate)",
      flush=True)
print(f"pack_ranges(8, skip 0) again: {t(pack):.3f} ms", flush=True)
local._drop_reservation()
local.merge(k[:1], c[:1], f[:1], L)   # any other mutation: occupancy stale -> counting pass
print(f"pack_ranges(8, skip 0) with a counting pass: {t(pack):.3f} ms", flush=True)
q = int(pparts[1].item())
rec7 = rec[:q].repeat(7, 1)
pruns = [(i * q, (i + 1) * q, 0) for i in range(7)]


def merge_packed():
    dst.reset()
    dst.merge_packed(rec7, pruns, 1, 8, L)


print(f"merge_packed 7 x {q} records into owner 1: {t(merge_packed):.3f} ms (incl. table reset)", flush=True)
assert not dst.overflowed()
