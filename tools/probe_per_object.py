#!/usr/bin/env python3
"""Per-object drop-in API (pack from bytes / str, str(), ^, hash, ==) against the reference's own
objects (oracle/_ref) at 20-1000 nt, ns per call (best of 3 passes over 200k / 50k reads)."""
import sys, time
import os
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle
sys.path.insert(0, oracle.REF_DIR)
import shortseq.short_seq as R
import shortseq_amd as S
import numpy as np
def bench(f, xs, reps=3):
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter(); f(xs); best = min(best, time.perf_counter() - t0)
    return best / len(xs) * 1e9
for L in (20, 32, 75, 200, 1000):
    n = 200_000 if L < 500 else 50_000
    a = oracle.gen_reads(3, 0, n, L)
    reads = [a[i * L:(i + 1) * L].tobytes() for i in range(n)]
    sreads = [r.decode() for r in reads]
    for name, M in (("ref", R), ("ours", S)):
        objs = [M.pack(r) for r in reads]
        o2 = objs[1:] + objs[:1]
        t_pack = bench(lambda xs: [M.pack(r) for r in xs], reads)
        t_packs = bench(lambda xs: [M.pack(r) for r in xs], sreads)
        t_str = bench(lambda xs: [str(o) for o in xs], objs)
        t_xor = bench(lambda xs: [x ^ y for x, y in zip(xs, o2)], objs)
        t_hash = bench(lambda xs: [hash(o) for o in xs], objs)
        t_eq = bench(lambda xs: [x == y for x, y in zip(xs, objs)], o2)
        print(f"L={L:4d} {name:4s} pack(bytes) {t_pack:6.1f} pack(str) {t_packs:6.1f} str {t_str:6.1f} xor {t_xor:6.1f} hash {t_hash:6.1f} eq {t_eq:6.1f} ns")
