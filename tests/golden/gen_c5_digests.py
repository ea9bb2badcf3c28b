#!/usr/bin/env python3
"""Generator-derived digests of the C5 counter workload at full shard size.

No reference code is involved: the counter result of pool-drawn reads follows from the generator
alone (oracle.pool_counter_table: keys = generator word of each drawn pool item, counts = bincount
of the draw indices, first = index of the first draw).  The same construction is pinned against
oracle.count (itself pinned to the reference's counter digest, tests/golden/golden_digests.json)
on small prefixes by tests/test_oracle_golden.py::test_pool_counter_table_matches_oracle_count.

    python3 tests/golden/gen_c5_digests.py            # writes tests/golden/c5_digests.json (~10 min)
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, REPO)
import oracle  # noqa: E402

SEED, POOL_SEED, L = 5, 77, 32          # bench.py bench_counter / tests/test_c5_full.py
N = 125_000_000                          # one GPU's shard of the 1B-read C5 job


def zipf_cdf(U, s):
    # the same table as shortseq_amd.batch.zipf_cdf (restated here so the generator script does not
    # import the product)
    w = np.arange(1, U + 1, dtype=np.float64) ** (-float(s))
    c = np.cumsum(w)
    c /= c[-1]
    cdf = np.floor(c * 2.0 ** 63).astype(np.uint64)
    cdf[-1] = np.uint64(1 << 63)
    return cdf


CASES = [
    # name, U, zipf s (None = uniform), i0, n
    ("uniform_U24_shard0", 1 << 24, None, 0, N),
    ("uniform_U24_shard7", 1 << 24, None, 7 * N, N),
    ("uniform_U20_shard0", 1 << 20, None, 0, N),
    ("zipf1.1_U24_shard0", 1 << 24, 1.1, 0, N),
    ("zipf1.1_U20_shard0", 1 << 20, 1.1, 0, N),
]


def main():
    out = {"_meta": {"seed": SEED, "pool_seed": POOL_SEED, "L": L,
                     "script": "tests/golden/gen_c5_digests.py",
                     "rows": "(key, count, first) uint64 rows sorted by key, SHA-256 (oracle.table_digest)"}}
    path = os.path.join(HERE, "c5_digests.json")
    if os.path.exists(path):
        out.update(json.load(open(path)))
    only = set(sys.argv[1:])
    for name, U, s, i0, n in CASES:
        if only and name not in only:
            continue
        t = time.time()
        cdf = zipf_cdf(U, s) if s else None
        k, c, f = oracle.pool_counter_table(SEED, POOL_SEED, U, n, L, i0=i0, cdf=cdf)
        out[name] = {"U": U, "zipf_s": s, "i0": i0, "n": n, "unique": int(len(k)),
                     "max_count": int(c.max()), "digest": oracle.table_digest(k, c, f)}
        print(name, out[name], f"{time.time() - t:.0f} s", flush=True)
        json.dump(out, open(path, "w"), indent=1)
    # whole jobs over W shards of N reads (the multi-GPU C5: rank r counts reads [r N, (r + 1) N)):
    # the union of the shard tables, for the 8-rank rehearsal test and bench.py's world > 1 check
    for W in (2, 4, 8):
        name = f"uniform_U24_job{W}"
        if only and name not in only:
            continue
        t = time.time()
        U = 1 << 24
        counts = np.zeros(U, dtype=np.uint64)
        first = np.full(U, np.iinfo(np.uint64).max, dtype=np.uint64)
        for r in range(W):
            for s0 in range(0, N, 1 << 23):
                m = min(1 << 23, N - s0)
                ids = oracle.pool_ids(POOL_SEED, r * N + s0, m, U)
                counts += np.bincount(ids.astype(np.int64), minlength=U).astype(np.uint64)
                u, pos = np.unique(ids, return_index=True)
                new = first[u] == np.iinfo(np.uint64).max
                first[u[new]] = np.uint64(r * N + s0) + pos[new].astype(np.uint64)
        used = np.nonzero(counts)[0]
        keys = oracle.splitmix64_np(np.uint64(SEED) + used.astype(np.uint64))
        out[name] = {"U": U, "zipf_s": None, "i0": 0, "n": W * N, "shards": W,
                     "unique": int(len(used)), "max_count": int(counts.max()),
                     "digest": oracle.table_digest(keys, counts[used], first[used])}
        print(name, out[name], f"{time.time() - t:.0f} s", flush=True)
        json.dump(out, open(path, "w"), indent=1)

if __name__ == "__main__":
    main()
