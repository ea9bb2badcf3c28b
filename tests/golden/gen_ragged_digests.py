#!/usr/bin/env python3
"""Generator-derived digests of the f2 ragged workload (mixed 50-150-nt reads counted
by the drop-in engine, one table per length).

No reference code is involved: the counter rows of ragged pool-drawn reads follow from the generator
alone (oracle.ragged_pool_rows: the drawn items in first-occurrence order with their lengths, draw
counts and words).  That construction is pinned to oracle.count (itself pinned to the reference's
counter) on small prefixes by tests/test_oracle_golden.py::test_ragged_pool_rows_match_oracle_count.

    python3 tests/golden/gen_ragged_digests.py        # writes tests/golden/ragged_digests.json
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402

# bench.py F2 lines / tests/test_ragged.py (U24: the high-diversity line, ~16M distinct keys)
CASES = {"ragged_50M_L50-150_U20": dict(seed=41, pool_seed=42, U=1 << 20, n=50_000_000, Lmin=50, Lmax=150),
         "ragged_1M_L1-300_U16": dict(seed=43, pool_seed=44, U=1 << 16, n=1_000_000, Lmin=1, Lmax=300),
         "ragged_50M_L50-150_U24": dict(seed=41, pool_seed=42, U=1 << 24, n=50_000_000, Lmin=50, Lmax=150)}


def main():
    """python3 gen_ragged_digests.py [names...]: (re)computes the named cases (default: all) and keeps
    the others already in ragged_digests.json."""
    path = os.path.join(HERE, "ragged_digests.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    only = set(sys.argv[1:]) or set(CASES)
    for name, c in CASES.items():
        if name not in only:
            continue
        t = time.time()
        lens, counts, words = oracle.ragged_pool_rows(c["seed"], c["pool_seed"], c["U"], c["n"], c["Lmin"], c["Lmax"])
        out[name] = dict(c, unique=int(len(lens)), nt=int((lens.astype("u8") * counts).sum()),
                         digest=oracle.rows_digest(lens, counts, words))
        print(name, out[name], f"{time.time() - t:.1f}s", flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
