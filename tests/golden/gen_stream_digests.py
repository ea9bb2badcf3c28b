#!/usr/bin/env python3
"""Generator-derived digests of the streaming workloads at BASELINE size.

No reference code is involved.  The device generator writes read i as the ASCII of the words
splitmix64(seed + i*W + w) (oracle/ss_oracle.c:ora_gen_word), so a correct encode returns exactly
those words, and the hamming distance of read i to read 0 follows from them by the reference's
XOR-collapse-popcount (short_seq_64.pyx:82-84; oracle.hamming_ref_batch restates it and is pinned
to the reference's golden vectors).  tests/test_oracle_golden.py checks this numpy construction
against oracle.gen_reads + oracle.encode_batch + oracle.hamming_ref_batch on a prefix.

    python3 tests/golden/gen_stream_digests.py      # writes tests/golden/stream_digests.json (~2 min)
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# name, reads, L, seed (tests/test_gpu_parity.py::test_full_size_digests uses these)
CASES = [
    ("C2_100000000x32", 100_000_000, 32, 1),
    ("C3_100000000x96", 100_000_000, 96, 1),
    ("C4_50000000x512", 50_000_000, 512, 1),
]
CHUNK = 1 << 22   # reads per numpy step


def splitmix64(x):
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def gen_words(seed, i0, n, L):
    """Packed words of generator reads i0 .. i0+n-1, L % 32 == 0 (no masked tail word)."""
    assert L % 32 == 0
    W = L // 32
    with np.errstate(over="ignore"):
        base = np.uint64(seed) + np.arange(i0, i0 + n, dtype=np.uint64) * np.uint64(W)
        x = base[:, None] + np.arange(W, dtype=np.uint64)[None, :]
    return splitmix64(x)


def hamming_ref(words, ref):
    """short_seq_64.pyx:82-84 per word: xor, collapse each 2-bit code onto its low bit, popcount."""
    x = words ^ ref[None, :]
    y = (x | (x >> np.uint64(1))) & np.uint64(0x5555555555555555)
    return np.bitwise_count(y).sum(axis=1, dtype=np.uint32)


def digests(n, L, seed, chunk=CHUNK):
    hw, hd = hashlib.sha256(), hashlib.sha256()
    ref = gen_words(seed, 0, 1, L)[0]
    for i0 in range(0, n, chunk):
        m = min(chunk, n - i0)
        w = gen_words(seed, i0, m, L)
        hw.update(w.tobytes())
        hd.update(hamming_ref(w, ref).tobytes())
    return hw.hexdigest(), hd.hexdigest()


def main():
    out = {"_meta": {"script": "tests/golden/gen_stream_digests.py",
                     "words": "SHA-256 of the packed u64 words, read-major",
                     "hamming_vs_read0": "SHA-256 of the u32 distances of every read to read 0"}}
    for name, n, L, seed in CASES:
        ws, ds = digests(n, L, seed)
        out[name] = {"n": n, "L": L, "seed": seed, "words_sha256": ws, "hamming_vs_read0_sha256": ds}
        print(name, ws[:16], ds[:16], flush=True)
    with open(os.path.join(HERE, "stream_digests.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    sys.exit(main())
