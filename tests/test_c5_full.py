"""C5 counter at its per-GPU size and under skew, on the GPU.

Full shards: 125M x 32-nt reads drawn from a pool of U in {2^20, 2^24} 32-mers, uniform and Zipf
s = 1.1, counted by the partitioned insert in one call, compared to the generator-derived digests of
tests/golden/c5_digests.json (sorted (key, count, first) rows; the construction is pinned to the
reference counter's own digest and to oracle.count on CPU, tests/test_oracle_golden.py).

Skew: inputs that concentrate reads on few keys or few bins (Zipf pools, clustered runs, thousands of
distinct keys in one coarse bin that overflow its sub-bins and spill, the sentinel key "G" * 32 in
bulk), compared element-wise with oracle.count (counter.pyx:41-54 semantics: every duplicate
counted, dict order = first occurrence).
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
C5 = json.load(open(os.path.join(HERE, "golden", "c5_digests.json")))
SHARDS = sorted(k for k in C5 if not k.startswith("_") and "job" not in k)


def _table_rows(c):
    keys, lens, counts, first, parts = c.extract(1)
    m = int(parts.sum().item())
    assert not c.overflowed()
    k = keys[:m].cpu().numpy().view(np.uint64)
    return k, counts[:m].cpu().numpy().astype(np.uint64), first[:m].cpu().numpy().astype(np.uint64)


@pytest.mark.parametrize("case", SHARDS)
def test_c5_shard_digest(gpu, oracle, case):
    import shortseq_amd.batch as B
    d, meta = C5[case], C5["_meta"]
    n, U, i0, L = d["n"], d["U"], d["i0"], meta["L"]
    torch.cuda.empty_cache()
    if d["zipf_s"]:
        ascii = B.synth_zipf_reads(n, L, meta["seed"], meta["pool_seed"], B.zipf_cdf(U, d["zipf_s"]), i0=i0,
                                   device=gpu)
    else:
        ascii = B.synth_pool_reads(n, L, meta["seed"], meta["pool_seed"], U, i0=i0, device=gpu)
    c = B.GpuCounter(2 * U, device=gpu)
    c.insert(ascii, L, base_index=i0, partitioned=True)
    del ascii
    k, cnt, f = _table_rows(c)
    c.close()
    torch.cuda.empty_cache()
    assert len(k) == d["unique"]
    assert int(cnt.sum()) == n and int(cnt.max()) == d["max_count"]
    assert oracle.table_digest(k, cnt, f) == d["digest"], case


def _rows_of(exp, i0=0):
    k = np.array([w[0] for (w, _l, _c, _f) in exp], np.uint64)
    c = np.array([x[2] for x in exp], np.uint64)
    f = np.array([x[3] for x in exp], np.uint64) + np.uint64(i0)
    return k, c, f


def _count_gpu(B, gpu, a, L, cap, base=0, splits=1):
    c = B.GpuCounter(cap, device=gpu)
    t = torch.from_numpy(a).to(gpu).view(-1, L)
    n = t.shape[0]
    step = -(-n // splits)
    for lo in range(0, n, step):
        c.insert(t[lo:lo + step], L, base_index=base + lo, partitioned=True)
    rows = _table_rows(c)
    c.close()
    return rows


def test_counter_zipf_small(gpu, oracle):
    import shortseq_amd.batch as B
    U, n = 1 << 16, 3_000_000
    cdf = B.zipf_cdf(U, 1.1)
    a = B.synth_zipf_reads(n, 32, 5, 77, cdf, device=gpu)
    c = B.GpuCounter(1 << 22, device=gpu)
    c.insert(a, 32, partitioned=True)
    k, cnt, f = _table_rows(c)
    c.close()
    ek, ec, ef = oracle.pool_counter_table(5, 77, U, n, 32, cdf=cdf)
    assert oracle.table_digest(k, cnt, f) == oracle.table_digest(ek, ec, ef)


def test_counter_clustered_runs(gpu, oracle):
    """Sorted input: every key's copies contiguous (one key fills whole tiles)."""
    import shortseq_amd.batch as B
    n, U = 2_000_000, 997
    pool = oracle.gen_reads(9, 0, U, 32).reshape(U, 32)
    ids = (np.arange(n, dtype=np.int64) * U) // n
    a = np.ascontiguousarray(pool[ids]).reshape(-1)
    k, cnt, f = _count_gpu(B, gpu, a, 32, 1 << 20, splits=2)
    first = np.searchsorted(ids, np.arange(U))
    ek = oracle.gen_words(9, 0, U, 32)[:, 0]
    ec = np.bincount(ids, minlength=U).astype(np.uint64)
    assert oracle.table_digest(k, cnt, f) == oracle.table_digest(ek, ec, first.astype(np.uint64))


def test_counter_one_bin_spills(gpu, oracle):
    """6000 distinct keys that all hash into ONE coarse bin (a crafted worst case): every tile's bin
    is heavy, dedup keeps ~all of them, the sub-bins overflow and the rest spills to the direct insert."""
    import shortseq_amd.batch as B
    C = 0x9E3779B97F4A7C15
    Cinv = pow(C, -1, 1 << 64)
    rng = np.random.default_rng(3)
    hs = [(5 << 57) | int(x) for x in rng.integers(0, 1 << 57, size=6000, dtype=np.uint64)]
    keys = np.array([(h * Cinv) & ((1 << 64) - 1) for h in hs], dtype=np.uint64)
    shifts = np.arange(32, dtype=np.uint64) * np.uint64(2)
    codes = ((keys[:, None] >> shifts[None, :]) & np.uint64(3)).astype(np.int64)
    pool = np.frombuffer(b"ACTG", np.uint8)[codes]
    n = 400_000
    ids = rng.integers(0, len(keys), size=n)
    a = np.ascontiguousarray(pool[ids]).reshape(-1)
    k, cnt, f = _count_gpu(B, gpu, a, 32, 1 << 20)
    exp = oracle.count([a[i * 32:(i + 1) * 32].tobytes() for i in range(n)])
    assert oracle.table_digest(k, cnt, f) == oracle.table_digest(*_rows_of(exp))


def test_counter_sentinel_bulk(gpu, oracle):
    """30 % of the reads are "G" * 32 (packed word ~0 = the EMPTY pattern -> sentinel slot), shuffled."""
    import shortseq_amd.batch as B
    n = 1_000_000
    a = oracle.gen_pool_reads(4, 8, 50_000, 0, n, 32).reshape(n, 32)
    rng = np.random.default_rng(5)
    a[rng.random(n) < 0.3] = ord("G")
    a = a.reshape(-1)
    k, cnt, f = _count_gpu(B, gpu, a, 32, 1 << 20, base=1000, splits=3)
    exp = oracle.count([a[i * 32:(i + 1) * 32].tobytes() for i in range(n)])
    assert oracle.table_digest(k, cnt, f) == oracle.table_digest(*_rows_of(exp, 1000))


def test_counter_slot_hash_edge_keys(gpu, oracle):
    """The partition records carry h = key * C (C the slot-hash multiplier) and the aggregate's LDS
    slice marks free slots with h(~0): the key whose h is ~0 (K* = ~0 * C^-1) is an ordinary key
    there, "G" * 32 (key ~0) the sentinel, key 0 ("A" * 32) an ordinary one; all three in bulk among
    pool reads, over three batches (the later ones load the slices the first wrote back)."""
    import shortseq_amd.batch as B
    C = 0x9E3779B97F4A7C15
    kstar = (((1 << 64) - 1) * pow(C, -1, 1 << 64)) & ((1 << 64) - 1)
    assert (kstar * C) & ((1 << 64) - 1) == (1 << 64) - 1
    shifts = np.arange(32, dtype=np.uint64) * np.uint64(2)

    def read_of(key):
        codes = ((np.uint64(key) >> shifts) & np.uint64(3)).astype(np.int64)
        return np.frombuffer(b"ACTG", np.uint8)[codes]

    n = 1_200_000
    a = oracle.gen_pool_reads(6, 9, 60_000, 0, n, 32).reshape(n, 32)
    rng = np.random.default_rng(11)
    pick = rng.random(n)
    a[pick < 0.1] = read_of(kstar)
    a[(pick >= 0.1) & (pick < 0.2)] = ord("G")
    a[(pick >= 0.2) & (pick < 0.25)] = read_of(0)
    a = a.reshape(-1)
    k, cnt, f = _count_gpu(B, gpu, a, 32, 1 << 20, base=7, splits=3)
    exp = oracle.count([a[i * 32:(i + 1) * 32].tobytes() for i in range(n)])
    assert oracle.table_digest(k, cnt, f) == oracle.table_digest(*_rows_of(exp, 7))
    assert kstar in set(int(x) for x in k)


def test_counter_index_limit(gpu):
    """Read indices live in 32 bits: an insert past 2^32 - 1 is refused (SS_EARG), not truncated."""
    import shortseq_amd.batch as B
    from shortseq_amd._native import NativeError
    c = B.GpuCounter(1 << 12, device=gpu)
    a = B.synth_reads(100, 32, seed=1, device=gpu)
    c.insert(a, 32, base_index=(1 << 32) - 101)
    with pytest.raises(NativeError):
        c.insert(a, 32, base_index=(1 << 32) - 100)
    c.close()


def test_counter_slabs_multi_batch(gpu, oracle):
    """Fine-pass slabs (a 42M-read reservation on a 2^25-slot table: 320 reads per (sub-bin, region)
    on average, so the slab layout is on) with three 14M-read batches into ONE table: the second and
    third merge into already-written slices (no fresh reset).  Compared with the generator-derived
    table of all 42M draws."""
    import shortseq_amd.batch as B
    U, nb, nbat = 1 << 24, 14_000_000, 3
    c = B.GpuCounter(1 << 25, device=gpu)
    assert c.reserve(nb * nbat)
    for b in range(nbat):
        a = B.synth_pool_reads(nb, 32, 5, 77, U, i0=b * nb, device=gpu)
        c.insert(a, 32, base_index=b * nb, partitioned=True)
        del a
    k, cnt, f = _table_rows(c)
    c.close()
    torch.cuda.empty_cache()
    ek, ec, ef = oracle.pool_counter_table(5, 77, U, nb * nbat, 32)
    assert len(k) == len(ek)
    assert oracle.table_digest(k, cnt, f) == oracle.table_digest(ek, ec, ef)


def test_counter_slabs_zipf_spill(gpu, oracle):
    """Slab layout under Zipf s = 1.1 over 2^24 (40M reads, one batch, 128 regions per coarse bin): a
    region's copies of a heavy key arrive as one weighted record per coarse tile and overrun its slab,
    so records take the spill list (folded per wave, then inserted directly) -- still exact."""
    import shortseq_amd.batch as B
    U, n = 1 << 24, 40_000_000
    cdf = B.zipf_cdf(U, 1.1)
    a = B.synth_zipf_reads(n, 32, 5, 77, cdf, device=gpu)
    c = B.GpuCounter(1 << 25, device=gpu)
    c.insert(a, 32, base_index=7, partitioned=True)
    del a
    k, cnt, f = _table_rows(c)
    c.close()
    torch.cuda.empty_cache()
    ek, ec, ef = oracle.pool_counter_table(5, 77, U, n, 32, cdf=cdf)
    assert oracle.table_digest(k, cnt, f) == oracle.table_digest(ek, ec, ef + np.uint64(7))
