"""GPU parity: the HIP kernels (through the C ABI) against the oracle and the reference's fixtures.

Bit-exact for everything (integer work).  Small/medium sizes compare element-wise with the oracle;
full BASELINE sizes are checked through size-independent properties (known-answer generator words,
encode -> decode round trip) and whole-batch digests of the words and distances derived from the
generator (tests/golden/stream_digests.json).
"""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ALIASES = np.array([1, 3, 7, 20], np.uint8)


STREAM = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "stream_digests.json")))


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


def _rand_reads(rng, n, L, p_alias=0.0, p_bad=0.0):
    a = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=n * L)]
    if p_alias:
        m = rng.random(n * L) < p_alias
        a = np.where(m, ALIASES[rng.integers(0, 4, size=n * L)], a)
    if p_bad:
        m = rng.random(n * L) < p_bad
        a = np.where(m, np.uint8(ord("N")), a)
    return a.astype(np.uint8)


LENGTHS = sorted(set(list(range(1, 100)) + [112, 127, 128, 129, 160, 255, 256, 257, 500, 511, 512,
                                            513, 768, 1000, 1008, 1023, 1024]))


@pytest.mark.parametrize("p_alias", [0.0, 0.03])
def test_encode_fixed_all_lengths(gpu, oracle, p_alias):
    import shortseq_amd.batch as B
    rng = np.random.default_rng(11)
    for L in LENGTHS:
        n = 257
        a = _rand_reads(rng, n, L, p_alias)
        exp, rc, _ = oracle.encode_batch(a, n, L)
        assert rc == 0
        got = B.encode(torch.from_numpy(a).to(gpu).view(n, L), L)
        assert np.array_equal(_u64(got), exp), L


@pytest.mark.parametrize("L", [16, 32, 48, 64, 96, 100, 512, 1024])
def test_encode_stride_and_padding(gpu, oracle, L):
    """stride > L (general path even for L % 16 == 0 when stride is odd) and wpr > ceil(L/32)."""
    import shortseq_amd.batch as B
    rng = np.random.default_rng(L)
    n = 300
    for stride in (L, L + 16, L + 3):
        a = _rand_reads(rng, n, stride, p_alias=0.02)
        wpr = min(32, B.wpr_for(L) + 1)
        exp, rc, _ = oracle.encode_batch(a, n, L, stride=stride, wpr=wpr)
        got = B.encode(torch.from_numpy(a).to(gpu), L, stride=stride, wpr=wpr)
        assert np.array_equal(_u64(got), exp), (L, stride)


def test_golden_vectors_gpu(gpu, golden):
    import shortseq_amd.batch as B
    for v in golden["vectors"]:
        L = v["L"]
        if L == 0:
            continue
        t = torch.tensor(list(v["a"].encode()), dtype=torch.uint8, device=gpu).view(1, L)
        w = _u64(B.encode(t, L))[0]
        exp = [int(h, 16) for h in v["words_a"]][: B.wpr_for(L)]
        assert [int(x) for x in w] == exp, L
        s = B.decode(B.encode(t, L), L)
        assert bytes(s.cpu().numpy()[0]).decode() == v["str_a"]
        tb = torch.tensor(list(v["b"].encode()), dtype=torch.uint8, device=gpu).view(1, L)
        d = B.hamming_pair(B.encode(t, L), B.encode(tb, L), L)
        assert int(d[0]) == v["hamming"]


def test_golden_aliased_gpu(gpu, golden):
    import shortseq_amd.batch as B
    for c in golden["aliased"]:
        seq = bytes.fromhex(c["input_hex"])
        L = len(seq)
        t = torch.tensor(list(seq), dtype=torch.uint8, device=gpu).view(1, L)
        w = _u64(B.encode(t, L))[0]
        exp = [int(h, 16) for h in c["words"]][: B.wpr_for(L)]
        assert [int(x) for x in w] == exp, (L, c["pos"])


def test_errors_first_bad_read(gpu, oracle, golden):
    import shortseq_amd.batch as B
    rng = np.random.default_rng(5)
    for L in [1, 7, 16, 31, 32, 33, 48, 64, 96, 100, 512, 1024]:
        n = 1000
        a = _rand_reads(rng, n, L)
        bad_rows = sorted(rng.choice(n, size=3, replace=False))
        for r in bad_rows:
            a[r * L + rng.integers(0, L)] = ord("N")
        with pytest.raises(Exception) as ei:
            B.encode(torch.from_numpy(a).to(gpu).view(n, L), L)
        assert ei.value.read_index == bad_rows[0]
        seq = a[bad_rows[0] * L:(bad_rows[0] + 1) * L].tobytes()
        _, err = oracle.encode_one(seq, 32)
        bad = seq[err.byte_offset: err.byte_offset + err.nbytes]
        assert str(ei.value) == "Unsupported base character: " + bad.decode()
    # the golden error messages, one read per batch
    for c in golden["errors"]["pack"]:
        if c["ctor"] not in ("pack_bytes", "pack_bytes_hex") or "raises" not in c:
            continue
        seq = c["input"].encode() if c["ctor"] == "pack_bytes" else bytes.fromhex(c["input"])
        if len(seq) > 1024:
            continue
        t = torch.tensor(list(seq), dtype=torch.uint8, device=gpu).view(1, len(seq))
        with pytest.raises(BaseException) as ei:
            B.encode(t, len(seq))
        assert (type(ei.value).__name__, str(ei.value)) == (c["raises"], c["message"])


def test_decode_roundtrip_and_var(gpu, oracle):
    import shortseq_amd.batch as B
    rng = np.random.default_rng(9)
    for L in LENGTHS:
        n = 129
        a = _rand_reads(rng, n, L)
        w = B.encode(torch.from_numpy(a).to(gpu).view(n, L), L)
        back = B.decode(w, L)
        assert np.array_equal(back.cpu().numpy().reshape(-1), a), L
        assert np.array_equal(back.cpu().numpy().reshape(-1), oracle.decode_batch(_u64(w), n, L))
    # ragged batch 0..1024 incl. empty reads
    lens = np.array([0, 1, 31, 32, 33, 64, 95, 96, 97, 1000, 1024, 5, 0, 512] * 20, np.int32)
    reads = [_rand_reads(rng, 1, int(L), p_alias=0.02).tobytes() for L in lens]
    offs = np.zeros(len(lens), np.int64)
    offs[1:] = np.cumsum(lens[:-1])
    blob = np.frombuffer(b"".join(reads) + b"\0", np.uint8)
    words = B.encode_var(torch.from_numpy(blob.copy()).to(gpu), torch.from_numpy(offs).to(gpu),
                         torch.from_numpy(lens).to(gpu), wpr=32)
    wn = _u64(words)
    for i, r in enumerate(reads):
        exp, _ = oracle.encode_one(r, 32)
        assert np.array_equal(wn[i], exp), (i, len(r))
    out = B.decode_var(words, torch.from_numpy(lens).to(gpu), torch.from_numpy(offs).to(gpu))
    clean = b"".join(oracle.decode_batch(wn[i:i + 1], 1, int(L), 32).tobytes() for i, L in enumerate(lens))
    assert out.cpu().numpy().tobytes() == clean
    # too-long read in a ragged batch
    lens2 = np.array([10, 1025, 10], np.int32)
    offs2 = np.array([0, 10, 1035], np.int64)
    blob2 = np.frombuffer(b"A" * 1045, np.uint8).copy()
    with pytest.raises(Exception) as ei:
        B.encode_var(torch.from_numpy(blob2).to(gpu), torch.from_numpy(offs2).to(gpu),
                     torch.from_numpy(lens2).to(gpu))
    assert str(ei.value) == "Sequences longer than 1024 bases are not supported."
    assert ei.value.read_index == 1


def test_hamming(gpu, oracle):
    import shortseq_amd.batch as B
    rng = np.random.default_rng(13)
    for L in LENGTHS:
        n = 200
        a = _rand_reads(rng, n, L, p_alias=0.01)
        b = a.copy()
        flip = rng.random(n * L) < 0.1
        b[flip] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, flip.sum())]
        wa = B.encode(torch.from_numpy(a).to(gpu).view(n, L), L)
        wb = B.encode(torch.from_numpy(b).to(gpu).view(n, L), L)
        pair = B.hamming_pair(wa, wb, L).cpu().numpy().astype(np.uint32)
        assert np.array_equal(pair, oracle.hamming_pair_batch(_u64(wa), _u64(wb), n, L)), L
        ref = B.hamming_ref(wa, L, wb[7]).cpu().numpy().astype(np.uint32)
        assert np.array_equal(ref, oracle.hamming_ref_batch(_u64(wa), n, L, _u64(wb)[7])), L
        words, dist = B.encode_hamming_ref(torch.from_numpy(a).to(gpu).view(n, L), L, wb[7])
        assert np.array_equal(_u64(words), _u64(wa))
        assert np.array_equal(dist.cpu().numpy().astype(np.uint32), ref), L
        _, dist2 = B.encode_hamming_ref(torch.from_numpy(a).to(gpu).view(n, L), L, wb[7], store_words=False)
        assert np.array_equal(dist2.cpu().numpy().astype(np.uint32), ref), L


@pytest.mark.parametrize("L", [1, 31, 32, 33, 64, 96, 100, 128, 150, 176, 200, 224, 256, 300, 500, 512, 1000, 1024])
def test_hamming_dense_multiblock(gpu, oracle, L):
    """k_ham_dense (packed rows, wpr == words): batches spanning several blocks, odd word counts
    ending on a half pair, and row views off the 16-B grid (those take k_ham_group)."""
    import shortseq_amd.batch as B
    rng = np.random.default_rng(1000 + L)
    for n in (1, 3, 4097, 9001):
        a = _rand_reads(rng, n, L, p_alias=0.01)
        b = a.copy()
        flip = rng.random(n * L) < 0.2
        b[flip] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, flip.sum())]
        wa = B.encode(torch.from_numpy(a).to(gpu).view(n, L), L)
        wb = B.encode(torch.from_numpy(b).to(gpu).view(n, L), L)
        ua, ub = _u64(wa), _u64(wb)
        pair = B.hamming_pair(wa, wb, L).cpu().numpy().astype(np.uint32)
        assert np.array_equal(pair, oracle.hamming_pair_batch(ua, ub, n, L)), (L, n)
        k = n // 2
        ref = B.hamming_ref(wa, L, wb[k]).cpu().numpy().astype(np.uint32)
        assert np.array_equal(ref, oracle.hamming_ref_batch(ua, n, L, ub[k])), (L, n)
        if n > 1:
            p1 = B.hamming_pair(wa[1:], wb[1:], L).cpu().numpy().astype(np.uint32)
            assert np.array_equal(p1, pair[1:]), (L, n)
            r1 = B.hamming_ref(wa[1:], L, wb[k]).cpu().numpy().astype(np.uint32)
            assert np.array_equal(r1, ref[1:]), (L, n)


def test_hamming_out_alignment(gpu, oracle):
    """Distance arrays off the 8-B grid (and reference / row pointers off 16 B) take the lane-group
    kernel; the results are the same as the streaming kernels'."""
    import shortseq_amd.batch as B
    from shortseq_amd._native import lib
    rng = np.random.default_rng(77)
    for L in (32, 96, 512):
        n = 3001
        a = _rand_reads(rng, n, L)
        wa = B.encode(torch.from_numpy(a).to(gpu).view(n, L), L)
        wpr = wa.shape[1]
        ref = wa[n // 3].clone()
        want = oracle.hamming_ref_batch(_u64(wa), n, L, _u64(ref.view(1, -1))[0])
        buf = torch.zeros(n + 1, dtype=torch.int32, device=gpu)
        out = buf[1:]                                   # 4-B aligned, not 8-B
        s = torch.cuda.current_stream(gpu).cuda_stream
        assert lib().ss_hamming_ref(wa.data_ptr(), n, L, wpr, ref.data_ptr(), out.data_ptr(), s) == 0
        assert np.array_equal(out.cpu().numpy().astype(np.uint32), want), L
        pair = torch.zeros(n + 1, dtype=torch.int32, device=gpu)[1:]
        assert lib().ss_hamming_pair(wa.data_ptr(), wa.data_ptr(), n, L, wpr, pair.data_ptr(), s) == 0
        assert int(pair.abs().sum()) == 0, L
        # 8-B aligned, off the 16-B grid: the streaming kernels, with the 96-nt kernel's per-distance
        # stores in place of its dwordx4 runs
        out8 = torch.zeros(n + 2, dtype=torch.int32, device=gpu)[2:]
        assert out8.data_ptr() % 16 == 8
        assert lib().ss_hamming_ref(wa.data_ptr(), n, L, wpr, ref.data_ptr(), out8.data_ptr(), s) == 0
        assert np.array_equal(out8.cpu().numpy().astype(np.uint32), want), L
        pair8 = torch.full((n + 2,), -1, dtype=torch.int32, device=gpu)[2:]
        assert lib().ss_hamming_pair(wa.data_ptr(), wa.data_ptr(), n, L, wpr, pair8.data_ptr(), s) == 0
        assert int(pair8.abs().sum()) == 0, L


def test_synth_matches_oracle_generator(gpu, oracle):
    import shortseq_amd.batch as B
    for L in [1, 16, 31, 32, 33, 96, 100, 512, 1024]:
        n = 500
        t = B.synth_reads(n, L, seed=42, i0=1000, device=gpu)
        assert np.array_equal(t.cpu().numpy().reshape(-1), oracle.gen_reads(42, 1000, n, L)), L
        p = B.synth_pool_reads(n, L, 3, 4, 97, i0=77, device=gpu)
        exp = oracle.gen_pool_reads(3, 4, 97, 77, n, L)
        assert np.array_equal(p.cpu().numpy().reshape(-1), exp), L


@pytest.mark.parametrize("key", ["1000000x32", "1000000x96", "200000x512", "300000x100"])
def test_golden_digests_gpu(gpu, digests, key):
    """Reference-produced SHA-256 of the packed words / distances, reproduced on the GPU."""
    import shortseq_amd.batch as B
    d = digests[key]
    n, L = d["n"], d["L"]
    ascii = B.synth_reads(n, L, seed=d["seed"], device=gpu)
    words = B.encode(ascii, L)
    assert _sha(_u64(words)) == d["words_sha256"]
    m = d["hamming_vs_read0_n"]
    _, dist = B.encode_hamming_ref(ascii[:m], L, words[0], store_words=False)
    dist = dist.cpu().numpy().astype(np.uint32)
    assert _sha(dist) == d["hamming_vs_read0_sha256"]


@pytest.mark.parametrize("L,n", [(32, 100_000_000), (96, 100_000_000), (512, 50_000_000)])
def test_full_size_properties(gpu, oracle, L, n):
    """BASELINE sizes: round trip + checksum of sampled reads vs oracle + fused hamming sum."""
    import shortseq_amd.batch as B
    torch.cuda.empty_cache()
    ascii = B.synth_reads(n, L, seed=1, device=gpu)
    words = B.encode(ascii, L)
    back = B.decode(words, L)
    assert torch.equal(back, ascii)
    del back
    idx = np.linspace(0, n - 1, 4096).astype(np.int64)
    samp = _u64(words[torch.from_numpy(idx).to(gpu)])
    exp = np.stack([oracle.gen_words(1, int(i), 1, L)[0] for i in idx])
    assert np.array_equal(samp, exp)
    # whole-batch digests derived from the generator (tests/golden/gen_stream_digests.py, pinned to
    # the oracle on CPU by tests/test_oracle_golden.py::test_stream_digest_construction)
    d = STREAM[f"{'C2' if L == 32 else 'C3' if L == 96 else 'C4'}_{n}x{L}"]
    assert d["seed"] == 1
    assert _sha(_u64(words)) == d["words_sha256"]
    # hamming vs read 0: the dense kernel on the packed words, and for C3 the fused encode+hamming
    d2 = B.hamming_ref(words, L, words[0])
    assert _sha(d2.cpu().numpy().astype(np.uint32)) == d["hamming_vs_read0_sha256"]
    if L == 96:
        _, dist = B.encode_hamming_ref(ascii, L, words[0], store_words=False)
        assert torch.equal(dist, d2)
    del d2
    del ascii, words
    torch.cuda.empty_cache()


def test_counter_gpu(gpu, oracle, digests):
    import shortseq_amd.batch as B
    d = digests["counter_1000000x32_pool65536"]
    n, L = d["n"], d["L"]
    ascii = B.synth_pool_reads(n, L, d["seed"], d["pool_seed"], d["U"], device=gpu)
    c = B.GpuCounter(1 << 18, device=gpu)
    half = n // 2
    c.insert(ascii[:half], L, base_index=0)
    c.insert(ascii[half:], L, base_index=half)
    assert c.size() == d["unique"]
    keys, counts, first = c.items_sorted()
    ordered = np.stack([keys, np.full(len(keys), L, np.uint64), counts.astype(np.uint64)], 1)
    assert _sha(ordered.astype(np.uint64)) == d["ordered_sha256"]
    c.close()
    # mixed small cases vs oracle, incl. the EMPTY-colliding word (G * 32) and L = 16 / odd L
    rng = np.random.default_rng(1)
    for L in [1, 5, 16, 31, 32]:
        pool = [_rand_reads(rng, 1, L, p_alias=0.05).tobytes() for _ in range(50)]
        if L == 32:
            pool[3] = b"G" * 32
        reads = [pool[i] for i in rng.integers(0, len(pool), 5000)]
        exp = oracle.count(reads)
        c = B.GpuCounter(1024, device=gpu)
        t = torch.from_numpy(np.frombuffer(b"".join(reads), np.uint8).copy()).to(gpu).view(-1, L)
        c.insert(t, L)
        k, cnt, f = c.items_sorted()
        assert [(int(x),) for x in k] == [w for (w, _L, _c, _f) in exp]
        assert list(cnt) == [cc for (_w, _L, cc, _f) in exp]
        assert list(f) == [ff for (_w, _L, _c, ff) in exp]
        c.close()


def test_counter_extract_parts_and_merge(gpu, oracle):
    import shortseq_amd.batch as B
    n, L, U = 200_000, 32, 5000
    ascii = B.synth_pool_reads(n, L, 9, 10, U, device=gpu)
    full = B.GpuCounter(1 << 14, device=gpu)
    full.insert(ascii, L)
    k0, c0, f0 = full.items_sorted()
    # two "ranks": each counts half, partitions by owner, owners merge
    parts = []
    for r in range(2):
        c = B.GpuCounter(1 << 14, device=gpu)
        c.insert(ascii[r * n // 2:(r + 1) * n // 2], L, base_index=r * n // 2)
        parts.append(c.extract(n_parts=3))
    merged = [B.GpuCounter(1 << 14, device=gpu) for _ in range(3)]
    for keys, lens, counts, first, pc in parts:
        pc = pc.cpu().numpy()
        off = np.concatenate([[0], np.cumsum(pc)])
        for p in range(3):
            s, e = int(off[p]), int(off[p + 1])
            merged[p].merge(keys[s:e], counts[s:e], first[s:e], L)
    allk, allc, allf = [], [], []
    for m in merged:
        k, c, f = m.items_sorted()
        allk.append(k), allc.append(c), allf.append(f)
    k, c, f = np.concatenate(allk), np.concatenate(allc), np.concatenate(allf)
    o = np.argsort(f, kind="stable")
    assert np.array_equal(k[o], k0) and np.array_equal(c[o], c0) and np.array_equal(f[o], f0)
    assert c0.sum() == n


@pytest.mark.parametrize("cap,U,n", [(1 << 12, 300, 200_000), (1 << 16, 20_000, 500_000),
                                     (1 << 22, 1_000_000, 3_000_000),
                                     # > 128 regions: the optimistic coarse partition; few keys pile
                                     # up in a few coarse bins -> overflow -> direct-insert fallback
                                     (1 << 20, 5, 400_000), (1 << 20, 3000, 400_000)])
def test_counter_partitioned_equals_direct(gpu, oracle, cap, U, n):
    """The partitioned (LDS-aggregated) insert and the direct atomic insert give identical tables,
    across several inserts (persistent table, global first indices), incl. the EMPTY-colliding key."""
    import shortseq_amd.batch as B
    L = 32
    ascii = B.synth_pool_reads(n, L, 21, 22, U, device=gpu)
    ascii[7] = ord("G")                     # read 7 = "G" * 32 -> packed word ~0 (sentinel slot)
    ascii[n // 2 + 3] = ord("G")
    res = []
    for partitioned in (True, False):
        c = B.GpuCounter(cap, device=gpu)
        third = n // 3
        for lo, hi in ((0, third), (third, 2 * third), (2 * third, n)):
            c.insert(ascii[lo:hi], L, base_index=lo, partitioned=partitioned)
        assert not c.overflowed()
        res.append(c.items_sorted())
        c.close()
    (k1, c1, f1), (k2, c2, f2) = res
    assert np.array_equal(k1, k2) and np.array_equal(c1, c2) and np.array_equal(f1, f2)
    assert int(c1.sum()) == n
    assert k1[np.argmax(f1 == 7)] == np.uint64(0xFFFFFFFFFFFFFFFF)
    # and against the oracle on the first 200k reads
    m = min(n, 200_000)
    c = B.GpuCounter(cap, device=gpu)
    c.insert(ascii[:m], L, partitioned=True)
    k, cnt, f = c.items_sorted()
    a = ascii[:m].cpu().numpy().reshape(-1)
    exp = oracle.count([a[i * L:(i + 1) * L].tobytes() for i in range(m)])
    assert [int(x) for x in k] == [w[0] for (w, _L, _c, _f) in exp]
    assert list(cnt) == [cc for (_w, _L, cc, _f) in exp]
    c.close()


@pytest.mark.parametrize("L,cap,U,n", [(33, 1 << 12, 500, 50_000), (64, 1 << 16, 5000, 200_000),
                                       (96, 1 << 20, 20_000, 300_000), (100, 1 << 14, 3000, 100_000),
                                       (150, 1 << 18, 50_000, 200_000), (512, 1 << 13, 800, 30_000),
                                       (1024, 1 << 12, 300, 10_000)])
def test_counter_multiword(gpu, oracle, L, cap, U, n):
    """Multi-word keys (L > 32: ShortSeq192 / ShortSeqVar keys): fingerprint-partitioned insert with
    word comparison, over three inserts into one table (global first indices), against the oracle
    on the same reads (keys, counts, first occurrence, dict order).  Pool reads one base apart
    (same fingerprint region unlikely, same words except one) check the word comparison."""
    import shortseq_amd.batch as B
    ascii = B.synth_pool_reads(n, L, 31 + L, 32, U, device=gpu)
    ascii[5] = ascii[4]
    ascii[5, L - 1] = ord("A") if int(ascii[4, L - 1]) != ord("A") else ord("C")   # last base differs
    ascii[6] = ascii[4]
    ascii[6, 0] = ord("G") if int(ascii[4, 0]) != ord("G") else ord("T")           # first base differs
    c = B.GpuCounter(cap, device=gpu)
    third = n // 3
    for lo, hi in ((0, third), (third, 2 * third), (2 * third, n)):
        c.insert(ascii[lo:hi], L, base_index=lo)
    assert c.words == (L + 31) // 32
    assert not c.overflowed()
    words, cnt, f = c.items_sorted_words()
    a = ascii.cpu().numpy().reshape(-1)
    exp = oracle.count([a[i * L:(i + 1) * L].tobytes() for i in range(n)])
    assert [tuple(int(x) for x in row) for row in words] == [w for (w, _L, _c, _f) in exp]
    assert list(cnt) == [cc for (_w, _L, cc, _f) in exp]
    assert list(f) == [ff for (_w, _L, _c, ff) in exp]
    assert c.size() == len(exp)
    c.close()


def test_counter_multiword_bad_read(gpu):
    import shortseq_amd.batch as B
    L, n = 150, 70_000
    ascii = B.synth_pool_reads(n, L, 3, 4, 100, device=gpu)
    ascii[40_000, 77] = ord("N")
    ascii[50_000, 3] = ord("*")
    c = B.GpuCounter(1 << 12, device=gpu)
    c.insert(ascii, L, check_errors=False)
    assert int(B.first_bad_buffer(gpu).item()) == 40_000
    with pytest.raises(Exception):
        c.insert(ascii, L)
    c.close()


@pytest.mark.parametrize("W,U,n,shift", [(3, 5000, 200_000, 0), (6, 100_000, 400_000, 0), (33, 300, 20_000, 0),
                                         (2, 3000, 100_000, 1), (4, 50_000, 300_000, 0), (4, 50_000, 300_000, 1),
                                         (5, 20_000, 150_000, 1), (6, 20_000, 150_000, 1), (7, 20_000, 150_000, 0),
                                         (8, 20_000, 150_000, 0)])
def test_counter_insert_words(gpu, W, U, n, shift):
    """Packed-word keys (ss_counter_set_words / ss_counter_insert_words, the drop-in engine's
    length-class tables): rows compared whole, counts and first index against numpy over two
    inserts; rows one word apart (incl. only the last word, the class's length word) stay apart.
    W 2-7 take the aggregate's chunked row gathers (shift 1: rows 8 B off a 16-B boundary, the
    realigning form); W 8 and 33 the any-width one."""
    import torch
    import shortseq_amd.batch as B
    rng = np.random.default_rng(W)
    pool = rng.integers(0, 1 << 62, size=(U, W), dtype=np.int64)
    pool[1] = pool[0]
    pool[1, W - 1] ^= 1                       # differs in the last word only
    pool[2] = pool[0]
    pool[2, 0] ^= 1 << 40                     # differs in the first word only
    idx = rng.integers(0, U, size=n)
    idx[:3] = [0, 1, 2]
    rows = pool[idx]
    c = B.GpuCounter(1 << max(12, int(2 * U).bit_length()), device=gpu)
    h = n // 2
    def dev_rows(a):
        buf = torch.zeros(a.size + 2, dtype=torch.int64, device=gpu)
        v = buf[shift:shift + a.size].view(-1, W)
        v.copy_(torch.from_numpy(a))
        return v

    c.insert_words(dev_rows(rows[:h]))
    c.insert_words(dev_rows(rows[h:]), base_index=h)
    assert c.words == W and c.length == -2 and not c.overflowed()
    words, cnt, f = c.items_sorted_words()
    _u, first, counts = np.unique(idx, return_index=True, return_counts=True)
    o = np.argsort(first)
    assert np.array_equal(f, first[o]) and np.array_equal(cnt, counts[o])
    assert np.array_equal(words.view(np.int64), rows[first[o]])
    with pytest.raises(Exception):            # a packed-word handle takes no ASCII inserts
        c.insert(B.synth_reads(10, 40, seed=1, device=gpu), 40)
    c.close()


@pytest.mark.parametrize("world,cap,U,n", [(3, 1 << 16, 20_000, 300_000), (8, 1 << 22, 500_000, 1_000_000),
                                           (2, 1 << 12, 300, 50_000)])
def test_counter_region_owner_merge(gpu, oracle, world, cap, U, n):
    """Region-range ownership on one GPU: `world` tables count their shards, extract the other
    owners' regions (region-sorted runs), each owner folds the runs into its own table; the union
    of the owned regions equals the oracle over the whole stream (incl. the sentinel key ~0)."""
    import torch
    import shortseq_amd.batch as B
    from shortseq_amd.dist import owner_of_region_np
    L = 32
    ascii = B.synth_pool_reads(n, L, 31, 32, U, device=gpu)
    ascii[5] = ord("G")                        # "G" * 32: the EMPTY-colliding sentinel key
    ascii[n - 2] = ord("G")
    per = n // world
    tabs = [B.GpuCounter(cap, device=gpu) for _ in range(world)]
    ex = []
    for r, t in enumerate(tabs):
        hi = n if r == world - 1 else (r + 1) * per
        t.insert(ascii[r * per:hi], L, base_index=r * per)
        keys, _l, counts, first, parts = t.extract_ranges(world)
        starts = [0] + np.cumsum(parts.cpu().numpy()).tolist()
        ex.append((keys, counts, first, starts))
    for p, t in enumerate(tabs):
        ks, cs, fs, runs, pos = [], [], [], [], 0
        for src in range(world):
            keys, counts, first, starts = ex[src]
            a, b = int(starts[p]), int(starts[p + 1])
            ks.append(keys[a:b]), cs.append(counts[a:b]), fs.append(first[a:b])
            if src != p and b > a:
                runs.append((pos, pos + b - a))
            pos += b - a
        t.merge_runs(torch.cat(ks), torch.cat(cs), torch.cat(fs), runs, p, world, L)
    torch.cuda.synchronize()
    allk, allc, allf = [], [], []
    for p, t in enumerate(tabs):
        assert not t.overflowed()
        keys, _l, counts, first, parts = t.extract_ranges(world)
        starts = [0] + np.cumsum(parts.cpu().numpy()).tolist()
        a, b = int(starts[p]), int(starts[p + 1])
        k = keys[a:b].cpu().numpy().view(np.uint64)
        assert (owner_of_region_np(k, world, *t.geometry()) == p).all()
        allk.append(k), allc.append(counts[a:b].cpu().numpy()), allf.append(first[a:b].cpu().numpy())
        t.close()
    k, c, f = np.concatenate(allk), np.concatenate(allc), np.concatenate(allf)
    o = np.argsort(f, kind="stable")
    a = ascii.cpu().numpy().reshape(-1)
    exp = oracle.count([a[i * L:(i + 1) * L].tobytes() for i in range(n)])
    assert [int(x) for x in k[o]] == [w[0] for (w, _L, _c, _f) in exp]
    assert [int(x) for x in c[o]] == [cc for (_w, _L, cc, _f) in exp]
    assert [int(x) for x in f[o]] == [ff for (_w, _L, _c, ff) in exp]


@pytest.mark.parametrize("world,cap,U,n,mode", [
    (2, 1 << 19, 5000, 300_000, "partitioned"),     # occupancy from the aggregate (one pass)
    (2, 1 << 17, 5000, 200_000, "partitioned"),     # <= 128 regions: the exact partition passes
    (3, 1 << 19, 40_000, 400_000, "partitioned"),
    (8, 1 << 20, 300_000, 1_200_000, "partitioned"),
    (3, 1 << 19, 3, 300_000, "overflow"),           # 3 keys: the optimistic partition overflows
    (2, 1 << 16, 900, 20_000, "direct"),            # small batches: direct insert, counting pass
])
def test_counter_packed_exchange(gpu, oracle, world, cap, U, n, mode):
    """The multi-GPU exchange in packed records on one GPU: `world` tables count their shards, pack
    the other owners' regions (16-B records, first relative to the shard base), each owner folds
    the records of every other table into its own; the union of the owned regions equals the
    oracle over the whole stream (incl. the sentinel key ~0)."""
    import torch
    import shortseq_amd.batch as B
    from shortseq_amd.dist import owner_of_region_np
    L = 32
    ascii = B.synth_pool_reads(n, L, 41, 42, U, device=gpu)
    ascii[7] = ord("G")                        # "G" * 32: the EMPTY-colliding sentinel key
    ascii[n - 3] = ord("G")
    per = n // world
    tabs = [B.GpuCounter(cap, device=gpu) for _ in range(world)]
    packs = []
    for r, t in enumerate(tabs):
        hi = n if r == world - 1 else (r + 1) * per
        t.insert(ascii[r * per:hi], L, base_index=r * per, partitioned=(mode != "direct"))
        rec, parts = t.pack_ranges(world, skip=r, first_base=r * per)
        assert not t.overflowed()
        pc = parts.cpu().numpy()
        assert pc[r] == 0
        starts = [0] + np.cumsum(pc).tolist()
        packs.append((rec, starts))
    for p, t in enumerate(tabs):
        segs, runs, pos = [], [], 0
        for src in range(world):
            rec, starts = packs[src]
            a, b = int(starts[p]), int(starts[p + 1])
            if b > a:
                segs.append(rec[a:b])
                runs.append((pos, pos + b - a, src * per))
                pos += b - a
        if segs:
            t.merge_packed(torch.cat(segs), runs, p, world, L)
    torch.cuda.synchronize()
    allk, allc, allf = [], [], []
    for p, t in enumerate(tabs):
        assert not t.overflowed()
        keys, _l, counts, first, parts = t.extract_ranges(world)
        starts = [0] + np.cumsum(parts.cpu().numpy()).tolist()
        a, b = int(starts[p]), int(starts[p + 1])
        k = keys[a:b].cpu().numpy().view(np.uint64)
        assert (owner_of_region_np(k, world, *t.geometry()) == p).all()
        allk.append(k), allc.append(counts[a:b].cpu().numpy()), allf.append(first[a:b].cpu().numpy())
        t.close()
    k, c, f = np.concatenate(allk), np.concatenate(allc), np.concatenate(allf)
    o = np.argsort(f, kind="stable")
    a = ascii.cpu().numpy().reshape(-1)
    exp = oracle.count([a[i * L:(i + 1) * L].tobytes() for i in range(n)])
    assert [int(x) for x in k[o]] == [w[0] for (w, _L, _c, _f) in exp]
    assert [int(x) for x in c[o]] == [cc for (_w, _L, cc, _f) in exp]
    assert [int(x) for x in f[o]] == [ff for (_w, _L, _c, ff) in exp]


def test_counter_pack_records_layout(gpu):
    """pack_ranges record fields and grouping: part order, region order inside a part, counts and
    first indices relative to first_base, the sentinel last in its owner's segment."""
    import shortseq_amd.batch as B
    from shortseq_amd.dist import owner_of_region_np
    L, n, world = 32, 200_000, 4
    ascii = B.synth_pool_reads(n, L, 3, 4, 20_000, device=gpu)
    ascii[11] = ord("G")
    t = B.GpuCounter(1 << 18, device=gpu)
    t.insert(ascii, L, base_index=1000)
    rec, parts = t.pack_ranges(world, skip=-1, first_base=1000)
    keys, _l, counts, first, eparts = t.extract_ranges(world)
    assert np.array_equal(parts.cpu().numpy(), eparts.cpu().numpy())
    m = int(parts.sum())
    r = rec[:m].cpu().numpy()
    k = r[:, 0].view(np.uint64)
    c = (r[:, 1].view(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.int64)
    f = (r[:, 1].view(np.uint64) >> np.uint64(32)).astype(np.int64) + 1000
    log2cap, slice_log = t.geometry()
    own = owner_of_region_np(k, world, log2cap, slice_log)
    starts = np.cumsum([0] + parts.cpu().numpy().tolist())
    for p in range(world):
        seg = slice(starts[p], starts[p + 1])
        assert (own[seg] == p).all()
        kk = k[seg]
        notsent = kk != np.uint64(0xFFFFFFFFFFFFFFFF)
        with np.errstate(over="ignore"):
            reg = ((kk[notsent] * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(64 - log2cap)) >> np.uint64(slice_log)
        assert (np.diff(reg.astype(np.int64)) >= 0).all()
        if not notsent.all():
            assert not notsent[-1] and notsent[:-1].all()
    ek = keys[:m].cpu().numpy().view(np.uint64)
    d = dict(zip(ek.tolist(), zip(counts[:m].cpu().numpy().tolist(), first[:m].cpu().numpy().tolist())))
    assert len(d) == m
    for kk, cc, ff in zip(k.tolist(), c.tolist(), f.tolist()):
        assert d[kk] == (cc, ff)
    t.close()


@pytest.mark.parametrize("U,n,cap,partitioned", [
    (40_000, 400_000, 1 << 19, True),      # optimistic partition, fresh aggregate
    (3, 300_000, 1 << 19, True),           # optimistic overflow: fresh slice resets + direct insert
    (5_000, 200_000, 1 << 17, True),       # exact partition passes, fresh aggregate
    (900, 20_000, 1 << 16, False),         # direct insert: the pending reset is flushed first
])
def test_counter_lazy_reset(gpu, oracle, U, n, cap, partitioned):
    """ss_counter_reset is lazy (the next partitioned insert writes whole slices instead of a memset
    + slice read): a table filled with other keys, reset, then counted equals the oracle; so does
    reset -> size (flush) and two inserts after one reset."""
    import shortseq_amd.batch as B
    L = 32
    t = B.GpuCounter(cap, device=gpu)
    junk = B.synth_pool_reads(n, L, 91, 92, 50_000, device=gpu)
    t.insert(junk, L, partitioned=partitioned)
    ascii = B.synth_pool_reads(n, L, 51, 52, U, device=gpu)
    ascii[9] = ord("G")                        # "G" * 32: the sentinel key
    t.reset()
    t.insert(ascii, L, partitioned=partitioned)
    k, c, f = t.items_sorted()
    a = ascii.cpu().numpy().reshape(-1)
    exp = oracle.count([a[i * L:(i + 1) * L].tobytes() for i in range(n)])
    assert [int(x) for x in k] == [w[0] for (w, _L, _c, _f) in exp]
    assert [int(x) for x in c] == [cc for (_w, _L, cc, _f) in exp]
    assert [int(x) for x in f] == [ff for (_w, _L, _c, ff) in exp]
    assert not t.overflowed()
    t.reset()
    assert t.size() == 0
    # two halves after one reset: the second insert sees the first's slices
    t.reset()
    t.insert(ascii[: n // 2], L, partitioned=partitioned)
    t.insert(ascii[n // 2:], L, base_index=n // 2, partitioned=partitioned)
    k2, c2, f2 = t.items_sorted()
    assert np.array_equal(k2, k) and np.array_equal(c2, c) and np.array_equal(f2, f)
    t.close()
