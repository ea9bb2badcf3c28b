"""Pin the CPU oracle (oracle/ss_oracle.c) to the reference's own outputs.

Fixtures in tests/golden/ were produced by tests/golden/gen_golden.py from the unmodified reference
(built by oracle/build_ref.sh).  When oracle/_ref is present the oracle is also fuzzed directly
against the reference's compiled kernels (the capsule functions of short_seq_64.pyx:96 and
util.pyx:78).  CPU only.
"""
import hashlib

import numpy as np
import pytest

ALIASES = [1, 3, 7, 20]


def _w(hexlist):
    return [int(h, 16) for h in hexlist]


def _wpr_class(L):
    return 1 if L <= 32 else (3 if L <= 96 else (L + 31) // 32)


def test_vectors(oracle, golden):
    assert len(golden["vectors"]) > 100
    for v in golden["vectors"]:
        L = v["L"]
        words, err = oracle.encode_one(v["a"].encode(), _wpr_class(L))
        assert err.kind == 0
        assert [int(x) for x in words] == _w(v["words_a"]), L
        wb, _ = oracle.encode_one(v["b"].encode(), _wpr_class(L))
        assert [int(x) for x in wb] == _w(v["words_b"])
        out = np.zeros(max(L, 1), np.uint8)
        oracle.lib().ora_decode(words.ctypes.data, L, out.ctypes.data)
        assert bytes(out[:L]).decode() == v["str_a"]
        assert oracle.lib().ora_hamming(words.ctypes.data, wb.ctypes.data, L) == v["hamming"]


def test_aliased_bytes(oracle, golden):
    """SURVEY Q1 (table-path carry) and Q2 (full-block path, no carry)."""
    n = 0
    for c in golden["aliased"]:
        seq = bytes.fromhex(c["input_hex"])
        words, err = oracle.encode_one(seq, _wpr_class(len(seq)))
        assert "raises" not in c
        assert err.kind == 0
        assert [int(x) for x in words] == _w(c["words"]), (c["L"], c["pos"])
        n += 1
    assert n > 250


def _message(seq: bytes, err):
    if err.kind == 2:
        return "Exception", "Sequences longer than 1024 bases are not supported."
    bad = seq[err.byte_offset: err.byte_offset + err.nbytes]
    try:
        return "Exception", "Unsupported base character: " + bad.decode("ascii")
    except UnicodeDecodeError as e:
        return "UnicodeDecodeError", str(e)


def test_error_cases(oracle, golden):
    checked = 0
    for c in golden["errors"]["pack"]:
        if c["ctor"] in ("pack_str", "pack_bytes", "from_bytes", "from_str"):
            seq = c["input"].encode()
        elif c["ctor"] == "pack_bytes_hex":
            seq = bytes.fromhex(c["input"])
        else:
            continue  # Python type errors: covered by the drop-in front tests
        words, err = oracle.encode_one(seq, max(32, _wpr_class(len(seq))))
        if "raises" not in c:
            assert err.kind == 0
            continue
        assert err.kind in (1, 2)
        assert _message(seq, err) == (c["raises"], c["message"]), c["input"][:80]
        checked += 1
    assert checked > 40


def test_counter_cases(oracle, golden):
    for case in golden["counter"]:
        if "reads_hex" not in case:
            continue
        reads = [bytes.fromhex(h) for h in case["reads_hex"]]
        if "raises" in case:
            with pytest.raises(ValueError) as ei:
                oracle.count(reads)
            kind, idx, off, nb = ei.value.args[0]
            assert kind == 1 and idx == 1
            continue
        got = oracle.count(reads)
        exp = [(tuple(_w(it["words"])[:1 if it["length"] <= 32 else (it["length"] + 31) // 32]),
                it["length"], it["count"]) for it in case["items"]]
        assert [(w, L, c) for (w, L, c, _f) in got] == exp


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("key", ["1000000x32", "1000000x96", "200000x512", "300000x100"])
def test_digests(oracle, digests, key):
    d = digests[key]
    n, L, seed = d["n"], d["L"], d["seed"]
    ascii = oracle.gen_reads(seed, 0, n, L)
    words, rc, _ = oracle.encode_batch(ascii, n, L)
    assert rc == 0
    assert _sha(words) == d["words_sha256"]
    # known-answer: the generator's own words
    assert np.array_equal(words[:64], oracle.gen_words(seed, 0, 64, L))
    m = d["hamming_vs_read0_n"]
    ham = oracle.hamming_ref_batch(words[:m], m, L, words[0])
    assert _sha(ham) == d["hamming_vs_read0_sha256"]
    assert int(ham.sum()) == d["hamming_vs_read0_sum"]


def test_counter_digest(oracle, digests):
    d = digests["counter_1000000x32_pool65536"]
    n, L = d["n"], d["L"]
    ascii = oracle.gen_pool_reads(d["seed"], d["pool_seed"], d["U"], 0, n, L)
    reads = [ascii[i * L:(i + 1) * L].tobytes() for i in range(n)]
    got = oracle.count(reads)
    assert len(got) == d["unique"]
    ordered = np.array([(w[0], ln, c) for (w, ln, c, _f) in got], dtype=np.uint64)
    assert _sha(ordered) == d["ordered_sha256"]


@pytest.mark.skipif("not __import__('oracle').ref_available()")
def test_fuzz_against_reference_kernels(oracle):
    """Oracle == the reference's compiled kernels on random reads incl. aliased bytes < 0x80."""
    rng = np.random.default_rng(7)
    valid = np.frombuffer(b"ACGT", np.uint8)
    for L in list(range(1, 70)) + [95, 96, 97, 127, 128, 129, 200, 511, 512, 513, 1000, 1024]:
        n = 300
        a = valid[rng.integers(0, 4, size=n * L)]
        mask = rng.random(n * L) < 0.05
        a = np.where(mask, np.array(ALIASES, np.uint8)[rng.integers(0, 4, size=n * L)], a).astype(np.uint8)
        ref = oracle.ref_encode_batch(a, n, L)
        ora, rc, _ = oracle.encode_batch(a, n, L)
        assert rc == 0
        assert np.array_equal(ref, ora), L


def test_pool_counter_table_matches_reference_digest(oracle, digests):
    """The generator-derived counter (keys from the pool generator, counts = bincount of the draw
    indices, first = first draw; what tests/golden/c5_digests.json is built from) reproduces the
    reference ShortSeqCounter's own digest of the 1M x 32 pool-65536 list (dict order = first draw)."""
    d = digests["counter_1000000x32_pool65536"]
    k, c, f = oracle.pool_counter_table(d["seed"], d["pool_seed"], d["U"], d["n"], d["L"])
    assert len(k) == d["unique"] and int(c.max()) == d["max_count"]
    o = np.argsort(f, kind="stable")
    ordered = np.stack([k[o], np.full(len(k), d["L"], np.uint64), c[o]], 1).astype(np.uint64)
    assert _sha(ordered) == d["ordered_sha256"]


@pytest.mark.parametrize("s", [None, 1.1])
def test_pool_counter_table_matches_oracle_count(oracle, s):
    """Uniform and Zipf pools: the vectorised construction equals oracle.count over the same reads,
    at shard offsets, so the full-shard C5 digests (tests/test_c5_full.py) are pinned to the oracle."""
    U, n, i0 = 1 << 13, 300_000, 123_456_789
    cdf = None
    if s:
        w = np.arange(1, U + 1, dtype=np.float64) ** -s
        cc = np.cumsum(w) / w.sum()
        cdf = np.floor(cc * 2.0 ** 63).astype(np.uint64)
        cdf[-1] = np.uint64(1 << 63)
        a = oracle.gen_zipf_reads(5, 77, cdf, i0, n, 32)
        assert np.array_equal(oracle.pool_ids(77, i0, 64, U, cdf),
                              [oracle.lib().ora_zipf_index(77, i0 + j, cdf.ctypes.data, U) for j in range(64)])
    else:
        a = oracle.gen_pool_reads(5, 77, U, i0, n, 32)
    exp = oracle.count([a[i * 32:(i + 1) * 32].tobytes() for i in range(n)])
    k, c, f = oracle.pool_counter_table(5, 77, U, n, 32, i0=i0, cdf=cdf, chunk=1 << 16)
    ek = np.array([w[0] for (w, _l, _c, _f) in exp], np.uint64)
    ec = np.array([x[2] for x in exp], np.uint64)
    ef = np.array([x[3] for x in exp], np.uint64) + np.uint64(i0)
    assert oracle.table_digest(k, c, f) == oracle.table_digest(ek, ec, ef)


@pytest.mark.parametrize("L,i0", [(32, 0), (96, 0), (96, 77_777_777), (512, 0), (512, 49_990_000)])
def test_stream_digest_construction(oracle, L, i0):
    """The numpy construction behind tests/golden/stream_digests.json (generator words, distances to
    read 0) equals the oracle's encode / hamming of the generator's ASCII, at offsets into the batch."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "gen_stream_digests", os.path.join(os.path.dirname(__file__), "golden", "gen_stream_digests.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    n = 3000
    ascii = oracle.gen_reads(1, i0, n, L)
    words, rc, _ = oracle.encode_batch(ascii, n, L)
    assert rc == 0
    mine = g.gen_words(1, i0, n, L)
    assert np.array_equal(words, mine)
    ref = g.gen_words(1, 0, 1, L)[0]
    assert np.array_equal(g.hamming_ref(mine, ref), oracle.hamming_ref_batch(words, n, L, ref))
    if i0 == 0:   # the chunked digest of a prefix equals the SHA of the oracle's arrays
        ws, ds = g.digests(n, L, 1, chunk=700)
        assert ws == _sha(words)
        assert ds == _sha(oracle.hamming_ref_batch(words, n, L, words[0]))


def test_ragged_pool_rows_match_oracle_count():
    """The f2 ragged workload's generator-derived rows (oracle.ragged_pool_rows: items in first-draw
    order, equal contents merged) equal oracle.count over the generated reads (pins
    tests/golden/ragged_digests.json, tests/golden/gen_ragged_digests.py)."""
    import oracle
    for seed, ps, U, n, lo, hi in ((41, 42, 1 << 20, 20_000, 50, 150), (43, 44, 1 << 16, 30_000, 1, 300),
                                   (45, 46, 400, 5_000, 0, 6)):
        reads = oracle.ragged_pool_reads(seed, ps, U, 0, n, lo, hi)
        assert all(lo <= len(r) <= hi for r in reads)
        exp = oracle.count(reads)
        lens, counts, words = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
        got, w = [], 0
        for L, c in zip(lens.tolist(), counts.tolist()):
            nw = (L + 31) // 32
            ws = tuple(int(x) for x in words[w:w + nw]) or (0,)
            w += nw
            got.append((ws, L, c))
        assert got == [(ws, L, c) for ws, L, c, _f in exp], (seed, n)
        assert w == len(words)
