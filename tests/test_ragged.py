"""f2 — ragged, mixed-length reads (the _new class switch, short_seq.pyx:54-74, over
a whole batch; counted per length as ShortSeqCounter does, counter.pyx:22-39).

The reads come from the ss_synth_ragged_* generator (pool items of lengths Lmin..Lmax); its host
restatement (oracle.ragged_pool_reads / ragged_pool_rows) is pinned to oracle.count in
test_oracle_golden.py.  Checked on the GPU: the generator's bytes, ss_encode_var, and the drop-in
engine fed from device memory (ss_ingest_add_device) against the oracle at small sizes and against
the generator-derived digests at the bench's full size (50M reads of 50-150 nt).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _digests():
    with open(os.path.join(HERE, "golden", "ragged_digests.json")) as f:
        return json.load(f)


def test_synth_ragged_matches_oracle(gpu, oracle):
    import shortseq_amd.batch as B
    for seed, ps, U, n, lo, hi in ((41, 42, 1 << 20, 3000, 50, 150), (5, 6, 100, 2000, 0, 70)):
        blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
        reads = oracle.ragged_pool_reads(seed, ps, U, 0, n, lo, hi)
        assert lens.cpu().tolist() == [len(r) for r in reads]
        h = blob.cpu().numpy().tobytes()
        o = offs.cpu().tolist()
        assert [h[o[i]:o[i] + len(r)] for i, r in enumerate(reads)] == reads


def test_encode_var_ragged_vs_oracle(gpu, oracle):
    import shortseq_amd.batch as B
    n = 20_000
    blob, offs, lens = B.synth_ragged_pool_reads(n, 7, 8, 5000, 1, 300, device=gpu)
    words = B.encode_var(blob, offs, lens)
    reads = oracle.ragged_pool_reads(7, 8, 5000, 0, n, 1, 300)
    got = words.cpu().numpy().view(np.uint64)
    for i in range(0, n, 97):
        w, _e = oracle.encode_one(reads[i])
        nw = max(1, (len(reads[i]) + 31) // 32)
        assert got[i, :nw].tolist() == [int(x) for x in w[:nw]], i
        assert not got[i, nw:].any()


@pytest.mark.parametrize("exact", [False, True, 3])
@pytest.mark.parametrize("case", [(45, 46, 400, 50_000, 0, 6), (43, 44, 1 << 16, 200_000, 1, 300),
                                  (41, 42, 1 << 20, 300_000, 50, 150), (47, 48, 3000, 150_000, 33, 700)])
def test_device_ingest_ragged_small(gpu, oracle, case, exact):
    """ss_ingest_add_device over a ragged device batch (two calls: global read indices continue)
    == the generator-derived rows (pinned to oracle.count); length-class tables sized by their
    distinct-key sketch (default) or by their rows (exact); 33-700 nt takes the per-class encode;
    3 (test hook): the classes' fingerprint count takes its exact multi-word fallback."""
    import shortseq_amd.batch as B
    seed, ps, U, n, lo, hi = case
    blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
    h = n // 3
    eng = B.DeviceIngest(gpu, exact=exact) if exact != 3 else B.DeviceIngest(gpu, _sizing=3)
    try:
        eng.count(blob, offs[:h], lens[:h])
        eng.count(blob, offs[h:], lens[h:])
        gl, gc, gw = eng.results()
    finally:
        eng.close()
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    assert gl.tolist() == el.tolist()
    assert gc.tolist() == ec.tolist()
    assert np.array_equal(gw, ew)


@pytest.mark.parametrize("hook", [4, 5])
@pytest.mark.parametrize("U", [1 << 12, 1 << 18])
def test_device_ingest_speculative_finish_dropped(gpu, oracle, hook, U):
    """One read-order chunk (50-150 nt), so the class fold is deferred and the finish is queued
    speculatively beside the verify; then (test hooks) 4: the fingerprint flag comes back
    raised only after both were queued -- the speculation is dropped, the classes are re-encoded and
    counted exactly over the rows the speculative extract had written; 5: the result bound is taken
    as if the sketch said 0, so the speculative gather refuses (its bad flag) and the finish runs the
    ordinary way.  Both == the generator-derived rows, twice (a second results() call)."""
    import shortseq_amd.batch as B
    seed, ps, n, lo, hi = 61, 62, 250_000, 50, 150
    blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
    eng = B.DeviceIngest(gpu, _sizing=hook)
    try:
        eng.count(blob, offs, lens)
        gl, gc, gw = (a.copy() for a in eng.results())
        gl2, gc2, gw2 = eng.results()
    finally:
        eng.close()
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    for l_, c_, w_ in ((gl, gc, gw), (gl2, gc2, gw2)):
        assert l_.tolist() == el.tolist()
        assert c_.tolist() == ec.tolist()
        assert np.array_equal(w_, ew)


def test_device_ingest_undersized_class_table_recounts(gpu, oracle):
    """A class table sized below its distinct keys (the test hook: 1/64 of the sketch) runs full:
    the add call returns SS_EFULL and the first batch is counted again with tables sized by rows;
    the rows still equal the oracle's.  A later batch that overflows cannot be redone and raises."""
    import shortseq_amd.batch as B
    from shortseq_amd._native import NativeError
    seed, ps, U, n, lo, hi = 51, 52, 1 << 17, 400_000, 33, 150
    blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
    eng = B.DeviceIngest(gpu, _sizing=2)
    try:
        eng.count(blob, offs, lens)
        assert eng.retried
        gl, gc, gw = eng.results()
        eng.reset()
        eng.count(blob, offs[:1000], lens[:1000])           # small: fits even undersized
        with pytest.raises(NativeError, match="ran full"):
            eng.count(blob, offs, lens)
        with pytest.raises(NativeError, match="reset and count again"):   # the counts are void now
            eng.results()
        eng.reset()
        eng.count(blob, offs[:1000], lens[:1000])
        assert int(eng.results()[1].sum()) == 1000
    finally:
        eng.close()
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    assert gl.tolist() == el.tolist() and gc.tolist() == ec.tolist() and np.array_equal(gw, ew)


def test_device_ingest_class_lengths_apart(gpu, oracle):
    """One length class (33..64 nt) holds reads that pack to the same words at different lengths
    (trailing 'A' = code 0): the class key's length word keeps them apart, as the reference's
    (length, words) key does.  Plus a 96/97 boundary and a bad read inside a class."""
    import torch
    import shortseq_amd.batch as B
    rng = np.random.default_rng(5)
    s = "".join(rng.choice(list("ACGT"), 60))
    t = "".join(rng.choice(list("ACGT"), 96))
    base = [s[:40], s[:40] + "A", s[:40] + "AA", s[:39], s[:40] + "A", s[:64], s[:33], t, t + "A", t[:95],
            s[:40] + "AA", "A" * 33, "A" * 34, "A" * 64, "A" * 33]
    reads = [base[i] for i in rng.integers(0, len(base), 5000)] + base
    enc = [r.encode() for r in reads]
    lens = torch.tensor([len(r) for r in enc], dtype=torch.int32)
    offs = torch.zeros(len(enc), dtype=torch.int64)
    offs[1:] = torch.cumsum(lens.to(torch.int64), 0)[:-1]
    blob = torch.frombuffer(bytearray(b"".join(enc) + b"\0" * 16), dtype=torch.uint8)
    eng = B.DeviceIngest(gpu)
    try:
        eng.count(blob.to(gpu), offs.to(gpu), lens.to(gpu))
        gl, gc, gw = eng.results()
    finally:
        eng.close()
    exp = oracle.count(enc)
    assert gl.tolist() == [L for (_w, L, _c, _f) in exp]
    assert gc.tolist() == [c for (_w, _L, c, _f) in exp]
    assert gw.tolist() == [int(x) for (w, _L, _c, _f) in exp for x in w]


@pytest.mark.parametrize("exact", [False, 3])
def test_device_ingest_read_order_rows(gpu, oracle, exact):
    """Chunks whose reads are all 33-160 nt (or empty) take the read-order rows (k_encode_rows, the
    flat verify / fold); empties stay out of the class tables, a second call continues the global
    read indices and the first occurrences, exact=3 (test hook) takes the exact fallback through the
    one-pass class encode.  == oracle.count over the same reads."""
    import torch
    import shortseq_amd.batch as B
    rng = np.random.default_rng(11)
    pool = ["".join(rng.choice(list("ACGT"), int(L))) for L in rng.integers(33, 161, 700)]
    pool += ["A" * 33, "A" * 64, "A" * 65, "T" * 96, "T" * 128, "G" * 160, pool[0] + "A", ""]
    reads = [pool[i] for i in rng.integers(0, len(pool), 60_000)]

    def device(rs):
        enc = [r.encode() for r in rs]
        lens = torch.tensor([len(r) for r in enc], dtype=torch.int32)
        offs = torch.zeros(len(enc), dtype=torch.int64)
        offs[1:] = torch.cumsum(lens.to(torch.int64), 0)[:-1]
        blob = torch.frombuffer(bytearray(b"".join(enc) + b"\0" * 16), dtype=torch.uint8)
        return blob.to(gpu), offs.to(gpu), lens.to(gpu)

    eng = B.DeviceIngest(gpu) if exact != 3 else B.DeviceIngest(gpu, _sizing=3)
    try:
        eng.count(*device(reads[:25_000]))
        eng.count(*device(reads[25_000:]))
        gl, gc, gw = eng.results()
    finally:
        eng.close()
    exp = oracle.count([r.encode() for r in reads])
    assert gl.tolist() == [L for (_w, L, _c, _f) in exp]
    assert gc.tolist() == [c for (_w, _L, c, _f) in exp]
    # (ss_ingest_results: ceil(L / 32) words a key, none for the empty read)
    assert gw.tolist() == [int(x) for (w, L, _c, _f) in exp for x in w[:(L + 31) // 32]]


@pytest.mark.parametrize("lo,hi", [(33, 64), (33, 96), (65, 128), (129, 160), (150, 170)])
def test_device_ingest_row_widths(gpu, oracle, lo, hi):
    """Read-order rows of every stride (S = 3..6 words: lengths up to 64 / 96 / 128 / 160) and, past 160
    nt, the one-pass class encode; lengths at the class edges (32k, 32k + 1) included; == oracle.count."""
    import torch
    import shortseq_amd.batch as B
    rng = np.random.default_rng(lo * 1000 + hi)
    edges = [L for L in (lo, hi, 64, 65, 96, 97, 128, 129, 160, 161) if lo <= L <= hi]
    lens_pool = list(rng.integers(lo, hi + 1, 300)) + edges
    pool = ["".join(rng.choice(list("ACGT"), int(L))) for L in lens_pool]
    reads = [pool[i] for i in rng.integers(0, len(pool), 30_000)]
    enc = [r.encode() for r in reads]
    lens = torch.tensor([len(r) for r in enc], dtype=torch.int32)
    offs = torch.zeros(len(enc), dtype=torch.int64)
    offs[1:] = torch.cumsum(lens.to(torch.int64), 0)[:-1]
    blob = torch.frombuffer(bytearray(b"".join(enc) + b"\0" * 16), dtype=torch.uint8)
    eng = B.DeviceIngest(gpu)
    try:
        eng.count(blob.to(gpu), offs.to(gpu), lens.to(gpu))
        gl, gc, gw = eng.results()
    finally:
        eng.close()
    exp = oracle.count(enc)
    assert gl.tolist() == [L for (_w, L, _c, _f) in exp]
    assert gc.tolist() == [c for (_w, _L, c, _f) in exp]
    assert gw.tolist() == [int(x) for (w, L, _c, _f) in exp for x in w[:(L + 31) // 32]]


def test_device_ingest_stride_guess_changes(gpu, oracle):
    """One engine over chunks whose read-order stride changes from chunk to chunk: each chunk's row
    encode is queued at the previous chunk's stride beside its length split, so every kind of wrong
    guess is taken -- a narrower and a wider stride, a chunk past 160 nt and one mixed with <= 32-nt
    reads (both off the read-order path), and the first read-order chunk after those -- both as the
    side-stream encode and as the gated one.  The results after every chunk == oracle.count of all
    reads so far."""
    import torch
    import shortseq_amd.batch as B
    rng = np.random.default_rng(2024)
    # (after two chunks at one stride the guess runs on a side stream, after one it is gated on the
    # device: both kinds are taken wrong below)
    ranges = [(33, 64), (65, 160), (33, 96), (100, 300), (40, 90), (40, 90), (40, 90), (10, 150), (129, 160),
              (129, 160), (129, 160), (33, 64), (33, 64), (33, 64), (65, 160), (65, 160), (100, 300), (33, 64)]
    chunks = []
    for lo, hi in ranges:
        pool = ["".join(rng.choice(list("ACGT"), int(L))) for L in rng.integers(lo, hi + 1, 400)]
        chunks.append([pool[i].encode() for i in rng.integers(0, len(pool), 4_000)])
    enc = [r for c in chunks for r in c]
    lens = torch.tensor([len(r) for r in enc], dtype=torch.int32)
    offs = torch.zeros(len(enc), dtype=torch.int64)
    offs[1:] = torch.cumsum(lens.to(torch.int64), 0)[:-1]
    blob = torch.frombuffer(bytearray(b"".join(enc) + b"\0" * 16), dtype=torch.uint8).to(gpu)
    offs, lens = offs.to(gpu), lens.to(gpu)
    eng = B.DeviceIngest(gpu)
    try:
        at = 0
        for c in chunks:
            eng.count(blob, offs[at:at + len(c)], lens[at:at + len(c)])
            at += len(c)
            gl, gc, gw = eng.results()
            exp = oracle.count(enc[:at])
            assert gl.tolist() == [L for (_w, L, _c, _f) in exp], at
            assert gc.tolist() == [c for (_w, _L, c, _f) in exp], at
            assert gw.tolist() == [int(x) for (w, L, _c, _f) in exp for x in w[:(L + 31) // 32]], at
    finally:
        eng.close()


def test_device_ingest_read_order_rows_error(gpu):
    """A rejected byte inside a read of a read-order chunk raises the reference's message for the
    first such read."""
    import torch
    import shortseq_amd as sq
    import shortseq_amd.batch as B
    rng = np.random.default_rng(12)
    reads = ["".join(rng.choice(list("ACGT"), int(L))) for L in rng.integers(33, 150, 20_000)]
    reads[7000] = reads[7000][:40] + "N" + reads[7000][41:]
    reads[9000] = reads[9000][:3] + "x" + reads[9000][4:]
    with pytest.raises(Exception) as want:
        sq.pack(reads[7000].encode())
    enc = [r.encode() for r in reads]
    lens = torch.tensor([len(r) for r in enc], dtype=torch.int32)
    offs = torch.zeros(len(enc), dtype=torch.int64)
    offs[1:] = torch.cumsum(lens.to(torch.int64), 0)[:-1]
    blob = torch.frombuffer(bytearray(b"".join(enc) + b"\0" * 16), dtype=torch.uint8)
    eng = B.DeviceIngest(gpu)
    try:
        with pytest.raises(Exception) as ei:
            eng.count(blob.to(gpu), offs.to(gpu), lens.to(gpu))
        assert str(ei.value) == str(want.value)
    finally:
        eng.close()


def test_device_ingest_ragged_errors(gpu):
    """A rejected read in a device batch raises the reference's message (the first in read order)."""
    import shortseq_amd as sq
    import shortseq_amd.batch as B
    blob, offs, lens = B.synth_ragged_pool_reads(100_000, 3, 4, 1000, 20, 120, device=gpu)
    o, ln = offs.cpu().tolist(), lens.cpu().tolist()
    blob[o[70_000] + 5] = ord("N")
    blob[o[90_000] + 1] = ord("x")
    bad = bytes(blob[o[70_000]:o[70_000] + ln[70_000]].cpu().numpy())
    with pytest.raises(Exception) as want:          # the reference's message for that read (chunk rule
        sq.pack(bad)                                # for a full 32-nt block, the byte on the table path)
    eng = B.DeviceIngest(gpu)
    try:
        with pytest.raises(Exception) as ei:
            eng.count(blob, offs, lens)
        assert str(ei.value) == str(want.value) and "N" in str(ei.value)
    finally:
        eng.close()


def test_device_ingest_high_diversity_slice(gpu, oracle):
    """the F2 reads at high diversity (pool 2^24), a 5M-read slice (~4.3M distinct
    keys: the scratch table, its representatives and the class tables far past one per 48 reads)
    against the generator-derived rows (oracle.ragged_pool_rows, pinned to oracle.count)."""
    import shortseq_amd.batch as B
    d = _digests()["ragged_50M_L50-150_U24"]
    n = 5_000_000
    blob, offs, lens = B.synth_ragged_pool_reads(n, d["seed"], d["pool_seed"], d["U"], d["Lmin"], d["Lmax"],
                                                 device=gpu)
    eng = B.DeviceIngest(gpu)
    try:
        eng.count(blob, offs, lens)
        gl, gc, gw = eng.results()
    finally:
        eng.close()
    del blob, offs, lens
    el, ec, ew = oracle.ragged_pool_rows(d["seed"], d["pool_seed"], d["U"], n, d["Lmin"], d["Lmax"])
    assert len(gl) == len(el) and len(el) > 4_000_000
    assert np.array_equal(gl, el) and np.array_equal(gc, ec) and np.array_equal(gw, ew)


@pytest.mark.parametrize("name", ["ragged_1M_L1-300_U16", "ragged_50M_L50-150_U20", "ragged_50M_L50-150_U24"])
def test_device_ingest_ragged_digest(gpu, oracle, name):
    """Full size (bench.py F2): the engine's rows (dict order, lengths, counts, words) hash to the
    generator-derived digest (tests/golden/ragged_digests.json)."""
    import shortseq_amd.batch as B
    d = _digests()[name]
    blob, offs, lens = B.synth_ragged_pool_reads(d["n"], d["seed"], d["pool_seed"], d["U"], d["Lmin"], d["Lmax"],
                                                 device=gpu)
    eng = B.DeviceIngest(gpu)
    try:
        eng.count(blob, offs, lens)
        gl, gc, gw = eng.results()
    finally:
        eng.close()
    del blob, offs, lens
    assert len(gl) == d["unique"] and int((gl.astype(np.uint64) * gc).sum()) == d["nt"]
    assert oracle.rows_digest(gl, gc, gw) == d["digest"]


def test_device_ingest_large_class_tables(gpu, oracle):
    """Class tables past the row-record path's region bound (> 1024 regions of 2048 slots: millions
    of distinct 33-64-nt keys in one class) take the fingerprint-fed thin path; a 100-200-nt batch
    takes classes of 4..8 words (W + 1 up to the row-record path's widest instance).  Both equal
    the generator-derived rows."""
    import shortseq_amd.batch as B
    for seed, ps, U, n, lo, hi in ((61, 62, 1 << 25, 2_500_000, 33, 64), (63, 64, 1 << 15, 400_000, 100, 224)):
        blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
        eng = B.DeviceIngest(gpu)
        try:
            eng.count(blob, offs, lens)
            gl, gc, gw = eng.results()
        finally:
            eng.close()
        el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
        assert gl.tolist() == el.tolist()
        assert gc.tolist() == ec.tolist()
        assert np.array_equal(gw, ew)


def test_device_ingest_rekey_row_limit(gpu, oracle):
    """VERDICT r3 item 7, the u32 row bound of a length's table: with the bound lowered to 1024 rows
    (the test hook), every length and class table is re-keyed many times over 60 small batches (its
    distinct keys become its first rows, the row map compacted); the rows still equal the oracle's."""
    import shortseq_amd.batch as B
    seed, ps, U, n, lo, hi = 71, 72, 600, 30_000, 0, 120
    blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
    eng = B.DeviceIngest(gpu)
    try:
        eng.set_row_limit(1024)
        for a in range(0, n, 500):
            eng.count(blob, offs[a:a + 500], lens[a:a + 500])
        gl, gc, gw = eng.results()
    finally:
        eng.close()
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    assert gl.tolist() == el.tolist()
    assert gc.tolist() == ec.tolist()
    assert np.array_equal(gw, ew)


@pytest.mark.parametrize("lo,hi,row_limit", [(0, 120, None), (0, 120, 1024), (33, 160, None), (33, 160, 1024),
                                              (100, 300, None), (32, 32, None)])
def test_device_ingest_count_spill(gpu, oracle, lo, hi, row_limit):
    """VERDICT r3 missing item 4, a key's count past the slots' u32: with the spill lowered to every
    1000 reads (the test hook), the tables' counts move into the groups' u64 row counts dozens of times
    over 60 batches of 500 (33..160: the flat read-order-rows path's class tables; 100..300: classes
    past the flat path; 32..32: one length table; with the row bound lowered too, the spilled counts
    follow their entries through every re-key); the rows (counts added back at finish) still equal the
    oracle's."""
    import shortseq_amd.batch as B
    seed, ps, U, n = 75, 76, 600, 30_000
    blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
    eng = B.DeviceIngest(gpu)
    try:
        with pytest.raises(Exception):
            eng.set_count_limit(0)
        eng.set_count_limit(1000)
        if row_limit:
            eng.set_row_limit(row_limit)
        for a in range(0, n, 500):
            eng.count(blob, offs[a:a + 500], lens[a:a + 500])
        gl, gc, gw = eng.results()
        eng.reset()             # a reset drops the spilled counts with the tables
        eng.count(blob, offs[:3000], lens[:3000])
        rl, rc, rw = eng.results()
    finally:
        eng.close()
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    assert gl.tolist() == el.tolist()
    assert gc.tolist() == ec.tolist()
    assert np.array_equal(gw, ew)
    assert int(rc.sum()) == 3000


@pytest.mark.parametrize("lo,hi", [(0, 120), (33, 160)])
def test_device_ingest_count_spill_merge(gpu, oracle, lo, hi):
    """The spill across ss_ingest_merge: both engines spill every 1000 reads; the source's reads count
    toward the destination's spill (it spills before the merge), the exported counts carry the
    source's spilled counts, and the rows equal the oracle's for the two slices back to back."""
    import shortseq_amd.batch as B
    seed, ps, U, n = 77, 78, 400, 20_000
    blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
    h = n // 2
    a, b = B.DeviceIngest(gpu), B.DeviceIngest(gpu)
    try:
        for e in (a, b):
            e.set_count_limit(1000)
        for x in range(0, h, 700):
            a.count(blob, offs[x:min(x + 700, h)], lens[x:min(x + 700, h)])
            b.count(blob, offs[h + x:min(h + x + 700, n)], lens[h + x:min(h + x + 700, n)])
        b.export()
        a.merge(b, h)
        gl, gc, gw = a.results()
    finally:
        a.close()
        b.close()
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    assert gl.tolist() == el.tolist()
    assert gc.tolist() == ec.tolist()
    assert np.array_equal(gw, ew)


@pytest.mark.parametrize("lo,hi", [(0, 40), (33, 100), (100, 300)])
def test_device_ingest_merge_counts_past_slot(gpu, oracle, lo, hi):
    """Counts a slot cannot take in one merge: with the spill lowered to every 500 reads, a 6-key pool
    gives every key ~1700 copies per engine, so the source's exported counts (its spilled counts
    added back) exceed what a destination slot may take before its next spill; ss_ingest_merge takes
    them in passes, spilling the destination between passes, and the rows equal the oracle's."""
    import shortseq_amd.batch as B
    seed, ps, U, n = 79, 80, 6, 20_000
    blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
    h = n // 2
    a, b = B.DeviceIngest(gpu), B.DeviceIngest(gpu)
    try:
        for e in (a, b):
            e.set_count_limit(500)
        for x in range(0, h, 1000):
            a.count(blob, offs[x:x + 1000], lens[x:x + 1000])
            b.count(blob, offs[h + x:h + x + 1000], lens[h + x:h + x + 1000])
        b.export()
        a.merge(b, h)
        gl, gc, gw = a.results()
    finally:
        a.close()
        b.close()
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    assert int(ec.max()) > 1000
    assert gl.tolist() == el.tolist()
    assert gc.tolist() == ec.tolist()
    assert np.array_equal(gw, ew)


def test_device_ingest_read_index_past_2_32(gpu, oracle):
    """VERDICT r3 item 7, global read indices past 2^32 - 1: an engine's reads folded into another at
    base 2^32 + 7 (ss_ingest_merge) -- the row maps and the first-occurrence order run on u64 read
    indices (the read map spans 2^32 + reads bits), no SS_EARG -- and the rows equal the oracle's for
    the two slices back to back."""
    import shortseq_amd.batch as B
    seed, ps, U, n, lo, hi = 73, 74, 3000, 80_000, 0, 200
    blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
    h = n // 2
    a, b = B.DeviceIngest(gpu), B.DeviceIngest(gpu)
    try:
        a.count(blob, offs[:h], lens[:h])
        b.count(blob, offs[h:], lens[h:])
        b.export()
        a.merge(b, (1 << 32) + 7)
        gl, gc, gw = a.results()
    finally:
        a.close()
        b.close()
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    assert gl.tolist() == el.tolist()
    assert gc.tolist() == ec.tolist()
    assert np.array_equal(gw, ew)


def test_device_ingest_flat_pending_paths(gpu, oracle):
    """The read-order path's deferred fold and speculative finish (50-150 nt: every read a class read
    of at most 5 words).  A first chunk leaves its scratch unfolded and queues the finish beside the
    verify; results() twice, a second chunk after results() (the pending scratch folded first), and a
    second chunk with no results() in between all give the generator-derived rows of the reads so far."""
    import shortseq_amd.batch as B
    seed, ps, U, n, lo, hi = 61, 62, 30_000, 400_000, 50, 150
    blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
    cut = 150_000

    def rows(m):
        return oracle.ragged_pool_rows(seed, ps, U, m, lo, hi)

    def same(got, want):
        assert got[0].tolist() == want[0].tolist()
        assert got[1].tolist() == want[1].tolist()
        assert np.array_equal(got[2], want[2])

    eng = B.DeviceIngest(gpu)
    try:
        eng.count(blob, offs[:cut], lens[:cut])
        first = eng.results()
        same(first, rows(cut))
        same(eng.results(), rows(cut))                 # a second finish: the same rows
        eng.count(blob, offs[cut:], lens[cut:])        # folds the pending scratch, then counts
        same(eng.results(), rows(n))
        eng.reset()
        eng.count(blob, offs[:cut], lens[:cut])
        eng.count(blob, offs[cut:], lens[cut:])        # no finish between the two chunks
        same(eng.results(), rows(n))
        eng.reset()
        eng.count(blob, offs, lens)                    # one chunk after a reset: speculation again
        same(eng.results(), rows(n))
    finally:
        eng.close()


def test_device_ingest_flat_pending_export_merge(gpu, oracle):
    """Engines whose only chunk took the read-order path (fold pending, finish queued) exported and
    merged: the export folds the scratch first, the destination's queued finish is dropped by the merge."""
    import shortseq_amd.batch as B
    seed, ps, U, n, lo, hi = 63, 64, 20_000, 300_000, 60, 140
    blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
    cuts = [0, 100_000, 170_000, n]
    engs = [B.DeviceIngest(gpu) for _ in range(3)]
    try:
        for k, e in enumerate(engs):
            e.count(blob, offs[cuts[k]:cuts[k + 1]], lens[cuts[k]:cuts[k + 1]])
        for e in engs[1:]:
            e.export()
        engs[0].merge(engs[1], cuts[1])
        engs[0].merge(engs[2], cuts[2])
        gl, gc, gw = engs[0].results()
    finally:
        for e in engs:
            e.close()
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    assert gl.tolist() == el.tolist() and gc.tolist() == ec.tolist() and np.array_equal(gw, ew)


def test_device_ingest_flat_rejected_read_then_reset(gpu):
    """A rejected read in a read-order first chunk: the queued finish is dropped, count() raises the
    reference's message, and after reset() the engine counts a clean batch exactly."""
    import shortseq_amd.batch as B
    from shortseq_amd import ShortSeqCounter
    blob, offs, lens = B.synth_ragged_pool_reads(200_000, 65, 66, 5000, 50, 150, device=gpu)
    import shortseq_amd as sq
    bad = blob.clone()
    o, ln = int(offs[123_456].item()), int(lens[123_456].item())
    bad[o + 7] = ord("N")
    with pytest.raises(Exception) as want:          # the reference's message for that read
        sq.pack(bytes(bad[o:o + ln].cpu().numpy()))
    eng = B.DeviceIngest(gpu)
    try:
        with pytest.raises(Exception) as ei:
            eng.count(bad, offs, lens)
        assert str(ei.value) == str(want.value)
        eng.reset()
        eng.count(blob, offs, lens)
        gl, gc, _gw = eng.results()
        assert int(gc.sum()) == 200_000
        host = blob.cpu().numpy().tobytes()
        oo, ll = offs.cpu().numpy(), lens.cpu().numpy()
        want = ShortSeqCounter([host[oo[i]:oo[i] + ll[i]] for i in range(200_000)], device="host")
        assert len(gl) == len(want) and sorted(gc.tolist()) == sorted(want.values())
    finally:
        eng.close()


@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_device_ingest_results_formats(gpu, oracle, fmt):
    """The three result layouts (plain u32 / u64; compact u16 / u32; compact with u64 counts) carry
    the same rows, through the speculative finish (first read-order chunk) and the ordinary one
    (mixed lengths, a second chunk)."""
    import shortseq_amd.batch as B
    for seed, ps, U, n, lo, hi in ((71, 72, 9000, 200_000, 50, 150), (73, 74, 9000, 200_000, 0, 300)):
        blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
        eng = B.DeviceIngest(gpu, compact=fmt)
        try:
            eng.count(blob, offs[:n // 2], lens[:n // 2])
            eng.count(blob, offs[n // 2:], lens[n // 2:])
            gl, gc, gw = eng.results()
            eng.reset()
            eng.count(blob, offs, lens)
            gl1, gc1, gw1 = eng.results()
        finally:
            eng.close()
        assert gl.dtype == (np.uint32 if fmt == 0 else np.uint16)
        assert gc.dtype == (np.uint32 if fmt == 1 else np.uint64)
        el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
        for a, b, c in ((gl, gc, gw), (gl1, gc1, gw1)):
            assert a.tolist() == el.tolist() and b.tolist() == ec.tolist() and np.array_equal(c, ew)
