"""The drop-in Python API (shortseq_amd) against the reference's behaviour.

Two sources of truth: (1) the golden fixtures captured from the reference (tests/golden), checked
exactly (class, packed words, str, len, hash, getsizeof, ^, error type + message, counter order);
(2) the behaviours the reference's own unit tests assert (shortseq/tests/unit_tests_main.py — empty
singleton :21-30, single bases :34-49, class switch :54-59, invalid chars :63-69 and :504-515, sizes
:73-86 and :495-500, round trip every length :91-118 and :275-287, subscripts :122-155 and :291-306,
hamming every length :159-166 and :456-463, slices :170-240 and :310-452, README :465-491),
restated here with a seeded RNG.  Host path only (CPU); the GPU counter path is in test_gpu_*.
"""
import os
import random
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

import shortseq_amd as sq
from shortseq_amd import (MAX_64_NT, MAX_192_NT, MAX_VAR_NT, MIN_64_NT, MIN_192_NT, MIN_VAR_NT,
                          ShortSeq64, ShortSeq192, ShortSeqCounter, ShortSeqVar)

RNG = random.Random(1234)


def rand_seq(n):
    return "".join(RNG.choice("ACTG") for _ in range(n))


def str_ham(a, b):
    return sum(x != y for x, y in zip(a, b))


# ---------------------------------------------------------------- golden (reference-captured) ----
def test_golden_vectors(golden):
    for v in golden["vectors"]:
        for ctor in (lambda s: sq.pack(s), lambda s: sq.pack(s.encode()),
                     lambda s: sq.from_str(s), lambda s: sq.from_bytes(s.encode())):
            a = ctor(v["a"])
            assert type(a).__name__ == v["class"]
            assert len(a) == v["length"]
            assert list(a.packed) == [int(h, 16) for h in v["words_a"]][:len(a.packed)]
            assert str(a) == v["str_a"]
            assert sys.getsizeof(a) == v["sizeof"]
            assert hash(a) == v["hash_a"]
            assert a ^ sq.pack(v["b"]) == v["hamming"]
            assert a == v["a"]


def test_golden_aliased(golden):
    for c in golden["aliased"]:
        seq = bytes.fromhex(c["input_hex"])
        a = sq.pack(seq)
        assert type(a).__name__ == c["class"]
        assert list(a.packed) == [int(h, 16) for h in c["words"]][:len(a.packed)], (c["L"], c["pos"])


def test_golden_errors(golden):
    for c in golden["errors"]["pack"]:
        ctor = c["ctor"]
        if ctor == "pack_str":
            call = lambda: sq.pack(c["input"])  # noqa: E731
        elif ctor == "pack_bytes":
            call = lambda: sq.pack(c["input"].encode())  # noqa: E731
        elif ctor == "pack_bytes_hex":
            call = lambda: sq.pack(bytes.fromhex(c["input"]))  # noqa: E731
        elif ctor == "from_bytes":
            call = lambda: sq.from_bytes(c["input"].encode())  # noqa: E731
        elif ctor == "from_str":
            call = lambda: sq.from_str(c["input"])  # noqa: E731
        else:
            call = lambda: sq.pack(eval(c["input"]))  # noqa: E731,S307 — fixture repr of a builtin
        if "raises" not in c:
            r = call()
            assert type(r).__name__ == c["class"] and len(r) == c["length"]
            continue
        with pytest.raises(BaseException) as ei:
            call()
        assert type(ei.value).__name__ == c["raises"]
        assert str(ei.value) == c["message"], ctor
    for h in golden["errors"]["hamming"]:
        a, b = sq.pack(h["a"]), sq.pack(h["b"])
        with pytest.raises(BaseException) as ei:
            a ^ b
        assert type(ei.value).__name__ == h["raises"]
        if h["raises"] == "Exception":
            assert str(ei.value) == h["message"]


def test_golden_counter_host(golden):
    for case in golden["counter"]:
        if "reads_str" in case:
            with pytest.raises(TypeError) as ei:
                ShortSeqCounter(case["reads_str"])
            assert str(ei.value) == case["message"]
            continue
        reads = [bytes.fromhex(h) for h in case["reads_hex"]]
        if "raises" in case:
            with pytest.raises(Exception) as ei:
                ShortSeqCounter(reads, device="host")
            assert str(ei.value) == case["message"]
            continue
        c = ShortSeqCounter(reads, device="host")
        got = [(type(k).__name__, str(k), len(k), v) for k, v in c.items()]
        exp = [(it["class"], it["str"], it["length"], it["count"]) for it in case["items"]]
        assert got == exp


# ------------------------------------------------------ behaviours of the reference's unit tests ----
def test_empty_singleton():
    a, b = sq.pack(""), sq.pack(b"")
    assert a == b and a is b and str(a) == "" and a == "" and len(a) == 0
    assert sq.from_str("") is a and sq.from_bytes(b"") is a


def test_single_bases():
    for b in "ATGC":
        for s in (sq.from_str(b), sq.from_bytes(b.encode())):
            assert s == b and str(s) == b and type(s) is ShortSeq64


def test_class_switch():
    assert type(sq.pack("A" * MAX_64_NT)) is ShortSeq64
    assert type(sq.pack("A" * (MAX_64_NT + 1))) is ShortSeq192
    assert type(sq.pack("A" * MAX_192_NT)) is ShortSeq192
    assert type(sq.pack("A" * MIN_VAR_NT)) is ShortSeqVar
    assert (MIN_64_NT, MAX_64_NT, MIN_192_NT, MAX_192_NT, MIN_VAR_NT, MAX_VAR_NT) == (0, 32, 33, 96, 97, 1024)


def test_invalid_chars():
    for p in ["N", "*", "N" * 33, "*" * 33]:
        with pytest.raises(Exception, match="Unsupported base character"):
            sq.pack(p)
    for L in range(MIN_VAR_NT, MAX_VAR_NT, 37):
        for p in "N*":
            with pytest.raises(Exception, match="Unsupported base character: "):
                sq.pack(rand_seq(L - 1) + p)


def test_sizes():
    assert sys.getsizeof(sq.pack(rand_seq(MIN_64_NT))) == 32
    assert sys.getsizeof(sq.pack(rand_seq(MAX_64_NT))) == 32
    assert sys.getsizeof(sq.pack(rand_seq(MIN_192_NT))) == 48
    assert sys.getsizeof(sq.pack(rand_seq(MAX_192_NT))) == 48
    assert sys.getsizeof(sq.pack(rand_seq(MIN_VAR_NT))) == 64
    assert sys.getsizeof(sq.pack(rand_seq(MAX_VAR_NT))) == 288


def test_round_trip_every_length():
    for L in range(0, MAX_VAR_NT + 1):
        s = rand_seq(L)
        o = sq.pack(s)
        assert len(o) == L and str(o) == s
    with pytest.raises(Exception, match=r"longer than 1024 bases"):
        sq.pack("ATGC" * 256 + "A")


def test_subscript():
    for L in list(range(1, 100)) + [200, 513, 1024]:
        s = rand_seq(L)
        o = sq.pack(s)
        for i in range(L):
            assert o[i] == s[i] and o[-i] == s[-i]
        for oob in (L, L + 1, -L - 1):
            with pytest.raises(IndexError):
                o[oob]
    with pytest.raises(TypeError):
        sq.pack("ACGT")["x"]


def test_hamming_every_length():
    for L in range(0, MAX_VAR_NT):
        a, b = rand_seq(L), rand_seq(L)
        assert sq.pack(a) ^ sq.pack(b) == str_ham(a, b)


def test_slices():
    for L in (MAX_64_NT, MAX_192_NT, MIN_VAR_NT, MAX_VAR_NT):
        s = rand_seq(L)
        o = sq.pack(s)
        assert str(o[:]) == s
        ids = set()
        for i in range(L):
            assert str(o[:i]) == s[:i] and str(o[:-i]) == s[:-i]
            assert str(o[i:]) == s[i:] and str(o[-i:]) == s[-i:]
            ids.add(id(o[i:i]))
        assert len(ids) == 1
    s = rand_seq(MAX_VAR_NT)
    o = sq.pack(s)
    for _ in range(3000):
        a = RNG.randint(0, MAX_VAR_NT // 2)
        b = RNG.randint(a, a + RNG.randint(1, MAX_VAR_NT - a))
        sl = o[a:b]
        assert str(sl) == s[a:b]
        n = len(s[a:b])
        assert type(sl) is (ShortSeq64 if n <= 32 else ShortSeq192 if n <= 96 else ShortSeqVar)
    with pytest.raises(TypeError):
        o[::2]


def test_slice_hamming():
    comp = {"A": "T", "T": "A", "G": "C", "C": "G"}
    a = rand_seq(MAX_VAR_NT)
    b = comp[a[0]] + a[1:-1] + comp[a[-1]]
    A, Bq = sq.pack(a), sq.pack(b)
    assert A ^ Bq == 2 and A[1:] ^ Bq[1:] == 1 and A[:-1] ^ Bq[:-1] == 1 and A[1:-1] ^ Bq[1:-1] == 0
    bc = "".join(comp[x] for x in a)
    Bc = sq.pack(bc)
    for cls, (slc, d) in {ShortSeqVar: (slice(1, -1), MAX_VAR_NT - 2),
                          ShortSeq192: (slice(1, MAX_192_NT - 1), MAX_192_NT - 2),
                          ShortSeq64: (slice(1, MAX_64_NT - 1), MAX_64_NT - 2)}.items():
        assert type(A[slc]) is cls and A[slc] ^ Bc[slc] == d


def test_readme():
    s1, s2 = sq.pack("ATGC"), sq.pack(b"ATGC")
    assert s1 == s2 == "ATGC" and len(s1) == len(s2) == 4
    s3 = sq.pack("TATTAGCGATTGACAGTTGTCCTGTAATAACGCCGGGTAAATTTGCCG")
    s4 = sq.pack("TATTACCGATTGACAGTTGTCCTGTAATAACGGCGGGTAAATTTGCTG")
    st = str(s4)
    assert s4[5:15] == st[5:15] and s4[-2] == st[-2]
    assert s3 ^ s4 == sum(a != b for a, b in zip(s3, s4)) == 3
    assert ShortSeqCounter([b"ATGC"] * 10) == {sq.pack("ATGC"): 10}


def test_counter_api():
    c = ShortSeqCounter()
    assert c == {}
    with pytest.raises(TypeError):
        c["ACGT"] = 1
    c[sq.pack("ACGT")] = 3
    assert c[sq.pack("ACGT")] == 3
    assert ShortSeqCounter((b"A", b"A")) == {}            # only lists are consumed (counter.pyx:14)
    big = ShortSeqCounter([b"G" * 32] * 3, device="host")
    assert big[sq.pack("G" * 32)] == 3                    # consistent hash (documented deviation Q5)
    v = ShortSeqCounter([b"A" * 200] * 3, device="host")
    assert list(v.values()) == [3]                        # content dedup for Var (deviation Q6)


def test_read_and_count_fastq(tmp_path, capsys):
    recs = []
    for i, s in enumerate(["ACGT", "ACGT", "GGGGA", "T" * 40, "ACGT"]):
        recs.append(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n")
    p = tmp_path / "x.fq"
    p.write_text("".join(recs) + "@last\nACGTA")           # last line has no newline: loses a base
    c = sq.read_and_count_fastq(str(p), device="host")
    assert [(str(k), v) for k, v in c.items()] == [("ACGT", 4), ("GGGGA", 1), ("T" * 40, 1)]
    assert "total seqs" in capsys.readouterr().out


def test_fill_rows_order_and_empty():
    """The GPU paths' dict rebuild (host side) from the engine's rows (ss_ingest_results layout):
    keys of several lengths and the empty read, in the given (first-occurrence) order, with their
    counts and hashes (dict lookups work, incl. "G" * 32 whose word is ~0: hash -1 -> -2)."""
    import numpy as np
    from shortseq_amd import _shortseq as S

    keys = ["C" * 40, "G" * 32, "", "A" * 32, "T" * 40, "ACGT" * 8, "A" * 100]
    counts = [5, 1, 6, 3, 4, 2, 7]
    words = [int(x) for k in keys if k for x in sq.pack(k).packed[:(len(k) + 31) // 32]]
    c = ShortSeqCounter()
    S._fill_from_arrays(c, np.array([len(k) for k in keys], np.uint32), np.array(counts, np.uint64),
                        np.array(words, np.uint64))
    assert [(str(k), v) for k, v in c.items()] == list(zip(keys, counts))
    assert c[sq.pack("G" * 32)] == 1 and c[sq.pack("ACGT" * 8)] == 2 and c[sq.pack("")] == 6
    assert c[sq.pack("A" * 100)] == 7


def test_import_does_not_load_torch():
    """The drop-in (per-object API and the GPU batch engine) goes Cython -> C ABI: importing it, and
    counting on the host, never imports torch."""
    import subprocess
    import sys
    code = ("import sys, shortseq_amd as sq; sq.ShortSeqCounter([b'ACGT'] * 3, device='host'); "
            "sq.pack('ACGT'); assert 'torch' not in sys.modules, 'torch imported'")
    subprocess.run([sys.executable, "-c", code], check=True, cwd=REPO)


def test_pack_every_byte_value_in_every_block_position(oracle):
    """The host codec's exact-ACGT fast path (AVX2 nibble lookup + PEXT) must hand every other
    byte value to the reference-exact path: each of the 256 byte values at several positions of
    32-, 64- and 75-nt reads packs (or raises) exactly as the oracle."""
    for L in (32, 64, 75):
        for pos in (0, 5, 31, L - 1):
            for b in range(256):
                seq = bytearray(b"ACGT" * 19)[:L]
                seq[pos] = b
                seq = bytes(seq)
                words, err = oracle.encode_one(seq, 32)
                if err.kind == 0:
                    got = sq.pack(seq)
                    nw = max(1, (L + 31) // 32)
                    assert [int(x) for x in got.packed][:nw] == [int(x) for x in words[:nw]], (L, pos, b)
                else:
                    with pytest.raises(BaseException):
                        sq.pack(seq)
