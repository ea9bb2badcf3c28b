"""Generate the golden fixtures in tests/golden/ from the UNMODIFIED reference.

Run in the dev container only (the reference never travels to the GPU box):

    make -C oracle && oracle/build_ref.sh
    cd /tmp && PYTHONPATH=/root/repo/oracle/_ref python3 /root/repo/tests/golden/gen_golden.py

The reference package is imported from oracle/_ref (built by oracle/build_ref.sh from
/root/reference's own .pyx sources).  Packed words are read straight from object memory, the layout
verified in SURVEY §8(c): ShortSeq64 {u64 @ +16, u8 len @ +24}, ShortSeq192 {u64[3] @ +16,
u8 len @ +40}, ShortSeqVar {u64* @ +16, size_t len @ +24}.  Outputs are data only (inputs and
expected outputs); no reference source text is stored.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os
import random
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "oracle"))

import oracle  # noqa: E402  (test infrastructure: generator + capsule harness)

import shortseq.short_seq as ref_sq  # noqa: E402
import shortseq.short_seq_64 as ref64  # noqa: E402
import shortseq.short_seq_192 as ref192  # noqa: E402
import shortseq.short_seq_var as refvar  # noqa: E402
import shortseq.counter as refcounter  # noqa: E402

assert ref_sq.__file__.startswith(oracle.REF_DIR), ref_sq.__file__


def packed_words(obj):
    """(class name, words, length) read from the reference object's memory."""
    a = id(obj)
    t = type(obj)
    if t is ref64.ShortSeq64:
        return "ShortSeq64", [C.c_uint64.from_address(a + 16).value], C.c_uint8.from_address(a + 24).value
    if t is ref192.ShortSeq192:
        return ("ShortSeq192", [C.c_uint64.from_address(a + 16 + 8 * i).value for i in range(3)],
                C.c_uint8.from_address(a + 40).value)
    if t is refvar.ShortSeqVar:
        ptr = C.c_uint64.from_address(a + 16).value
        L = C.c_size_t.from_address(a + 24).value
        n = (L + 31) // 32
        return "ShortSeqVar", [C.c_uint64.from_address(ptr + 8 * i).value for i in range(n)], L
    raise TypeError(t)


def hexw(ws):
    return ["%016x" % w for w in ws]


def exc_record(fn):
    try:
        r = fn()
    except BaseException as e:  # noqa: BLE001 — we record exactly what the reference raised
        return {"raises": type(e).__name__, "message": str(e)}
    cls, ws, L = packed_words(r)
    return {"class": cls, "words": hexw(ws), "length": L}


def vectors(rng):
    lengths = (list(range(0, 41)) + [63, 64, 65, 95, 96, 97, 98, 127, 128, 129, 511, 512, 513,
                                      1023, 1024])
    out = []
    for L in lengths:
        for rep in range(2):
            a = "".join(rng.choice("ACTG") for _ in range(L))
            b = "".join(rng.choice("ACTG") for _ in range(L))
            sa, sb = ref_sq.pack(a.encode()), ref_sq.pack(b)
            cls, ws, ln = packed_words(sa)
            _, wsb, _ = packed_words(sb)
            out.append({"L": L, "a": a, "b": b, "class": cls, "words_a": hexw(ws), "words_b": hexw(wsb),
                        "length": ln, "str_a": str(sa), "hamming": sa ^ sb, "sizeof": sys.getsizeof(sa),
                        "hash_a": hash(sa)})
    return out


def aliased(rng):
    """bloom-aliased bytes < 0x80 (\\x01 \\x03 \\x07 \\x14) at head/middle/tail."""
    out = []
    for L in [1, 2, 3, 8, 15, 16, 17, 31, 32, 33, 34, 40, 63, 64, 65, 95, 96, 97, 100, 128, 200, 1024]:
        for alias in [1, 3, 7, 20]:
            for pos in sorted({0, L // 2, L - 1}):
                seq = bytearray(rng.choice(b"ACGT") for _ in range(L))
                seq[pos] = alias
                r = exc_record(lambda: ref_sq.pack(bytes(seq)))
                r.update({"input_hex": bytes(seq).hex(), "L": L, "pos": pos})
                out.append(r)
        # runs of aliased bytes, incl. a whole block
        seq = bytearray(rng.choice(b"ACGT") for _ in range(L))
        for i in range(0, L, 3):
            seq[i] = [1, 3, 7, 20][i % 4]
        r = exc_record(lambda: ref_sq.pack(bytes(seq)))
        r.update({"input_hex": bytes(seq).hex(), "L": L, "pos": -1})
        out.append(r)
    r = exc_record(lambda: ref_sq.pack(b"\x01" * 40))
    r.update({"input_hex": (b"\x01" * 40).hex(), "L": 40, "pos": -1})
    out.append(r)
    return out


def errors(rng):
    cases = []

    def add(kind, value, fn):
        r = exc_record(fn)
        r.update({"ctor": kind, "input": value})
        cases.append(r)

    for s in ["N", "*", "N" * 33, "*" * 33, "n", "a", "U", "ACGTN", "NACGT", "ANCGNT",
              "ACGT" * 8 + "N", "N" + "ACGT" * 8, "ACGT" * 10 + "NN" + "ACGT" * 3,
              "ACGT" * 20 + "N" + "ACGT" * 5 + "*", "A" * 64 + "N" * 3, "A" * 96 + "N",
              "A" * 1000 + "N", "AC GT", "ACGT\n"]:
        add("pack_str", s, lambda s=s: ref_sq.pack(s))
        add("pack_bytes", s, lambda s=s: ref_sq.pack(s.encode()))
    # invalid at the last position, every length class boundary (reference test :504-515 shape)
    for L in [1, 2, 32, 33, 64, 65, 96, 97, 128, 1023, 1024]:
        s = "".join(rng.choice("ACGT") for _ in range(L - 1)) + "N"
        add("pack_bytes", s, lambda s=s: ref_sq.pack(s.encode()))
    add("pack_str", "ACGT" * 256 + "A", lambda: ref_sq.pack("ACGT" * 256 + "A"))
    add("from_bytes", "", lambda: ref_sq.from_bytes(b""))
    add("from_str", "", lambda: ref_sq.from_str(""))
    # non-ASCII byte inside a full-block chunk: message decode fails (UnicodeDecodeError)
    s = b"A" * 40 + b"\xff" + b"A" * 10
    add("pack_bytes_hex", s.hex(), lambda: ref_sq.pack(s))
    s2 = b"A" * 5 + b"\xff"
    add("pack_bytes_hex", s2.hex(), lambda: ref_sq.pack(s2))
    for bad in [1, 1.5, None, ["A"], bytearray(b"A")]:
        add("pack_obj", repr(bad), lambda bad=bad: ref_sq.pack(bad))
    # hamming length mismatch + cross-class type error
    ham = []
    for a, b in [("ACGT", "ACG"), ("A" * 40, "A" * 41), ("A" * 100, "A" * 101), ("A" * 32, "A" * 33)]:
        try:
            ref_sq.pack(a) ^ ref_sq.pack(b)
            ham.append({"a": a, "b": b, "raises": None})
        except BaseException as e:  # noqa: BLE001
            ham.append({"a": a, "b": b, "raises": type(e).__name__, "message": str(e)})
    return {"pack": cases, "hamming": ham}


def counter_cases(rng):
    cases = []
    inputs = [
        [b"ATGC"] * 10,
        [],
        [b"", b"A", b"AA", b"A", b"", b"AA", b"AAA"],
        [b"G" * 32, b"G" * 32, b"T" * 32, b"G" * 31],
        [b"ACGT" * 9, b"ACGT" * 9, b"ACGT" * 8 + b"ACG", b"A" * 96, b"A" * 96],
        [b"\x01A", b"CA", b"\x01A", b"AC"],
    ]
    pool = ["".join(rng.choice("ACGT") for _ in range(rng.choice([5, 20, 32, 33, 60, 96])))
            for _ in range(40)]
    inputs.append([rng.choice(pool).encode() for _ in range(500)])
    for reads in inputs:
        c = refcounter.ShortSeqCounter(list(reads))
        items = []
        for k, v in c.items():
            cls, ws, L = packed_words(k)
            items.append({"class": cls, "words": hexw(ws), "length": L, "str": str(k), "count": v})
        cases.append({"reads_hex": [r.hex() for r in reads], "items": items})
    # error mid-list: the reference raises on the first bad read (the counter is left partial)
    bad = [b"ACGT", b"ACGN", b"GGGG"]
    try:
        refcounter.ShortSeqCounter(bad)
        cases.append({"reads_hex": [r.hex() for r in bad], "raises": None})
    except BaseException as e:  # noqa: BLE001
        cases.append({"reads_hex": [r.hex() for r in bad], "raises": type(e).__name__, "message": str(e)})
    # str items are rejected (TypeError)
    try:
        refcounter.ShortSeqCounter(["ACGT"])
        cases.append({"reads_str": ["ACGT"], "raises": None})
    except BaseException as e:  # noqa: BLE001
        cases.append({"reads_str": ["ACGT"], "raises": type(e).__name__, "message": str(e)})
    return cases


def fastq_files(rng):
    """FASTQ inputs (bytes) for read_and_count_fastq (counter.pyx:57-70 / fast_read.pyx:3-20)."""
    def rec(i, seq, nl=b"\n"):
        return b"@r%d" % i + nl + seq + nl + b"+" + nl + b"I" * len(seq) + nl
    files = {}
    files["basic_no_trailing_newline"] = b"".join(rec(i, s) for i, s in enumerate(
        [b"ACGT", b"ACGT", b"GGGGA", b"T" * 40, b"ACGT"])) + b"@last\nACGTA"
    mixed = [b"", b"A", b"C" * 32, b"G" * 33, b"ACGT" * 24, b"T" * 97, b"ACG" * 67, b"A", b""]
    files["mixed_lengths"] = b"".join(rec(i, s) for i, s in enumerate(mixed + mixed[::-1]))
    files["crlf"] = b"".join(rec(i, s, b"\r\n") for i, s in enumerate([b"ACGT", b"GGCC"]))
    files["nul_inside"] = rec(0, b"ACGT") + b"@n\nGG\x00TT\n+\nIIIII\n" + rec(2, b"GG")
    files["nul_first"] = rec(0, b"ACGT") + b"@n\n\x00ACGT\n+\nIIIII\n"
    files["invalid_base"] = rec(0, b"ACGT") + rec(1, b"ACGNT") + rec(2, b"AC")
    files["invalid_base_long"] = rec(0, b"ACGT" * 20) + rec(1, b"ACGT" * 10 + b"N" + b"ACGT" * 10)
    files["too_long"] = rec(0, b"ACGT") + rec(1, b"A" * 1025)
    files["max_len"] = rec(0, b"ACGT" * 256) + rec(1, b"ACGT" * 256) + rec(2, b"G" * 1024)
    files["truncated_record"] = rec(0, b"ACGT") + b"@r1\nGGTT\n"
    files["header_only_tail"] = rec(0, b"ACGT") + b"@r1\n"
    files["empty_file"] = b""
    files["seq_no_newline_single"] = b"@r0\nA"
    pool = [bytes(rng.choice(b"ACGT") for _ in range(rng.choice([20, 32, 50, 100]))) for _ in range(50)]
    files["pool_2000"] = b"".join(rec(i, rng.choice(pool)) for i in range(2000))
    return files


def fastq_cases(rng):
    import contextlib
    import io
    import tempfile
    cases = {}
    with tempfile.TemporaryDirectory() as td:
        for name, data in fastq_files(rng).items():
            path = os.path.join(td, name + ".fq")
            with open(path, "wb") as f:
                f.write(data)
            case = {"file_hex": data.hex()}
            try:
                with contextlib.redirect_stdout(io.StringIO()):
                    c = refcounter.read_and_count_fastq(path)
                items = []
                for k, v in c.items():
                    cls, ws, L = packed_words(k)
                    items.append({"class": cls, "words": hexw(ws), "length": L, "str": str(k), "count": v})
                case["items"] = items
                case["raises"] = None
            except BaseException as e:  # noqa: BLE001
                case["raises"] = type(e).__name__
                case["message"] = str(e)
            cases[name] = case
    return cases


def slice_cases(rng):
    """ShortSeq.__getitem__ with slices and ints (short_seq.pyx:78-238, short_seq_64.pyx:53-75,
    short_seq_192.pyx:50-72, short_seq_var.pyx:37-59) on the reference objects."""
    cases = []
    lengths = [1, 2, 5, 31, 32, 33, 63, 64, 65, 95, 96, 97, 127, 128, 129, 200, 511, 512, 1000, 1024]
    for L in lengths:
        seq = "".join(rng.choice("ACGT") for _ in range(L))
        obj = ref_sq.pack(seq)
        items = []
        picks = set()
        for _ in range(40):
            a = rng.randrange(-L - 3, L + 4)
            b = rng.randrange(-L - 3, L + 4)
            picks.add((rng.choice([a, None]), rng.choice([b, None])))
        for a in (0, 1, 31, 32, 33, 63, 64, 65, 95, 96):
            for ln in (1, 31, 32, 33, 64, 96, 97):
                picks.add((a, a + ln))
        for a, b in sorted(picks, key=lambda t: (str(t[0]), str(t[1]))):
            out = obj[a:b]
            cls, ws, ln = packed_words(out)
            items.append({"start": a, "stop": b, "class": cls, "words": hexw(ws), "length": ln, "str": str(out)})
        for step in (2, -1):
            try:
                obj[::step]
                items.append({"step": step, "raises": None})
            except BaseException as e:  # noqa: BLE001
                items.append({"step": step, "raises": type(e).__name__, "message": str(e)})
        idx = []
        for i in sorted({0, L - 1, -1, -L, L, -L - 1, rng.randrange(L)}):
            try:
                out = obj[i]
                cls, ws, ln = packed_words(out)
                idx.append({"index": i, "class": cls, "words": hexw(ws), "length": ln})
            except BaseException as e:  # noqa: BLE001
                idx.append({"index": i, "raises": type(e).__name__, "message": str(e)})
        cases.append({"seq": seq, "slices": items, "indices": idx})
    return cases


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def digests():
    out = {}
    for seed, n, L in [(1, 1_000_000, 32), (2, 1_000_000, 96), (3, 200_000, 512), (4, 300_000, 100)]:
        ascii = oracle.gen_reads(seed, 0, n, L)
        words = oracle.ref_encode_batch(ascii, n, L)
        # independent cross-check on a prefix through the Python API objects
        for i in range(0, n, max(1, n // 500)):
            s = bytes(ascii[i * L:(i + 1) * L])
            _, ws, _ = packed_words(ref_sq.pack(s))
            assert ws[: words.shape[1]] == [int(x) for x in words[i]], (L, i)
        objs = [ref_sq.pack(bytes(ascii[i * L:(i + 1) * L])) for i in range(min(n, 200_000))]
        ham = np.array([o ^ objs[0] for o in objs], dtype=np.uint32)
        out[f"{n}x{L}"] = {"seed": seed, "n": n, "L": L, "wpr": int(words.shape[1]),
                           "words_sha256": sha(words), "hamming_vs_read0_n": len(objs),
                           "hamming_vs_read0_sha256": sha(ham),
                           "hamming_vs_read0_sum": int(ham.sum())}
    # counter: 1M x 32 drawn from a 2^16 pool
    n, L, U = 1_000_000, 32, 1 << 16
    ascii = oracle.gen_pool_reads(5, 77, U, 0, n, L)
    reads = [bytes(ascii[i * L:(i + 1) * L]) for i in range(n)]
    c = refcounter.ShortSeqCounter(reads)
    rows = []
    for k, v in c.items():
        _, ws, ln = packed_words(k)
        rows.append((ws[0], ln, v))
    ordered = np.array([(w, ln, v) for w, ln, v in rows], dtype=np.uint64)
    out["counter_1000000x32_pool65536"] = {
        "seed": 5, "pool_seed": 77, "U": U, "n": n, "L": L, "unique": len(rows),
        "ordered_sha256": sha(ordered), "sorted_sha256": sha(ordered[np.lexsort(ordered.T[::-1])]),
        "max_count": int(ordered[:, 2].max())}
    return out


def main():
    only = [a[len("--only-"):] for a in sys.argv[1:] if a.startswith("--only-")]
    if only:
        # add / refresh some case families without regenerating the other fixtures
        path = os.path.join(OUT, "golden_cases.json")
        with open(path) as f:
            data = json.load(f)
        if "fastq" in only:
            data["fastq"] = fastq_cases(random.Random(20260101))
        if "slices" in only:
            data["slices"] = slice_cases(random.Random(20260102))
        with open(path, "w") as f:
            json.dump(data, f, indent=0, sort_keys=True)
        print("wrote", only, "to", path)
        return
    rng = random.Random(20250216)
    data = {
        "provenance": {"reference": "/root/reference (AlexTate/ShortSeq snapshot 2025-02-16)",
                       "built_by": "oracle/build_ref.sh", "script": "tests/golden/gen_golden.py"},
        "vectors": vectors(rng),
        "aliased": aliased(rng),
        "errors": errors(rng),
        "counter": counter_cases(rng),
        "fastq": fastq_cases(random.Random(20260101)),
        "slices": slice_cases(random.Random(20260102)),
    }
    with open(os.path.join(OUT, "golden_cases.json"), "w") as f:
        json.dump(data, f, indent=0, sort_keys=True)
    with open(os.path.join(OUT, "golden_digests.json"), "w") as f:
        json.dump(digests(), f, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
