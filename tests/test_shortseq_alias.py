"""`import shortseq as sq` — the reference's import name (shortseq/__init__.py:1-14) — gives the
drop-in.  The reference's own tests start with exactly these imports (tests/unit_tests_main.py:6-9);
the checks below restate a seeded subset of what that file then asserts (empty singleton, class per
length, round trip over every length, hamming, rejection, the counter, slices) against the alias.

Runs in a child interpreter whose path holds only this repository: the main pytest process may
have the compiled reference (oracle/_ref) imported under the same name for the oracle tests.
"""
import os
import subprocess
import sys
import textwrap

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent(r'''
    import random
    import shortseq as sq
    from shortseq import ShortSeq64, ShortSeq192, ShortSeqVar
    from shortseq import MIN_VAR_NT, MAX_VAR_NT, MIN_64_NT, MAX_64_NT, MIN_192_NT, MAX_192_NT
    from shortseq.counter import ShortSeqCounter, read_and_count_fastq
    from shortseq.short_seq import pack, from_str, from_bytes
    import shortseq.short_seq_64, shortseq.short_seq_192, shortseq.short_seq_var

    assert sq.__file__.startswith(REPO), sq.__file__
    assert (MIN_64_NT, MAX_64_NT, MIN_192_NT, MAX_192_NT, MIN_VAR_NT, MAX_VAR_NT) == (0, 32, 33, 96, 97, 1024)
    rng = random.Random(1234)
    rand = lambda L: "".join(rng.choice("ACGT") for _ in range(L))
    # empty sequences are one singleton ShortSeq64, from str and from bytes
    assert sq.pack("") is sq.pack(b"") and type(sq.pack("")) is ShortSeq64 and len(sq.pack("")) == 0
    # the class follows the length, and every length round-trips (str and bytes input)
    for L in range(0, MAX_VAR_NT + 1):
        s = rand(L)
        a, b = sq.pack(s), sq.pack(s.encode())
        want = ShortSeq64 if L <= MAX_64_NT else ShortSeq192 if L <= MAX_192_NT else ShortSeqVar
        assert type(a) is want and type(b) is want and len(a) == L
        assert str(a) == s and str(b) == s and a == s
        # hamming distance against a copy with k substitutions
        if L:
            k = rng.randint(0, L)
            pos = rng.sample(range(L), k)
            t = list(s)
            for p in pos:
                t[p] = rng.choice([c for c in "ACGT" if c != t[p]])
            assert a ^ sq.pack("".join(t)) == k
        # subscripts and a random slice
        if L:
            i = rng.randrange(L)
            assert a[i] == s[i] and a[-1] == s[-1]
            x, y = sorted(rng.sample(range(L + 1), 2))
            assert str(a[x:y]) == s[x:y]
    # rejection of non-nucleotide characters and of over-long input
    for bad in ("ACGTN", "acgt", "ACGU" * 10):
        try:
            sq.pack(bad)
        except Exception as e:
            assert "Unsupported base character" in str(e)
        else:
            raise AssertionError(bad)
    try:
        sq.pack("A" * 1025)
    except Exception as e:
        assert "longer than 1024" in str(e)
    else:
        raise AssertionError("1025 nt accepted")
    # the counter: list of bytes, counts and first-occurrence order
    reads = [rand(rng.choice((0, 5, 32, 40, 96, 150))).encode() for _ in range(300)]
    reads += reads[:100]
    c = ShortSeqCounter(reads)
    exp = {}
    for r in reads:
        exp[r.decode()] = exp.get(r.decode(), 0) + 1
    assert [str(k) for k in c] == list(exp) and [c[k] for k in c] == list(exp.values())
    print("ALIAS OK")
''')


def test_import_shortseq_alias():
    env = dict(os.environ)
    env["PYTHONPATH"] = REPO
    env["REPO"] = REPO
    r = subprocess.run([sys.executable, "-c", f"REPO = {REPO!r}\n" + SCRIPT], cwd="/", env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "ALIAS OK" in r.stdout, r.stdout + r.stderr
