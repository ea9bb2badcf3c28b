"""Slicing / subscript: ShortSeq.__getitem__ (short_seq_64.pyx:53-75,
short_seq_192.pyx:50-72, short_seq_var.pyx:37-59 -> short_seq.pyx:78-238).

Golden: tests/golden/golden_cases.json["slices"], the unmodified reference's obj[a:b] / obj[i] on
20 read lengths (1..1024) with random and block-boundary bounds (gen_golden.py --only-slices).
CPU: the oracle's restatement (ora_slice) and the drop-in objects reproduce them.  GPU: the batch
kernels (ss_slice_fixed / ss_slice_var) against the oracle.
"""
import random

import numpy as np
import pytest

import shortseq_amd as sq


def _w(hexlist):
    return [int(h, 16) for h in hexlist]


def _same(got, exp):
    """Equal as packed sequences: ShortSeq192 keeps 3 words, unused ones 0."""
    m = max(len(got), len(exp))
    return list(got) + [0] * (m - len(got)) == list(exp) + [0] * (m - len(exp))


def _words_of(oracle, seq):
    L = len(seq)
    words, err = oracle.encode_one(seq.encode(), max(1, (L + 31) // 32))
    assert err.kind == 0
    return words


def test_oracle_slice_pinned_to_reference(oracle, golden):
    n = 0
    for case in golden["slices"]:
        seq = case["seq"]
        src = _words_of(oracle, seq)
        for it in case["slices"]:
            if "step" in it:
                continue
            st, sp, _ = slice(it["start"], it["stop"]).indices(len(seq))
            ln = max(0, sp - st)
            assert ln == it["length"]
            got = oracle.slice_words(src, st if ln else 0, ln)
            exp = _w(it["words"])
            assert _same(got, exp), (len(seq), it)
            n += 1
        for it in case["indices"]:
            if "raises" in it:
                continue
            i = it["index"] % len(seq)
            assert oracle.slice_words(src, i, 1) == _w(it["words"])
    assert n > 1500


def _cls(L):
    return "ShortSeq64" if L <= 32 else ("ShortSeq192" if L <= 96 else "ShortSeqVar")


def test_dropin_getitem_golden(golden):
    for case in golden["slices"]:
        obj = sq.pack(case["seq"])
        for it in case["slices"]:
            if "step" in it:
                with pytest.raises(TypeError) as ei:
                    obj[::it["step"]]
                assert str(ei.value) == it["message"]
                continue
            out = obj[it["start"]:it["stop"]]
            assert (type(out).__name__, len(out), str(out)) == (it["class"], it["length"], it["str"])
            if it["length"]:
                exp = _w(it["words"])
                assert _same(out.packed, exp)
        for it in case["indices"]:
            if "raises" in it:
                with pytest.raises(IndexError) as ei:
                    obj[it["index"]]
                assert str(ei.value) == it["message"]
            else:
                out = obj[it["index"]]
                assert type(out).__name__ == "ShortSeq64" and len(out) == 1
                assert list(out.packed) == _w(it["words"])


@pytest.mark.gpu
def test_slice_fixed_gpu(gpu, oracle):
    import torch
    import shortseq_amd.batch as B
    rng = random.Random(31)
    for L in (1, 7, 32, 33, 64, 96, 97, 150, 512, 1024):
        n = 3000
        ascii = oracle.gen_reads(40 + L, 0, n, L)
        words, rc, _ = oracle.encode_batch(ascii, n, L)
        d = torch.from_numpy(words.view(np.int64)).to(gpu)
        bounds = {(0, L), (0, 1), (L - 1, L), (None, None)}
        for _ in range(12):
            a, b = rng.randrange(-L - 2, L + 3), rng.randrange(-L - 2, L + 3)
            bounds.add((a, b))
        for s in (31, 32, 33, 64, 65):
            if s < L:
                bounds.add((s, min(L, s + 40)))
        for a, b in bounds:
            out, ln = B.slice_fixed(d, L, a, b)
            got = out.cpu().numpy().view(np.uint64)
            st = slice(a, b).indices(L)[0]
            for i in range(0, n, 97):
                exp = oracle.slice_words(words[i], st if ln else 0, ln)
                assert [int(x) for x in got[i]] == exp, (L, a, b, i)


@pytest.mark.gpu
def test_slice_var_gpu(gpu, oracle):
    import torch
    import shortseq_amd.batch as B
    rng = np.random.default_rng(32)
    n, L = 20000, 150
    ascii = oracle.gen_reads(50, 0, n, L)
    words, _, _ = oracle.encode_batch(ascii, n, L)
    rlens = rng.integers(0, L + 1, size=n).astype(np.int32)
    starts = rng.integers(0, L + 10, size=n).astype(np.int32)
    lens = rng.integers(0, L + 10, size=n).astype(np.int32)
    t = lambda a: torch.from_numpy(a).to(gpu)  # noqa: E731
    out = B.slice_var(t(words.view(np.int64)), t(starts), t(lens), read_lens=t(rlens))
    got = out.cpu().numpy().view(np.uint64)
    for i in range(n):
        st = min(int(starts[i]), int(rlens[i]))
        ln = min(int(lens[i]), int(rlens[i]) - st)
        exp = oracle.slice_words(words[i], st, ln)
        assert [int(x) for x in got[i][:len(exp)]] == exp and not got[i][len(exp):].any(), i
