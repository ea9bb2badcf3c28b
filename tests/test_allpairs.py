"""All-pairs thresholded hamming (UMI-style dedup).  The distance is the reference
__xor__ (short_seq_64.pyx:77-84 ...), checked against the oracle's pairwise hamming (pinned to the
reference by test_oracle_golden.py); the GPU kernel against brute force over every pair."""
import numpy as np
import pytest


def _brute(oracle, words, n, L, k):
    """Oracle distances of every pair (ora_hamming_ref_batch row by row) -> counts, sorted pairs."""
    cnt = np.zeros(n, dtype=np.int64)
    pairs = []
    for i in range(n - 1):
        d = oracle.hamming_ref_batch(words[i + 1:], n - i - 1, L, words[i])
        js = np.flatnonzero(d <= k) + i + 1
        cnt[i] += len(js)
        cnt[js] += 1
        pairs.extend((i, int(j)) for j in js)
    return cnt, pairs


def _umis(oracle, n, L, U, seed):
    """n reads drawn from U distinct L-mers plus 1-2 substitution variants (a UMI-like pool)."""
    rng = np.random.default_rng(seed)
    base = oracle.gen_reads(seed, 0, U, L).reshape(U, L)
    pick = base[rng.integers(0, U, size=n)].copy()
    mut = rng.random(n) < 0.4
    pos = rng.integers(0, L, size=n)
    pick[mut, pos[mut]] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=int(mut.sum()))]
    return pick.reshape(-1)


def test_brute_force_matches_oracle_pairwise(oracle):
    n, L = 60, 12
    ascii = _umis(oracle, n, L, 10, 1)
    words, _, _ = oracle.encode_batch(ascii, n, L)
    cnt, pairs = _brute(oracle, words, n, L, 1)
    for i, j in pairs[:50]:
        assert oracle.lib().ora_hamming(words[i].ctypes.data, words[j].ctypes.data, L) <= 1
    assert cnt.sum() == 2 * len(pairs)


@pytest.mark.gpu
@pytest.mark.parametrize("L,n,k", [(12, 3000, 1), (10, 2500, 2), (32, 1500, 3), (33, 1100, 2),
                                   (96, 1200, 4), (100, 600, 3), (128, 500, 5), (64, 900, 3),
                                   (150, 700, 6), (1024, 300, 700), (1, 2000, 0)])
def test_all_pairs_gpu(gpu, oracle, L, n, k):
    import torch
    import shortseq_amd.batch as B
    ascii = _umis(oracle, n, L, max(2, n // 20), L + n)
    words, _, _ = oracle.encode_batch(ascii, n, L)
    cnt_e, pairs_e = _brute(oracle, words, n, L, k)
    d = torch.from_numpy(words.view(np.int64)).to(gpu)
    cnt, pairs, total = B.hamming_all_pairs(d, L, k, max_pairs=len(pairs_e) + 10)
    assert total == len(pairs_e)
    assert np.array_equal(cnt.cpu().numpy().astype(np.int64), cnt_e)
    assert [tuple(int(x) for x in p) for p in pairs.cpu().numpy()] == pairs_e
    # count-only and truncated pair output
    cnt2, _, total2 = B.hamming_all_pairs(d, L, k)
    assert total2 == total and torch.equal(cnt2, cnt)
    if total > 4:
        _, p3, total3 = B.hamming_all_pairs(d, L, k, counts=False, max_pairs=3)
        assert total3 == total and p3.shape[0] == 3
