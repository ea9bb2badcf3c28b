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


@pytest.mark.gpu
@pytest.mark.parametrize("L,n,k", [(12, 3000, 1), (10, 2500, 2), (32, 1500, 3), (31, 1200, 5), (1, 2000, 0),
                                   (8, 1000, 15), (20, 1500, 0), (16, 800, 4),
                                   # multi-word rows (round 6): segments across word boundaries, longer
                                   # than 32 positions (hashed), the alias position in the last word
                                   (33, 1200, 1), (40, 1500, 2), (64, 1000, 3), (65, 900, 0), (96, 1000, 5),
                                   (100, 800, 1), (128, 700, 4), (127, 600, 15), (50, 900, 7)])
def test_all_pairs_pigeonhole_gpu(gpu, oracle, L, n, k):
    """The bucketed pigeonhole form against the oracle's brute force (same pairs, counts, total)."""
    import torch
    import shortseq_amd.batch as B
    ascii = _umis(oracle, n, L, max(2, n // 20), 3 * L + n)
    words, _, _ = oracle.encode_batch(ascii, n, L)
    cnt_e, pairs_e = _brute(oracle, words, n, L, k)
    d = torch.from_numpy(words.view(np.int64)).to(gpu)
    cnt, pairs, total = B.hamming_all_pairs(d, L, k, max_pairs=len(pairs_e) + 10, method="pigeonhole")
    assert total == len(pairs_e)
    assert np.array_equal(cnt.cpu().numpy().astype(np.int64), cnt_e)
    assert [tuple(int(x) for x in p) for p in pairs.cpu().numpy()] == pairs_e
    cnt2, _, total2 = B.hamming_all_pairs(d, L, k, method="pigeonhole")
    assert total2 == total and torch.equal(cnt2, cnt)
    if total > 4:    # truncated pair output: the total still counts every pair, the kept ones are real
        _, p3, total3 = B.hamming_all_pairs(d, L, k, counts=False, max_pairs=3, method="pigeonhole")
        assert total3 == total and p3.shape[0] == 3
        assert {tuple(int(x) for x in q) for q in p3.cpu().numpy()} <= set(pairs_e)


def _pair_set(pairs):
    p = pairs.cpu().numpy().astype(np.int64)
    return p[:, 0] * (1 << 32) + p[:, 1]


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["random12", "umi_pool12", "dups10", "random16k2", "random32_hashed", "one_read"])
def test_all_pairs_methods_agree_large(gpu, oracle, case):
    """At bench-like sizes (n >= 2^15, where auto may pick either form): tiles, pigeonhole and auto
    give the same counts, totals and pair sets, for uniform UMIs, a UMI pool with 1-nt variants,
    10-fold duplicates and a batch of one repeated read (every pair a hit)."""
    import torch
    import shortseq_amd.batch as B
    rng = np.random.default_rng(11)
    L, k, n = 12, 1, 100_000
    if case == "random12":
        ascii = oracle.gen_reads(5, 0, n, L)
    elif case == "umi_pool12":
        ascii = _umis(oracle, n, L, 20_000, 5)
    elif case == "dups10":
        base = oracle.gen_reads(6, 0, n // 10, L).reshape(-1, L)
        ascii = base[rng.integers(0, n // 10, size=n)].reshape(-1)
    elif case == "random16k2":
        L, k = 16, 2
        ascii = oracle.gen_reads(7, 0, n, L)
    elif case == "random32_hashed":      # 16-nt segments: buckets by a hash of 32 bits to 17
        L, k = 32, 1
        ascii = _umis(oracle, n, L, 30_000, 9)
    else:
        n = 40_000
        ascii = np.tile(oracle.gen_reads(8, 0, 1, L), n)
    words, _, _ = oracle.encode_batch(ascii, n, L)
    d = torch.from_numpy(words.view(np.int64)).to(gpu)
    cnt_t, _, tot_t = B.hamming_all_pairs(d, L, k, method="tiles")
    # one repeated read: auto must hand it to the tiles (forced pigeonhole runs on a slice below)
    for m in (("auto",) if case == "one_read" else ("pigeonhole", "auto")):
        cnt, _, tot = B.hamming_all_pairs(d, L, k, method=m)
        assert tot == tot_t and torch.equal(cnt, cnt_t), m
    if tot_t <= 2_000_000:
        _, p_t, _ = B.hamming_all_pairs(d, L, k, max_pairs=tot_t, counts=False, method="tiles")
        _, p_g, _ = B.hamming_all_pairs(d, L, k, max_pairs=tot_t, counts=False, method="pigeonhole")
        assert np.array_equal(_pair_set(p_t), _pair_set(p_g))
    assert int(cnt_t.sum().item()) == 2 * tot_t
    if case == "one_read":
        m = 3000
        cnt, _, tot = B.hamming_all_pairs(d[:m], L, k, method="pigeonhole")
        assert tot == m * (m - 1) // 2 and bool((cnt == m - 1).all())


@pytest.mark.gpu
def test_all_pairs_pigeonhole_refuses_long_reads(gpu):
    import torch
    import shortseq_amd.batch as B
    from shortseq_amd._native import NativeError
    d = torch.zeros((10, 5), dtype=torch.int64, device=gpu)
    with pytest.raises(NativeError):
        B.hamming_all_pairs(d, 130, 1, method="pigeonhole")
    with pytest.raises(NativeError):
        B.hamming_all_pairs(d[:, :1].contiguous(), 20, 16, method="pigeonhole")


@pytest.mark.gpu
def test_all_pairs_pigeonhole_past_2_22(gpu, oracle):
    """n > 2^22 reads (the bucket tables at their 2^22 cap: 1024 scan tiles per segment, hashed
    segment values): the pigeonhole form's counts and total equal the tiled form's."""
    import torch
    import shortseq_amd.batch as B
    n, L, k = (1 << 22) + 12345, 20, 1
    ascii = _umis(oracle, n, L, 1 << 21, 13)
    words, _, _ = oracle.encode_batch(ascii, n, L)
    d = torch.from_numpy(words.view(np.int64)).to(gpu)
    cnt_t, _, tot_t = B.hamming_all_pairs(d, L, k, method="tiles")
    cnt_p, _, tot_p = B.hamming_all_pairs(d, L, k, method="pigeonhole")
    assert tot_p == tot_t and torch.equal(cnt_p, cnt_t)
    assert int(cnt_t.sum().item()) == 2 * tot_t and tot_t > 0


@pytest.mark.gpu
def test_all_pairs_auto_is_capturable(gpu, oracle):
    """AUTO on a stream under hipGraph capture stays on the tiles (no allocation, no host read-back:
    ADVICE r5), so a batch auto would hand to the pigeonhole form captures and replays with the same
    counts and total as the eager call."""
    import torch
    import shortseq_amd.batch as B
    from shortseq_amd._native import lib, check
    n, L, k = 1 << 15, 12, 1
    ascii = _umis(oracle, n, L, 8000, 21)
    words, _, _ = oracle.encode_batch(ascii, n, L)
    d = torch.from_numpy(words.view(np.int64)).to(gpu)
    cnt_e, _, tot_e = B.hamming_all_pairs(d, L, k, method="auto")
    cnt = torch.empty(n, dtype=torch.int32, device=gpu)
    tot = torch.empty(1, dtype=torch.int64, device=gpu)
    torch.cuda.synchronize(gpu)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream(gpu).cuda_stream
        check(lib().ss_hamming_all_pairs_ex(d.data_ptr(), n, L, 1, k, cnt.data_ptr(), 0, 0, tot.data_ptr(),
                                            B.ALL_PAIRS_METHODS["auto"], s), "captured all pairs")
    cnt.fill_(-1)
    g.replay()
    torch.cuda.synchronize(gpu)
    assert int(tot.item()) == tot_e and torch.equal(cnt, cnt_e)


@pytest.mark.gpu
@pytest.mark.parametrize("L,k,U", [(64, 2, 20_000), (100, 1, 30_000), (128, 3, 20_000), (50, 4, 5_000)])
def test_all_pairs_multiword_methods_agree_large(gpu, oracle, L, k, U):
    """Multi-word reads at bench-like sizes (n = 60k, where auto may pick either form): the
    pigeonhole form over the row's words, the tiles and auto give the same counts, totals and pair
    sets (UMI-like pools with 1-2 substitution variants)."""
    import torch
    import shortseq_amd.batch as B
    n = 60_000
    ascii = _umis(oracle, n, L, U, L + k)
    words, _, _ = oracle.encode_batch(ascii, n, L)
    d = torch.from_numpy(words.view(np.int64)).to(gpu)
    cnt_t, _, tot_t = B.hamming_all_pairs(d, L, k, method="tiles")
    for m in ("pigeonhole", "auto"):
        cnt, _, tot = B.hamming_all_pairs(d, L, k, method=m)
        assert tot == tot_t and torch.equal(cnt, cnt_t), m
    if tot_t <= 2_000_000:
        _, p_t, _ = B.hamming_all_pairs(d, L, k, max_pairs=tot_t, counts=False, method="tiles")
        _, p_g, _ = B.hamming_all_pairs(d, L, k, max_pairs=tot_t, counts=False, method="pigeonhole")
        assert np.array_equal(_pair_set(p_t), _pair_set(p_g))
    assert tot_t > 0
