"""u64 counts in the bare counter handle (ss_counter; VERDICT r5 missing item 3).  The reference's
counts are Python ints (counter.pyx:47-54: 1, then old + 1): a key seen more than 2^32 - 1 times
must still count exactly.  Checked against oracle.count (pinned to the reference by
test_oracle_golden.py) times the number of repeats, and against plain arithmetic past 2^32."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pool(oracle, n, U, seed):
    return oracle.gen_pool_reads(seed, seed + 1, U, 0, n, 32)


@pytest.mark.parametrize("n,limit,partitioned", [(20_000, 1000, False), (300_000, 100_000, True),
                                                 (300_000, 1_000_000, True)])
def test_counter_spill_limit_exact(gpu, oracle, n, limit, partitioned):
    """A low spill limit (the test hook) moves the u32 slot counts into the u64 array between and
    before inserts many times; the counts (direct and partitioned inserts) still equal the oracle's,
    times the repeats, with first = the first occurrence."""
    import torch
    import shortseq_amd.batch as B
    pool = _pool(oracle, n, 3000, 7)
    reads = [pool[i * 32:(i + 1) * 32].tobytes() for i in range(n)]
    exp = oracle.count(reads)
    d = torch.from_numpy(pool).to(gpu).view(-1, 32)
    c = B.GpuCounter(1 << 14, device=gpu)
    try:
        c.set_spill_limit(limit)
        reps = 5
        for _ in range(reps):
            c.insert(d, 32, partitioned=partitioned)      # base_index 0 every time: same first indices
        k, cnt, f = c.items_sorted()
        assert [int(x) for x in k] == [w[0] for (w, _L, _c, _f) in exp]
        assert [int(x) for x in cnt] == [reps * cc for (_w, _L, cc, _f) in exp]
        assert [int(x) for x in f] == [ff for (_w, _L, _c, ff) in exp]
    finally:
        c.close()


def test_counter_merge_counts_past_2_32(gpu):
    """ss_counter_merge with u64 counts: a key merged twice at 3e9 (6e9 total), one at 2^32 + 5 in one
    entry, one that carries exactly at 2^32, the sentinel key ~0 ('G' * 32) past 2^32 -- exact, and
    the overflow word stays clear."""
    import torch
    import shortseq_amd.batch as B
    keys = torch.tensor([11, 22, 33, -1], dtype=torch.int64, device=gpu)
    counts = torch.tensor([3_000_000_000, (1 << 32) + 5, (1 << 32) - 1, 3_000_000_000], dtype=torch.int64, device=gpu)
    first = torch.tensor([5, 6, 7, 8], dtype=torch.int64, device=gpu)
    c = B.GpuCounter(1 << 12, device=gpu)
    try:
        c.merge(keys, counts, first, 32)
        c.merge(keys[[0, 2, 3]], torch.tensor([3_000_000_000, 1, 3_000_000_000], dtype=torch.int64, device=gpu),
                torch.tensor([9, 1, 2], dtype=torch.int64, device=gpu), 32)
        k, cnt, f = c.items_sorted()
        got = {int(a): (int(b), int(x)) for a, b, x in zip(k.view(np.int64), cnt, f)}
        assert got == {11: (6_000_000_000, 5), 22: ((1 << 32) + 5, 6), 33: (1 << 32, 1), -1: (6_000_000_000, 2)}
        assert not c.overflowed()
        # an insert after the merges spills first (the slots' u32 parts are no longer bounded)
        d = torch.frombuffer(bytearray(b"A" * 31 + b"C"), dtype=torch.uint8).to(gpu).view(1, 32)
        c.insert(d, 32, base_index=0, partitioned=False)
        k2, cnt2, _ = c.items_sorted()
        assert int(cnt2[list(k2.view(np.int64)).index(11)]) == 6_000_000_000 and len(k2) == 5
    finally:
        c.close()


def test_counter_one_key_past_2_32_reads(gpu):
    """The production partitioned insert counts one 32-mer 4.3e9 times (43 inserts of a 100M-read
    batch of copies, each at base index 0): the automatic spill keeps the count exact past 2^32."""
    import torch
    import shortseq_amd.batch as B
    n, reps = 100_000_000, 43
    row = torch.frombuffer(bytearray(b"ACGTTGCA" * 4), dtype=torch.uint8).to(gpu)
    d = row.expand(n, 32).contiguous()
    c = B.GpuCounter(1 << 20, device=gpu)
    try:
        for _ in range(reps):
            c.insert(d, 32, check_errors=False)
        k, cnt, f = c.items_sorted()
        assert len(k) == 1 and int(cnt[0]) == reps * n and int(f[0]) == 0
        assert reps * n > (1 << 32)
    finally:
        c.close()
        del d
        torch.cuda.empty_cache()
