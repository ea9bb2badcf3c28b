"""Multi-rank ShortSeqCounter protocol on CPU: world_size 2 (and 3) over gloo.

The per-rank tables are a host double with GpuCounter's interface (encode via the oracle, exact
counts / first indices, region-range ownership via shortseq_amd.dist.owner_of_region_np with the
device table's geometry); the extract / exchange / merge / gather logic is the product code in
shortseq_amd/dist.py, the same that runs over RCCL on GPUs.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class HostTable:
    """Test double of GpuCounter (same method names and tensor conventions)."""

    def __init__(self, capacity, device=None):
        self.d = {}
        self.log2cap = max(10, int(capacity - 1).bit_length())
        self.slice_log = min(self.log2cap, 11)

    def reset(self):
        self.d = {}

    def close(self):
        pass

    def geometry(self):
        return self.log2cap, self.slice_log

    def insert(self, ascii, L, base_index=0, check_errors=True):
        import oracle
        a = ascii.numpy().reshape(-1)
        n = a.size // L
        words, rc, _ = oracle.encode_batch(a, n, L)
        assert rc == 0
        self.W = words.shape[1] if L > 32 else 1
        for i in range(n):
            k = tuple(int(x) for x in words[i, :self.W]) if L > 32 else int(words[i, 0])
            c, f = self.d.get(k, (0, 1 << 62))
            self.d[k] = (c + 1, min(f, base_index + i))

    # multi-word keys (L > 32): rows of W words; the owner is owner_of(fingerprint) as on the device
    @staticmethod
    def _fp(words):
        m = (1 << 64) - 1

        h = 0x243F6A8885A308D3 ^ len(words)          # ss_device.h words_fp: fp_step per word, fp_final
        for w in words:
            h ^= w & m
            h ^= h >> 29
            h = (h * 0xBF58476D1CE4E5B9) & m
        h ^= h >> 32
        h = (h * 0x94D049BB133111EB) & m
        h ^= h >> 29
        return h if h != m else m - 1

    def extract_words(self, n_parts=1, cap=None):
        from shortseq_amd.dist import owner_of_np
        ks = sorted(self.d)
        fps = np.array([self._fp(k) for k in ks], dtype=np.uint64)
        own = owner_of_np(fps, n_parts) if len(ks) else np.zeros(0, np.int64)
        o = np.argsort(own, kind="stable")
        ks = [ks[i] for i in o]
        words = np.array(ks, dtype=np.uint64).reshape(len(ks), self.W)
        cs = np.array([self.d[k][0] for k in ks], np.int64)
        fs = np.array([self.d[k][1] for k in ks], np.int64)
        parts = np.bincount(own, minlength=n_parts).astype(np.int64)
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x))  # noqa: E731
        return (t(fps[o].view(np.int64)), t(np.zeros(len(ks), np.int32)), t(words.view(np.int64)), t(cs), t(fs),
                t(parts))

    def merge_words(self, words, counts, first):
        ws = words.numpy().view(np.uint64)
        for row, c, f in zip(ws.tolist(), counts.tolist(), first.tolist()):
            k = tuple(int(x) for x in row)
            c0, f0 = self.d.get(k, (0, 1 << 62))
            self.d[k] = (c0 + c, min(f0, f))

    def _region(self, ks):
        with np.errstate(over="ignore"):
            h = ks.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        return (h >> np.uint64(64 - self.log2cap)) >> np.uint64(self.slice_log)

    def _rows(self, ks, own, n_parts):
        o = np.lexsort((ks == np.uint64(0xFFFFFFFFFFFFFFFF), self._region(ks), own)) if len(ks) else np.zeros(0, int)
        ks = ks[o]
        cs = np.array([self.d[int(k)][0] for k in ks], np.int64)
        fs = np.array([self.d[int(k)][1] for k in ks], np.int64)
        parts = np.bincount(own, minlength=n_parts).astype(np.int64)
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x))  # noqa: E731
        return t(ks.view(np.int64)), t(np.full(len(ks), 32, np.int32)), t(cs), t(fs), t(parts)

    def extract(self, n_parts=1, cap=None):
        from shortseq_amd.dist import owner_of_np
        ks = np.array(sorted(self.d), dtype=np.uint64)
        own = owner_of_np(ks, n_parts) if len(ks) else np.zeros(0, np.int64)
        return self._rows(ks, own, n_parts)

    def extract_ranges(self, n_parts, cap=None):
        from shortseq_amd.dist import owner_of_region_np
        ks = np.array(sorted(self.d), dtype=np.uint64)
        own = owner_of_region_np(ks, n_parts, self.log2cap, self.slice_log) if len(ks) else np.zeros(0, np.int64)
        return self._rows(ks, own, n_parts)

    def overflow_word(self):
        return torch.zeros(1, dtype=torch.int64)

    def overflowed(self):
        return False

    def pack_ranges(self, n_parts, skip=-1, first_base=0, cap=None):
        """Records [m, 2] int64: key, count | (first - first_base) << 32 (ss_counter_pack_ranges)."""
        ks, _l, cs, fs, parts = self.extract_ranges(n_parts)
        own = np.repeat(np.arange(n_parts), parts.numpy())
        keep = own != skip
        c = cs.numpy()[keep].astype(np.uint64)
        f = (fs.numpy()[keep] - first_base).astype(np.uint64)
        assert (c < (1 << 32)).all() and (f < (1 << 32)).all()
        rec = np.stack([ks.numpy()[keep], (c | (f << np.uint64(32))).view(np.int64)], 1)
        parts = parts.clone()
        if skip >= 0:
            parts[skip] = 0
        return torch.from_numpy(np.ascontiguousarray(rec)), parts

    def merge_packed(self, rec, runs, part, n_parts, L):
        r = rec.numpy()
        kk = r[:, 0].view(np.uint64)
        lo = r[:, 1].view(np.uint64) & np.uint64(0xFFFFFFFF)
        hi = r[:, 1].view(np.uint64) >> np.uint64(32)
        for b, e, base in runs:
            self.merge_runs(torch.from_numpy(kk[b:e].view(np.int64)), torch.from_numpy(lo[b:e].astype(np.int64)),
                            torch.from_numpy(hi[b:e].astype(np.int64) + base), [(0, e - b)], part, n_parts, L)

    def merge_runs(self, keys, counts, first, runs, part, n_parts, L):
        from shortseq_amd.dist import owner_of_region_np
        kk = keys.numpy().view(np.uint64)
        for b, e in runs:
            assert (owner_of_region_np(kk[b:e], n_parts, self.log2cap, self.slice_log) == part).all()
            for k, c, f in zip(kk[b:e].tolist(), counts[b:e].tolist(), first[b:e].tolist()):
                c0, f0 = self.d.get(k, (0, 1 << 62))
                self.d[k] = (c0 + c, min(f0, f))


def _worker_words(rank, world, port, n, L, U, q):
    sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from shortseq_amd.dist import ShardedCounter
        per = n // world
        a = oracle.gen_pool_reads(7, 8, U, rank * per, per, L)
        sc = ShardedCounter(1 << 14, device="cpu", table_factory=HostTable)
        sc.count(torch.from_numpy(a).view(per, L), L, base_index=rank * per)
        res = sc.gather_items(dst=0)
        if rank == 0:
            q.put([np.asarray(x).tolist() for x in res])
    finally:
        dist.destroy_process_group()


def _worker(rank, world, port, n, L, U, q):
    sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from shortseq_amd.dist import ShardedCounter
        per = n // world
        a = oracle.gen_pool_reads(5, 6, U, rank * per, per, L)
        sc = ShardedCounter(1 << 14, device="cpu", table_factory=HostTable)
        sc.count(torch.from_numpy(a).view(per, L), L, base_index=rank * per)
        # every owned key really belongs to this rank
        keys, _c, _f = sc.owned_items()
        from shortseq_amd.dist import owner_of_region_np
        own = owner_of_region_np(keys.numpy().view(np.uint64), world, *sc.local.geometry())
        assert (own == rank).all()
        res = sc.gather_items(dst=0)
        if rank == 0:
            q.put([np.asarray(x).tolist() for x in res])
    finally:
        dist.destroy_process_group()


class OverflowTable(HostTable):
    """A HostTable whose rank-1 instance reports an overflowed table (one rank's overflow
    must raise on every rank, none left waiting in a collective)."""
    overflow_rank = 1

    def _ovf(self):
        return dist.get_rank() == self.overflow_rank

    def overflow_word(self):
        return torch.tensor([4 if self._ovf() else 0], dtype=torch.int64)

    def overflowed(self):
        return self._ovf()

    def extract_words(self, n_parts=1, cap=None):
        assert not self._ovf(), "an overflowed table must not be extracted and sent"
        return super().extract_words(n_parts, cap)


def _worker_overflow(rank, world, port, L, q):
    sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from shortseq_amd.dist import ShardedCounter
        per = 300
        a = oracle.gen_pool_reads(7, 8, 50, rank * per, per, L)
        sc = ShardedCounter(1 << 14, device="cpu", table_factory=OverflowTable)
        try:
            sc.count(torch.from_numpy(a).view(per, L), L, base_index=rank * per)
            q.put((rank, "no error"))
        except RuntimeError as e:
            q.put((rank, "overflow" if "overflow" in str(e) else repr(e)))
        dist.barrier()          # every rank got here: nobody hangs in the exchange
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_counter_gloo(oracle, world):
    n, L, U = 3000, 32, 200
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, L, U, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    keys, counts, first = res
    per = n // world
    a = oracle.gen_pool_reads(5, 6, U, 0, per * world, L)
    exp = oracle.count([a[i * L:(i + 1) * L].tobytes() for i in range(per * world)])
    assert [int(k) for k in keys] == [w[0] for (w, _L, _c, _f) in exp]
    assert counts == [c for (_w, _L, c, _f) in exp]
    assert first == [f for (_w, _L, _c, f) in exp]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_counter_gloo_multiword(oracle, world):
    """Keys longer than 32 nt (L = 100: four-word keys) through the sharded counter's row exchange
    (extract_words by owner, one all-to-all of rows, merge_words) over gloo: the gathered rows, in
    first-occurrence order, equal oracle.count over the whole stream."""
    n, L, U = 1800, 100, 150
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_words, args=(r, world, port, n, L, U, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    words, counts, first = res
    per = n // world
    a = oracle.gen_pool_reads(7, 8, U, 0, per * world, L)
    exp = oracle.count([a[i * L:(i + 1) * L].tobytes() for i in range(per * world)])
    assert [[int(x) for x in w] for w in words] == [[int(x) for x in w] for (w, _L, _c, _f) in exp]
    assert counts == [c for (_w, _L, c, _f) in exp]
    assert first == [f for (_w, _L, _c, f) in exp]


def test_owner_partition_is_balanced():
    from shortseq_amd.dist import owner_of_np
    keys = np.arange(100000, dtype=np.uint64) * np.uint64(0x9E3779B1)
    for world in (2, 4, 8):
        c = np.bincount(owner_of_np(keys, world), minlength=world)
        assert c.min() > 0.9 * len(keys) / world


def test_region_owner_is_balanced():
    from shortseq_amd.dist import owner_of_region_np
    keys = np.arange(200000, dtype=np.uint64) * np.uint64(0x9E3779B1) + np.uint64(12345)
    for world in (2, 3, 8):
        c = np.bincount(owner_of_region_np(keys, world, 25, 11), minlength=world)
        assert c.min() > 0.9 * len(keys) / world


@pytest.mark.parametrize("L", [32, 100])
def test_sharded_counter_overflow_raises_on_every_rank(L):
    """One rank's table overflows: every rank raises the overflow (single-word records: the word
    rides the size exchange; multi-word rows: checked before extraction and agreed across ranks) and
    all of them reach the barrier after it."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_overflow, args=(r, world, port, L, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == {r: "overflow" for r in range(world)}


def _worker_stats(rank, world, port, n, L, U, q):
    sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from shortseq_amd.dist import ShardedCounter, rank_spread
        per = n // world
        a = oracle.gen_pool_reads(5, 6, U, rank * per, per, L)
        sc = ShardedCounter(1 << 14, device="cpu", table_factory=HostTable)
        st = {}
        sc.count(torch.from_numpy(a).view(per, L), L, base_index=rank * per, stats=st)
        allst = [None] * world
        dist.all_gather_object(allst, st)
        res = sc.gather_items(dst=0)
        if rank == 0:
            q.put((allst, rank_spread(allst), len(res[0])))
    finally:
        dist.destroy_process_group()


def test_exchange_stats_fields_gloo():
    """The N > 1 bench line's per-rank split (unmeasured on GPU hardware: the
    driver's 8-GPU run is the first): ShardedCounter.count(stats=...) over 2 gloo ranks fills local /
    pack / all-to-all / merge ms, records and bytes sent and received, the backend and the world size;
    what the ranks sent equals what they received, and rank_spread gives [min, max] per field."""
    n, L, U, world = 3000, 32, 200, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_stats, args=(r, world, port, n, L, U, q)) for r in range(world)]
    for p in procs:
        p.start()
    allst, spread, uniq = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for k in ("local_ms", "pack_ms", "a2a_ms", "merge_ms", "records_sent", "bytes_sent", "records_received",
              "bytes_received", "backend", "world"):
        assert all(k in d for d in allst), k
    assert [d["rank"] for d in allst] == [0, 1]
    assert all(d["world"] == 2 and d["backend"] == "gloo" for d in allst)
    assert sum(d["records_sent"] for d in allst) == sum(d["records_received"] for d in allst) > 0
    assert all(d["bytes_sent"] == 16 * d["records_sent"] for d in allst)
    assert spread["backend"] == "gloo" and spread["world"] == 2 and spread["ranks"] == 2
    for k in ("local_ms", "pack_ms", "a2a_ms", "merge_ms", "records_sent"):
        lo, hi = spread[k]
        assert lo <= hi and lo == min(d[k] for d in allst)
    assert "rank" not in spread and uniq == U
