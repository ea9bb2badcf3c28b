"""Sharded ShortSeqCounter across GPUs: one process per GPU, torch.distributed.

Region-range ownership: the table's R regions (slices of 2048 slots, the unit the partitioned
insert aggregates) are split into `world` contiguous ranges, rank p owning
[ceil(p R / world), ceil((p + 1) R / world)); every rank's table has the same geometry.
  1. each rank counts its contiguous shard of the read stream in its own HBM table
     (GpuCounter.insert: fused encode + partitioned LDS aggregation);
  2. it packs the entries of the OTHER ranks' regions into 16-B records {key, count u32, first -
     base u32}, grouped by owner and sorted by region (GpuCounter.pack_ranges: one workgroup per
     region, one pass over the table using the occupancy the insert's aggregate recorded);
  3. ONE exchange step: all_to_all_single of (sizes, base index) per peer, then of the records —
     RCCL over xGMI on MI355X (backend "nccl"), gloo in the CPU tests;
  4. each rank folds what it received into its OWN table's owned regions (GpuCounter.merge_packed:
     one workgroup per region, the region's slice in LDS, no global atomics, no second table).
The result is the union of the ranks' owned regions; gather_items() brings it to one rank in
first-occurrence order (the reference dict's insertion order, counter.pyx:41-54).

Keys longer than 32 nt (ShortSeq192 / ShortSeqVar keys, W = ceil(L / 32) packed words, counted under
a 64-bit fingerprint with equality on the words): the owner is owner_of(fingerprint); each rank
extracts its entries grouped by owner (GpuCounter.extract_words), sends the other owners' rows
(W words, count, first) in one all_to_all_single of int64 rows, and folds what it receives into its
own table (GpuCounter.merge_words: find / claim on the words).  owned_items() / gather_items() then
return the words rows.

Encode / decode / hamming need no collective at all: their shards are independent.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

_M64 = (1 << 64) - 1


def owner_of_np(keys: np.ndarray, nparts: int) -> np.ndarray:
    """Host mirror of the device owner function (csrc/ss_counter.hip owner_of):
    (splitmix64(key) >> 32) % nparts.  Used by tests and by host-side routing."""
    with np.errstate(over="ignore"):
        z = keys.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return ((z >> np.uint64(32)) % np.uint64(nparts)).astype(np.int64)


def owner_of_region_np(keys: np.ndarray, nparts: int, log2cap: int, slice_log: int) -> np.ndarray:
    """Host mirror of the region-range owner (csrc/ss_counter.hip part_of, ranges = true): region =
    top log2cap bits of the Fibonacci hash >> slice_log; owner = region * nparts // R."""
    k = keys.astype(np.uint64)
    with np.errstate(over="ignore"):
        h = k * np.uint64(0x9E3779B97F4A7C15)
    top = (h >> np.uint64(64 - log2cap)) if log2cap > 0 else np.zeros_like(h)
    region = (top >> np.uint64(slice_log)).astype(np.int64)
    R = 1 << (log2cap - slice_log)
    return region * nparts // R


def exchange(keys: torch.Tensor, counts: torch.Tensor, first: torch.Tensor, part_counts: torch.Tensor,
             group=None, with_sizes: bool = False):
    """All-to-all of owner-grouped (key, count, first) int64 triples.

    keys/counts/first: entries grouped by destination rank, part_counts[r] of them for rank r (in
    rank order).  Returns the (keys, counts, first) this rank receives, concatenated in source-rank
    order (and the per-source sizes if with_sizes).  Works on any backend whose all_to_all_single
    supports uneven splits (nccl/RCCL, gloo)."""
    world = dist.get_world_size(group)
    dev = keys.device
    if dev.type != "cpu" and dist.get_backend(group) == "gloo":
        # rehearsal / CPU-collective path: gloo moves host tensors only
        out = exchange(keys.cpu(), counts.cpu(), first.cpu(), part_counts.cpu(), group, with_sizes)
        return tuple(x.to(dev) for x in out[:3]) + tuple(out[3:])
    sc = part_counts.to(torch.int64)
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rc, sc, group=group)
    sc_l = [int(x) for x in sc.tolist()]
    rc_l = [int(x) for x in rc.tolist()]
    m = sum(sc_l)
    send = torch.stack([keys[:m], counts[:m], first[:m]], 1).contiguous()
    recv = torch.empty((sum(rc_l), 3), dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv, send, output_split_sizes=rc_l, input_split_sizes=sc_l, group=group)
    out = (recv[:, 0].contiguous(), recv[:, 1].contiguous(), recv[:, 2].contiguous())
    return out + (rc_l,) if with_sizes else out


def exchange_rows(rows: torch.Tensor, part_counts, group=None, flag: int = 0):
    """All-to-all of owner-grouped int64 rows ([m, k], part_counts[r] rows for rank r in rank order):
    one small all-to-all of the sizes (each with this rank's error flag), one host sync, one
    all-to-all of the rows.  Returns (the rows this rank receives in source-rank order, per-source
    sizes, the largest flag any rank sent).  A raised flag anywhere skips the row all-to-all on
    every rank alike (no rank is left waiting in it), and the rows returned are then empty."""
    world = dist.get_world_size(group)
    dev = rows.device
    if dev.type != "cpu" and dist.get_backend(group) == "gloo":
        out, sizes, f = exchange_rows(rows.cpu(), torch.as_tensor(part_counts).cpu(), group, flag)
        return out.to(dev), sizes, f
    sc = torch.as_tensor(part_counts, dtype=torch.int64).to(dev)
    meta = torch.stack([sc, torch.full((world,), int(flag), dtype=torch.int64, device=dev)], 1)
    rmeta = torch.empty_like(meta)
    dist.all_to_all_single(rmeta, meta, group=group)
    host = torch.cat([sc, rmeta.reshape(-1)]).cpu().tolist()            # the one host sync
    sc_l = [int(x) for x in host[:world]]
    rc_l = [int(host[world + 2 * p]) for p in range(world)]
    fmax = max(int(flag), *[int(host[world + 2 * p + 1]) for p in range(world)])
    if fmax:
        return torch.empty((0, rows.shape[1]), dtype=torch.int64, device=dev), [0] * world, fmax
    m = sum(sc_l)
    recv = torch.empty((sum(rc_l), rows.shape[1]), dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv, rows[:m].contiguous(), output_split_sizes=rc_l, input_split_sizes=sc_l, group=group)
    return recv, rc_l, 0


def rank_spread(per_rank: list) -> dict:
    """Per-rank diagnostic dicts (ShardedCounter.count(stats=...)) -> {field: [min, max]} for the
    numeric fields, plus the backend and the world size every rank saw (a list if they differ)."""
    out = {}
    if not per_rank:
        return out
    for k in per_rank[0]:
        vals = [d.get(k) for d in per_rank]
        if k in ("backend", "world"):
            u = sorted(set(vals), key=str)
            out[k] = u[0] if len(u) == 1 else u
        elif all(isinstance(v, (int, float)) and not isinstance(v, bool) for v in vals) and k != "rank":
            out[k] = [min(vals), max(vals)]
    out["ranks"] = len(per_rank)
    return out


def agree_flag(flag: int, device, group=None) -> int:
    """The largest of every rank's flag (one all_reduce MAX): a check that raises on one rank raises
    on all of them, so none is left waiting in the next collective."""
    t = torch.tensor([int(flag)], dtype=torch.int64,
                     device=device if dist.get_backend(group) != "gloo" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def exchange_packed(rec: torch.Tensor, part_counts: torch.Tensor, first_base: int, group=None,
                    extra: torch.Tensor = None):
    """All-to-all of owner-grouped packed records (int64 [m, 2] = 16 B each, ss_counter_pack_ranges).

    One small all-to-all carries (records for you, my first_base, my `extra` word) per peer; then
    ONE host sync reads this rank's send sizes and the received metadata together, and one
    all-to-all moves the records (RCCL needs the split sizes on the host; a fixed-capacity exchange
    would avoid the sync but move the whole region range, 2x the records at the table's 0.5 load
    factor).  `extra` (e.g. the table's overflow word) travels to every peer: when any rank's is
    nonzero, every rank skips the record all-to-all and gets that word back, so all of them raise
    alike.  Returns (received records in source-rank order, per-source sizes, per-source first_base,
    [the OR of every rank's extra word] or None)."""
    world = dist.get_world_size(group)
    dev = rec.device
    if dev.type != "cpu" and dist.get_backend(group) == "gloo":
        out = exchange_packed(rec.cpu(), part_counts.cpu(), first_base, group,
                              None if extra is None else extra.cpu())
        return (out[0].to(dev),) + tuple(out[1:])
    ex_word = (extra.reshape(-1)[:1].to(torch.int64) if extra is not None
               else torch.zeros(1, dtype=torch.int64, device=dev))
    meta = torch.stack([part_counts.to(torch.int64),
                        torch.full((world,), first_base, dtype=torch.int64, device=dev),
                        ex_word.expand(world)], 1)
    rmeta = torch.empty_like(meta)
    dist.all_to_all_single(rmeta, meta, group=group)
    host = torch.cat([meta[:, 0], rmeta.reshape(-1)]).cpu().tolist()    # the one host sync
    sc_l = [int(x) for x in host[:world]]
    rc_l = [int(host[world + 3 * p]) for p in range(world)]
    bases = [int(host[world + 3 * p + 1]) for p in range(world)]
    ex_or = 0
    for p in range(world):
        ex_or |= int(host[world + 3 * p + 2]) & ((1 << 64) - 1)
    ex = [ex_or] if extra is not None else None
    if ex_or:            # some rank cannot send its records: nobody exchanges, everybody raises
        return torch.empty((0, 2), dtype=torch.int64, device=dev), [0] * world, bases, ex
    m = sum(sc_l)
    recv = torch.empty((sum(rc_l), 2), dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv, rec[:m], output_split_sizes=rc_l, input_split_sizes=sc_l, group=group)
    return recv, rc_l, bases, ex


class ShardedCounter:
    """Per-rank handle: one table per rank (it counts the rank's reads and, after the exchange, holds
    the rank's owned regions), reused across batches."""

    def __init__(self, capacity: int, device=None, group=None, table_factory=None):
        """table_factory(capacity, device) builds the per-rank table; default GpuCounter (HBM).
        Tests inject a host double with the same methods to exercise the exchange on gloo."""
        if table_factory is None:
            from .batch import GpuCounter as table_factory
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self.local = table_factory(capacity, device=self.device)
        self.L: Optional[int] = None

    def close(self) -> None:
        self.local.close()

    def _sync(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def count(self, ascii_local: torch.Tensor, L: int, base_index: int, check_errors: bool = True,
              stats: Optional[dict] = None):
        """Count this rank's shard (global read indices base_index ...) and run the exchange.
        Returns the rank's table; its owned regions hold the exact counts afterwards.
        stats (a diagnostic run): the device is synchronised around each phase and
        the dict receives local_ms (reset + insert), pack_ms, a2a_ms (both all-to-alls and their host
        sync), merge_ms, records / bytes sent and received, the backend and the world size seen."""
        import time
        clk = []

        def mark():
            if stats is not None:
                self._sync()
                clk.append(time.perf_counter())

        mark()
        self.L = L
        self.local.reset()
        self.local.insert(ascii_local, L, base_index=base_index, check_errors=check_errors)
        mark()
        if stats is not None:
            stats.update(world=self.world, rank=self.rank,
                         backend=dist.get_backend(self.group) if dist.is_initialized() else "none",
                         local_ms=(clk[1] - clk[0]) * 1e3)
        if self.world == 1:
            return self.local
        if L > 32:
            self._exchange_words()
            return self.local
        # the other owners' regions as 16-B records (the rank's own part stays in its table)
        rec, parts = self.local.pack_ranges(self.world, skip=self.rank, first_base=base_index)
        mark()
        # the table's overflow word rides along the exchange's one host sync
        recv, rsizes, rbases, ovf = exchange_packed(rec, parts, base_index, group=self.group,
                                                     extra=self.local.overflow_word())
        mark()
        if ovf[0]:
            raise RuntimeError("counter pack overflow (a count or first index past 32 bits, or the table)")
        runs, pos = [], 0
        for src, n in enumerate(rsizes):
            if n:
                runs.append((pos, pos + n, rbases[src]))
            pos += n
        self.local.merge_packed(recv, runs, self.rank, self.world, L)
        mark()
        if stats is not None:
            sent = int(parts.to(torch.int64).sum().item()) - int(parts[self.rank].item() if parts.numel() > self.rank else 0)
            stats.update(pack_ms=(clk[2] - clk[1]) * 1e3, a2a_ms=(clk[3] - clk[2]) * 1e3,
                         merge_ms=(clk[4] - clk[3]) * 1e3, records_sent=sent, bytes_sent=16 * sent,
                         records_received=int(sum(rsizes)), bytes_received=16 * int(sum(rsizes)))
        return self.local

    def _exchange_words(self) -> None:
        """Multi-word keys: the other owners' rows (W words, count, first) out in one all-to-all, the
        received rows folded into this rank's table (merge_words).  An overflowed table is checked
        before anything is extracted, and every overflow is agreed across the ranks (the size
        exchange's flag, then one all_reduce after the merge), so all ranks raise together."""
        ovf = bool(self.local.overflowed())
        if ovf:
            W = max(1, (int(self.L) + 31) // 32)
            send, sizes = torch.empty((0, W + 2), dtype=torch.int64, device=self.device), [0] * self.world
        else:
            _fps, _lens, words, counts, first, parts = self.local.extract_words(self.world)
            pc = [int(x) for x in parts.cpu().tolist()]
            starts = np.cumsum([0] + pc).tolist()
            a, b = starts[self.rank], starts[self.rank + 1]
            W = words.shape[1]
            rows = torch.cat([words[:starts[-1]], counts[:starts[-1], None], first[:starts[-1], None]], 1)
            send = torch.cat([rows[:a], rows[b:]], 0)                      # this rank's own part stays
            sizes = list(pc)
            sizes[self.rank] = 0
        recv, _rs, flag = exchange_rows(send, sizes, group=self.group, flag=int(ovf))
        if flag:
            raise RuntimeError("counter table overflow (a count or first index past 32 bits, or the table)")
        if recv.shape[0]:
            self.local.merge_words(recv[:, :W].contiguous(), recv[:, W].contiguous(), recv[:, W + 1].contiguous())
        if agree_flag(int(bool(self.local.overflowed())), self.device, self.group):
            raise RuntimeError("counter table overflow (a count or first index past 32 bits, or the table)")

    def owned(self):
        return self.local

    def owned_items(self):
        """(keys, counts, first) of the regions this rank owns, on its device (keys: words [m, W] for
        keys longer than 32 nt)."""
        if self.L is not None and self.L > 32:
            _fps, _lens, words, counts, first, parts = self.local.extract_words(self.world)
            starts = [0] + np.cumsum(parts.cpu().numpy()).tolist()
            a, b = int(starts[self.rank]), int(starts[self.rank + 1])
            return words[a:b], counts[a:b], first[a:b]
        if self.world == 1:
            keys, _l, counts, first, parts = self.local.extract(n_parts=1)
            m = int(parts.sum().item())
            return keys[:m], counts[:m], first[:m]
        keys, _l, counts, first, parts = self.local.extract_ranges(self.world)
        starts = [0] + np.cumsum(parts.cpu().numpy()).tolist()
        a, b = int(starts[self.rank]), int(starts[self.rank + 1])
        return keys[a:b], counts[a:b], first[a:b]

    def gather_items(self, dst: int = 0):
        """All owners' entries on rank `dst`, sorted by first occurrence: (keys u64, counts, first)
        as numpy arrays on dst, None elsewhere."""
        k, c, f = self.owned_items()
        if k.dim() == 2:                     # multi-word keys: rows of (W words, count, first)
            if self.world > 1:
                sizes = [0] * self.world
                sizes[dst] = k.shape[0]
                W = k.shape[1]
                rows, _, _f = exchange_rows(torch.cat([k, c[:, None], f[:, None]], 1), sizes, group=self.group)
                k, c, f = rows[:, :W], rows[:, W], rows[:, W + 1]
            if self.rank != dst:
                return None
            kk = k.cpu().numpy().view(np.uint64)
            cc = c.cpu().numpy()
            ff = f.cpu().numpy()
            o = np.argsort(ff, kind="stable")
            return kk[o], cc[o], ff[o]
        if self.world > 1:
            # a merge that overflowed a rank's table: every rank raises before the gather
            if agree_flag(int(bool(self.local.overflowed())), self.device, self.group):
                raise RuntimeError("counter table overflow after the merge (a count or first index past 32 bits)")
            sizes = torch.zeros(self.world, dtype=torch.int64, device=self.device)
            sizes[dst] = k.numel()
            k, c, f = exchange(k, c, f, sizes, self.group)
        if self.rank != dst:
            return None
        kk = k.cpu().numpy().view(np.uint64)
        cc = c.cpu().numpy()
        ff = f.cpu().numpy()
        o = np.argsort(ff, kind="stable")
        return kk[o], cc[o], ff[o]
