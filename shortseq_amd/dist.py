"""Sharded ShortSeqCounter across GPUs: one process per GPU, torch.distributed.

  1. each rank counts its contiguous shard of the read stream in its own HBM table
     (GpuCounter.insert: fused encode + hash + atomic count + first-occurrence index);
  2. the table is compacted and partitioned by owner = hash(key) % world (GpuCounter.extract);
  3. ONE exchange step: all_to_all_single of the per-owner sizes, then of the (key, count, first)
     triples — RCCL over xGMI on MI355X (backend "nccl"), gloo in the CPU tests;
  4. each owner merges what it received (GpuCounter.merge: counts add, first index = min).
The result is the union of disjoint owner tables; gather_items() brings it to one rank in
first-occurrence order (the reference dict's insertion order, counter.pyx:41-54).

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


def exchange(keys: torch.Tensor, counts: torch.Tensor, first: torch.Tensor, part_counts: torch.Tensor,
             group=None):
    """All-to-all of owner-grouped (key, count, first) int64 triples.

    keys/counts/first: entries grouped by destination rank, part_counts[r] of them for rank r (in
    rank order).  Returns the (keys, counts, first) this rank owns, concatenated in source-rank order.
    Works on any backend whose all_to_all_single supports uneven splits (nccl/RCCL, gloo)."""
    world = dist.get_world_size(group)
    dev = keys.device
    if dev.type != "cpu" and dist.get_backend(group) == "gloo":
        # rehearsal / CPU-collective path: gloo moves host tensors only
        k, c, f = exchange(keys.cpu(), counts.cpu(), first.cpu(), part_counts.cpu(), group)
        return k.to(dev), c.to(dev), f.to(dev)
    sc = part_counts.to(torch.int64)
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rc, sc, group=group)
    sc_l = [int(x) for x in sc.tolist()]
    rc_l = [int(x) for x in rc.tolist()]
    m = sum(sc_l)
    send = torch.stack([keys[:m], counts[:m], first[:m]], 1).contiguous()
    recv = torch.empty((sum(rc_l), 3), dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv, send, output_split_sizes=rc_l, input_split_sizes=sc_l, group=group)
    return recv[:, 0].contiguous(), recv[:, 1].contiguous(), recv[:, 2].contiguous()


class ShardedCounter:
    """Per-rank handle: a local table and (for world > 1) an owner table, reused across batches."""

    def __init__(self, capacity: int, device=None, group=None, table_factory=None):
        """table_factory(capacity, device) builds the per-rank tables; default GpuCounter (HBM).
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
        self.owner = table_factory(capacity, device=self.device) if self.world > 1 else None
        self.L: Optional[int] = None

    def close(self) -> None:
        self.local.close()
        if self.owner is not None:
            self.owner.close()

    def count(self, ascii_local: torch.Tensor, L: int, base_index: int, check_errors: bool = True):
        """Count this rank's shard (global read indices base_index ...) and run the exchange.
        Returns the table this rank owns afterwards (a GpuCounter)."""
        self.L = L
        self.local.reset()
        self.local.insert(ascii_local, L, base_index=base_index, check_errors=check_errors)
        if self.world == 1:
            return self.local
        keys, _lens, counts, first, parts = self.local.extract(n_parts=self.world)
        rk, rc, rf = exchange(keys, counts, first, parts, self.group)
        self.owner.reset()
        self.owner.merge(rk, rc, rf, L)
        return self.owner

    def owned(self):
        return self.owner if self.world > 1 else self.local

    def gather_items(self, dst: int = 0):
        """All owners' entries on rank `dst`, sorted by first occurrence: (keys u64, counts, first)
        as numpy arrays on dst, None elsewhere."""
        t = self.owned()
        keys, _lens, counts, first, parts = t.extract(n_parts=1)
        m = int(parts.sum().item())
        if self.world == 1:
            k, c, f = keys[:m], counts[:m], first[:m]
        else:
            sizes = torch.zeros(self.world, dtype=torch.int64, device=self.device)
            sizes[dst] = m
            k, c, f = exchange(keys, counts, first, sizes, self.group)
        if self.rank != dst:
            return None
        kk = k.cpu().numpy().view(np.uint64)
        cc = c.cpu().numpy()
        ff = f.cpu().numpy()
        o = np.argsort(ff, kind="stable")
        return kk[o], cc[o], ff[o]
