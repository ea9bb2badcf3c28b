"""Sharded counter on the GPU with 2 ranks sharing one device (gloo exchange staged through host
memory; on a multi-GPU node the same code runs over RCCL).  Real HBM tables, real kernels; result
checked against the oracle over the whole read stream."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, n, L, U, q):
    sys.path[:0] = [REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import shortseq_amd.batch as B
        from shortseq_amd.dist import ShardedCounter, owner_of_region_np
        dev = torch.device("cuda", 0)
        per = n // world
        ascii = B.synth_pool_reads(per, L, 5, 6, U, i0=rank * per, device=dev)
        sc = ShardedCounter(1 << 16, device=dev)
        sc.count(ascii, L, base_index=rank * per)
        keys, _c, _f = sc.owned_items()
        own = owner_of_region_np(keys.cpu().numpy().view(np.uint64), world, *sc.local.geometry())
        assert (own == rank).all()
        res = sc.gather_items(dst=0)
        sc.close()
        if rank == 0:
            q.put([np.asarray(x).tolist() for x in res])
    finally:
        dist.destroy_process_group()


def test_sharded_counter_two_ranks_one_gpu(oracle):
    n, L, U = 200_000, 32, 3000
    world = 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, L, U, q)) for r in range(world)]
    for p in procs:
        p.start()
    keys, counts, first = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    a = oracle.gen_pool_reads(5, 6, U, 0, n, L)
    exp = oracle.count([a[i * L:(i + 1) * L].tobytes() for i in range(n)])
    assert [int(k) for k in keys] == [w[0] for (w, _L, _c, _f) in exp]
    assert counts == [c for (_w, _L, c, _f) in exp]
    assert first == [f for (_w, _L, _c, f) in exp]
