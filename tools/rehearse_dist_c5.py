#!/usr/bin/env python3
"""Multi-rank C5 rehearsal on one GPU (gloo, every rank on cuda:0), with a timestamped line per phase:
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
      tools/rehearse_dist_c5.py [n_per_rank] [U_log2 ...]
Counts n reads per rank from a pool of 2^U (uniform), runs the exchange, gathers to rank 0 and checks
the total (and the job digest when tests/golden/c5_digests.json has one)."""
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
T0 = time.time()


def log(*a):
    print(f"[{time.time() - T0:7.1f}s r{os.environ.get('RANK', '0')}]", *a, flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
    ulogs = [int(x) for x in sys.argv[2:]] or [20, 24]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import shortseq_amd.batch as B
    from shortseq_amd.dist import ShardedCounter
    for ul in ulogs:
        U = 1 << ul
        i0 = rank * n
        log(f"U=2^{ul}: synth {n} reads")
        a = B.synth_pool_reads(n, 32, 5, 77, U, i0=i0, device=dev)
        sc = ShardedCounter(2 * U, device=dev)
        for step in range(3):
            torch.cuda.synchronize()
            t = time.time()
            sc.count(a, 32, base_index=i0, check_errors=False)
            torch.cuda.synchronize()
            log(f"U=2^{ul}: count step {step} {1e3 * (time.time() - t):.1f} ms")
        del a
        res = sc.gather_items(dst=0)
        log(f"U=2^{ul}: gathered")
        sc.close()
        if rank == 0:
            k, c, f = res
            assert int(c.sum()) == n * world, (int(c.sum()), n * world)
            log(f"U=2^{ul}: unique {len(k)} total ok")
        dist.barrier()
    dist.destroy_process_group()
    log("DONE")


if __name__ == "__main__":
    main()
