"""Chain vs tree reduce of the multi-device drop-in, rehearsed on one GPU.

D engines (DeviceIngest, all on cuda:0) each count one shard of S device-resident reads; every
shard's keys are distinct (pool 2^40, 32-nt: single-word tables; or --lo/--hi for length classes),
so every export carries ~S keys.  Timed: the exports, then the reduce into engine 0 -- the serial
chain (merge k -> 0 for k = 1..D-1) or the tree (adjacent pairs, each round's merges concurrently
from host threads, round-2+ sources re-exported) -- then engine 0's finish.  Rounds alternate the two
modes.  Unmeasured across real devices: on one GPU a "peer copy" is a device copy.

    python tools/probe_reduce.py [--engines 8] [--shard-log 24] [--rounds 3]
"""
import argparse
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engines", type=int, default=8)
    ap.add_argument("--shard-log", type=int, default=24)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--lo", type=int, default=32)
    ap.add_argument("--hi", type=int, default=32)
    a = ap.parse_args()
    import shortseq_amd.batch as B
    dev = torch.device("cuda", 0)
    D, S = a.engines, 1 << a.shard_log
    n = D * S
    blob, offs, lens = B.synth_ragged_pool_reads(n, 61, 62, 1 << 40, a.lo, a.hi, device=dev)
    engs = [B.DeviceIngest(dev) for _ in range(D)]
    cuts = [k * S for k in range(D + 1)]

    def count_all():
        for k, e in enumerate(engs):
            e.reset()
            e.count(blob, offs[cuts[k]:cuts[k + 1]], lens[cuts[k]:cuts[k + 1]])

    def par(jobs):
        ts = [threading.Thread(target=f, args=x) for f, x in jobs[1:]]
        for t in ts:
            t.start()
        jobs[0][0](*jobs[0][1])
        for t in ts:
            t.join()

    def reduce(mode):
        t0 = time.perf_counter()
        par([(e.export, ()) for e in engs[1:]])       # the shards' exports run in their own threads
        t1 = time.perf_counter()
        from shortseq_amd._native import lib as _lib
        reserve = hasattr(_lib(), "ss_ingest_reserve_merge")     # (an A/B against a build without it)
        if mode == "chain":
            if reserve:
                engs[0].reserve_merge(engs[1:])
            for k in range(1, D):
                engs[0].merge(engs[k], cuts[k])
        else:
            if reserve:
                par([(engs[p].reserve_merge, (engs[p + 1:min(D, p + ((p & -p) or D))],)) for p in range(0, D, 2)])
            step = 1
            while step < D:
                pairs = [(p, p + step) for p in range(0, D, 2 * step) if p + step < D]

                def job(p, q, again):
                    if again:
                        engs[q].export()
                    engs[p].merge(engs[q], cuts[q] - cuts[p])
                par([(job, (p, q, step > 1 and q + 1 < D)) for p, q in pairs])
                step *= 2
        t2 = time.perf_counter()
        lens_, cnts, _w = engs[0].results(copy=False)
        t3 = time.perf_counter()
        # (a 2^40 pool repeats ~n^2 / 2^41 items: distinct keys slightly below n)
        assert len(lens_) > 0.999 * n and int(cnts.sum()) == n, (len(lens_), int(cnts.sum()))
        return (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3

    last = {}
    for r in range(a.rounds + 1):
        for mode in ("chain", "tree"):
            count_all()
            torch.cuda.synchronize()
            ex, mg, fin = reduce(mode)
            last[mode] = mg
            if r:
                print(f"round {r} {mode:5s}: D={D} shard=2^{a.shard_log} L={a.lo}-{a.hi}: export {ex:7.2f} ms, "
                      f"reduce {mg:7.2f} ms, finish {fin:7.2f} ms", flush=True)
    print(f"last round reduce: chain {last['chain']:.2f} ms, tree {last['tree']:.2f} ms", flush=True)
    for e in engs:
        e.close()


if __name__ == "__main__":
    main()
