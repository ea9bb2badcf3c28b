#!/usr/bin/env python3
"""One-GPU rehearsal of the multi-device drop-in reduce: D engines on device 0
count consecutive shards of one read stream (ShortSeqCounter(list, device=[...]) shards the same
way), then either
  old: every engine finishes and ships ALL of its distinct rows to the host, where the dict is
       merged shard by shard (a key in k shards crosses PCIe k times and takes k dict probes);
  new: every engine exports, the others fold into engine 0 on the devices (ss_ingest_merge), and
       engine 0 alone finishes: each distinct key crosses PCIe once and gets one dict insert.
Reports per-phase wall times, the rows each way sends to the host, and the host dict build of the
new way's rows (Cython _fill_from_arrays, the drop-in's own loop).  Unmeasured on hardware across
real devices: here the peer copies are same-device copies.

    python tools/probe_merge.py [log2_U] [engines] [reads_per_key]
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd import ShortSeqCounter  # noqa: E402
from shortseq_amd import _shortseq as S  # noqa: E402


def main():
    lu = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    D = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    per_key = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    U = 1 << lu
    n = per_key * U
    L = 32
    dev = torch.device("cuda", 0)
    ascii = B.synth_pool_reads(n, L, 11, 12, U, device=dev)
    blob = ascii.view(-1)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * L
    lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    cuts = [n * k // D for k in range(D + 1)]
    torch.cuda.synchronize()
    print(f"U=2^{lu} engines={D} reads={n} ({per_key} per key)", flush=True)
    for rep in range(2):
        for way in ("old", "new"):
            engs = [B.DeviceIngest(dev) for _ in range(D)]
            try:
                t0 = time.perf_counter()
                for k, e in enumerate(engs):
                    e.count(blob, offs[cuts[k]:cuts[k + 1]], lens[cuts[k]:cuts[k + 1]])
                t1 = time.perf_counter()
                if way == "old":
                    rows = 0
                    for e in engs:
                        gl, _gc, _gw = e.results(copy=False)
                        rows += len(gl)
                    t2 = time.perf_counter()
                    print(f"rep {rep} old: count {1e3 * (t1 - t0):.1f} ms  finish+D2H of every shard "
                          f"{1e3 * (t2 - t1):.1f} ms  rows to host {rows}", flush=True)
                else:
                    for e in engs[1:]:
                        e.export()
                    t2 = time.perf_counter()
                    for k in range(1, D):
                        engs[0].merge(engs[k], cuts[k])
                    t3 = time.perf_counter()
                    gl, gc, gw = engs[0].results(copy=False)
                    t4 = time.perf_counter()
                    c = ShortSeqCounter()
                    S._fill_from_arrays(c, gl, gc, gw)
                    t5 = time.perf_counter()
                    assert len(c) == len(gl) and int(gc.sum()) == n
                    print(f"rep {rep} new: count {1e3 * (t1 - t0):.1f} ms  export {1e3 * (t2 - t1):.1f} ms  "
                          f"device merge {1e3 * (t3 - t2):.1f} ms  finish+D2H {1e3 * (t4 - t3):.1f} ms  "
                          f"rows to host {len(gl)}  host dict build {1e3 * (t5 - t4):.0f} ms", flush=True)
                    del c
            finally:
                for e in engs:
                    e.close()


if __name__ == "__main__":
    main()
