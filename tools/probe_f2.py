#!/usr/bin/env python3
"""f2 engine probe: where the device-fed drop-in engine's wall time goes on the bench's ragged
workload (50M reads of 50-150 nt): count (ss_ingest_add_device) vs results (ss_ingest_finish + copy
back), per rep.  Run under `rocprofv3 --kernel-trace --stats` to set the kernel time beside it.

    python tools/probe_f2.py [reps] [n] [Lmin] [Lmax] [log2 pool]     (default 4 50000000 50 150 20)
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import shortseq_amd.batch as B  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000_000
    lo = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    hi = int(sys.argv[4]) if len(sys.argv) > 4 else 150
    U = 1 << (int(sys.argv[5]) if len(sys.argv) > 5 else 20)
    dev = torch.device("cuda", 0)
    blob, offs, lens = B.synth_ragged_pool_reads(n, 41, 42, U, lo, hi, device=dev)
    eng = B.DeviceIngest(dev)
    tot = []
    for r in range(reps):
        eng.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.count(blob, offs, lens)
        t1 = time.perf_counter()
        gl, _gc, _gw = eng.results(copy=False)     # the pinned result buffers, as bench.py's f2 line
        t2 = time.perf_counter()
        if r:
            tot.append((t1 - t0, t2 - t1, t2 - t0))
        print(f"rep {r}: count {1e3 * (t1 - t0):.2f} ms  results {1e3 * (t2 - t1):.2f} ms  total {1e3 * (t2 - t0):.2f} ms  rows {len(gl)}",
              flush=True)
    eng.close()
    if tot:
        import statistics
        m = [statistics.median(x[k] for x in tot) * 1e3 for k in range(3)]
        print(f"median of reps 1..: count {m[0]:.3f} ms  results {m[1]:.3f} ms  total {m[2]:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
