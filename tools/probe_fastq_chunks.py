#!/usr/bin/env python3
"""a18 (read_and_count_fastq) by chunk size: with the reader ring, chunk k + 1's file reads and H2D
copies run beside chunk k's device index and count, so a file of several chunks overlaps the two.
Files: the bench's 528-MB small-RNA-like FASTQ and the same pool written 4x as long (2.1 GB).
Every setting runs in the same process, interleaved, median of `reps` calls; each dict is checked
against the single-chunk one.

    python tools/probe_fastq_chunks.py [reps=5] [chunk MB list, 0 = default] [file multiples]
"""
import contextlib
import io
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
import probe_fastq_e2e as P  # noqa: E402
import shortseq_amd as sq  # noqa: E402
from shortseq_amd import _shortseq  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
tmp = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
chunks = [int(c) << 20 for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else \
    [0, 512 << 20, 256 << 20, 128 << 20, 64 << 20]
mults = [int(m) for m in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 4]


def call(path, chunk):
    with contextlib.redirect_stdout(io.StringIO()):
        t0 = time.perf_counter()
        c = sq.read_and_count_fastq(path, device="cuda", _chunk_bytes=chunk)
        t = time.perf_counter() - t0
    st = (_shortseq.fastq_stage_times() or [{}])[0]
    return t, c, st


for mult in mults:
    name = f"{0.528 * mult:.1f}GB"
    path = os.path.join(tmp, f"pool{mult}.fq")
    n = P.write_pool_file(path, reps=128 * mult)
    ref = None
    ts = {c: [] for c in chunks}
    stages = {}
    for c in chunks:
        call(path, c)                                    # warm (pinned / device buffers of that size)
    for _ in range(reps):
        for c in chunks:
            t, d, st = call(path, c)
            ts[c].append(t)
            stages[c] = st
            if ref is None:
                ref = list(d.items())
            elif list(d.items()) != ref:
                raise SystemExit(f"PARITY FAILURE: chunk {c} dict differs")
            del d
    assert len(ref) == 65536 and sum(v for _, v in ref) == n
    for c in chunks:
        st = stages[c]
        sp = " ".join(f"{k[:-3]} {st[k]:.1f}" for k in ("read_ms", "h2d_dev_ms", "index_ms", "count_ms", "finish_ms",
                                                         "reduce_and_dict_ms") if k in st)
        print(f"{name} chunk {c >> 20 if c else 'default':>7} MB: {np.median(ts[c]) * 1e3:7.1f} ms "
              f"(min {min(ts[c]) * 1e3:.1f})  [{sp}]", flush=True)
    os.remove(path)
