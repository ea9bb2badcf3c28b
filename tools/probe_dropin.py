#!/usr/bin/env python3
"""Drop-in batch path timings (C1 lists, a18 FASTQ) through the C-ABI engine, no torch imported:
ShortSeqCounter(list) on 1M x 32-nt reads (all unique, and a 2^14 pool) and read_and_count_fastq on
the 528-MB small-RNA-like file; medians of 3 after a warm call.  Run under rocprofv3 --kernel-trace
to list every kernel the drop-in launches."""
import contextlib
import io
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import oracle  # noqa: E402  (the generator only)
import probe_fastq_e2e as P  # noqa: E402
import shortseq_amd as sq  # noqa: E402


def med(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2], r


n = 1_000_000
a = oracle.gen_reads(11, 0, n, 32)
reads = [a[i * 32:(i + 1) * 32].tobytes() for i in range(n)]
t, c = med(lambda: sq.ShortSeqCounter(reads, device="cuda"))
print(f"C1 all-unique: {t * 1e3:.1f} ms, {n / t / 1e6:.1f} M reads/s, {len(c)} keys", flush=True)
pa = oracle.gen_pool_reads(12, 13, 1 << 14, 0, n, 32)
preads = [pa[i * 32:(i + 1) * 32].tobytes() for i in range(n)]
t, c = med(lambda: sq.ShortSeqCounter(preads, device="cuda"))
print(f"C1 pool 2^14: {t * 1e3:.1f} ms, {n / t / 1e6:.1f} M reads/s, {len(c)} keys", flush=True)
d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
path = os.path.join(d, "smallrna.fq")
nrec = P.write_pool_file(path)
with contextlib.redirect_stdout(io.StringIO()):
    t, c = med(lambda: sq.read_and_count_fastq(path, device="cuda"))
print(f"a18 small-RNA FASTQ: {t * 1e3:.1f} ms, {nrec / t / 1e6:.1f} M records/s, {len(c)} keys", flush=True)
os.remove(path)
print("torch imported:", "torch" in sys.modules)
