#!/usr/bin/env python3
"""End-to-end read_and_count_fastq (counter.pyx:57-70): the drop-in's GPU path against the
reference's own function (oracle/_ref, when present) on the same synthetic FASTQ files:

  small-RNA-like: 8.4M records of 18-32 nt (ragged), 65,536 distinct sequences each seen 128 times
  unique-75:      2M records of 75 nt (ShortSeq192), all distinct

Prints wall seconds per call (file read + parse + count + dict), the dict sizes and whether the two
dicts agree."""
import contextlib
import io
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def write_pool_file(path, B=1 << 16, reps=128, lo=18, hi=32, seed=1):
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    parts = []
    for i in range(B):
        L = int(rng.integers(lo, hi + 1))
        seq = acgt[rng.integers(0, 4, L)].tobytes()
        parts.append(b"@p%06d\n" % i + seq + b"\n+\n" + b"I" * L + b"\n")
    block = b"".join(parts)
    with open(path, "wb") as f:
        for _ in range(reps):
            f.write(block)
    return B * reps


def write_unique_file(path, n=2_000_000, L=75, seed=2):
    """Fixed-width records "@r<9 digits>\n<seq>\n+\n<qual>\n", built as one uint8 matrix."""
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    idx = np.arange(n, dtype=np.int64)
    rec = np.empty((n, 16 + 2 * L), np.uint8)
    rec[:, 0] = ord("@")
    rec[:, 1] = ord("r")
    for k in range(9):
        rec[:, 2 + k] = ord("0") + (idx // 10 ** (8 - k)) % 10
    rec[:, 11] = ord("\n")
    rec[:, 12:12 + L] = acgt[rng.integers(0, 4, (n, L))]
    rec[:, 12 + L:15 + L] = np.frombuffer(b"\n+\n", np.uint8)
    rec[:, 15 + L:15 + 2 * L] = ord("I")
    rec[:, 15 + 2 * L] = ord("\n")
    rec.tofile(path)
    return n


def timed(fn, path):
    with contextlib.redirect_stdout(io.StringIO()):
        t0 = time.perf_counter()
        c = fn(path)
        return time.perf_counter() - t0, c


def main():
    import torch
    import oracle
    import shortseq_amd as sq
    ref = None
    if oracle.ref_available():
        sys.path.insert(0, oracle.REF_DIR)
        import shortseq.counter as ref
    tmp = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    cases = [("small-RNA 18-32 nt, 2^16 distinct x 128", os.path.join(tmp, "pool.fq"), write_pool_file),
             ("unique 75 nt", os.path.join(tmp, "uniq.fq"), write_unique_file)]
    out = {}
    for name, path, gen in cases:
        n = gen(path)
        size = os.path.getsize(path)
        timed(lambda p: sq.read_and_count_fastq(p, device="cuda"), path)      # warm (GPU init)
        t_gpu, c_gpu = timed(lambda p: sq.read_and_count_fastq(p, device="cuda"), path)
        torch.cuda.synchronize()
        row = {"records": n, "file_bytes": size, "dropin_gpu_s": t_gpu, "unique": len(c_gpu),
               "dropin_records_per_s": n / t_gpu}
        if ref is not None:
            t_ref, c_ref = timed(ref.read_and_count_fastq, path)
            row.update(reference_s=t_ref, reference_records_per_s=n / t_ref, reference_entries=len(c_ref))
            same = [(str(k), v) for k, v in c_gpu.items()] == [(str(k), v) for k, v in c_ref.items()]
            row["dicts_equal"] = same
            del c_ref
        del c_gpu
        out[name] = row
        print(name, row, flush=True)
        os.remove(path)
    return out


if __name__ == "__main__":
    main()
