#!/usr/bin/env python3
"""Throughput of the §8(f) kernels on one MI355X (device-resident inputs, HIP-event timing):
FASTQ index (ss_fastq_scan + ss_fastq_index), row gather, batch slice, all-pairs hamming.

    python tools/perf_extras.py [--reps 20]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd._native import check, lib  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def synth_fastq(n_rec, L, dev, seed=1):
    """Device FASTQ text: n_rec records, read length L, headers of 20-40 bytes (built from numpy
    templates on the host, ~1/16 of the records, tiled on the device)."""
    rng = np.random.default_rng(seed)
    m = min(n_rec, 1 << 16)
    parts = []
    for i in range(m):
        seq = rng.choice(np.frombuffer(b"ACGT", np.uint8), L).tobytes()
        hdr = b"@SYN:%08d:" % i + b"x" * int(rng.integers(8, 28))
        parts.append(hdr + b"\n" + seq + b"\n+\n" + b"I" * L + b"\n")
    block = np.frombuffer(b"".join(parts), np.uint8)
    reps = (n_rec + m - 1) // m
    t = torch.from_numpy(block).to(dev).repeat(reps)
    return t, m * reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L_ = lib()
    s = torch.cuda.current_stream(dev).cuda_stream

    # FASTQ index: 8M records of 100 nt (~2 GB)
    buf, nrec = synth_fastq(8 << 20, 100, dev)
    nbytes = buf.numel()
    ws_bytes = int(L_.ss_fastq_scan_ws_bytes(nbytes))
    ws = torch.empty((ws_bytes + 7) // 8, dtype=torch.int64, device=dev)
    cnt = torch.empty(2, dtype=torch.int64, device=dev)
    offs = torch.empty(nrec + 2, dtype=torch.int64, device=dev)
    lens = torch.empty(nrec + 2, dtype=torch.int32, device=dev)
    aux = torch.empty(nrec + 2, dtype=torch.int64, device=dev)

    def scan():
        check(L_.ss_fastq_scan(buf.data_ptr(), nbytes, ws.data_ptr(), ws_bytes, cnt.data_ptr(), s), "scan")

    def index():
        check(L_.ss_fastq_index(buf.data_ptr(), nbytes, 0, 1, ws.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                aux.data_ptr(), nrec + 2, cnt[1:].data_ptr(), s), "index")
    scan()
    index()
    torch.cuda.synchronize()
    assert int(cnt[1]) == nrec, (int(cnt[1]), nrec)
    assert int(lens[:nrec].min()) == 100 and int(lens[:nrec].max()) == 100
    ts = timed(scan, args.reps)
    ti = timed(index, args.reps)
    print(f"fastq: {nbytes / 1e9:.2f} GB, {nrec} records: scan {ts:.3f} ms ({nbytes / ts / 1e6:.0f} GB/s), "
          f"index {ti:.3f} ms ({nbytes / ti / 1e6:.0f} GB/s), total {nbytes / (ts + ti) / 1e6:.0f} GB/s of file, "
          f"{nrec / (ts + ti) / 1e6:.0f} G records/s", flush=True)

    # ragged encode straight from the FASTQ text (ss_encode_var on the index's offsets / lengths)
    o = offs[:nrec]
    ln = lens[:nrec]
    words_v = torch.empty((nrec, 4), dtype=torch.int64, device=dev)
    fbv = torch.empty(1, dtype=torch.int64, device=dev)
    tv = timed(lambda: check(L_.ss_encode_var(buf.data_ptr(), o.data_ptr(), ln.data_ptr(), nrec, words_v.data_ptr(), 4,
                                              fbv.data_ptr(), s), "encode_var"), args.reps)
    gbv = nrec * (100 + 32 + 12) / 1e9
    print(f"encode_var: {nrec} x 100 nt in FASTQ text: {tv:.3f} ms, {gbv / tv * 1e3:.0f} GB/s algorithmic "
          f"({nrec * 100 / tv / 1e9:.2f} T nt/s)", flush=True)
    del words_v

    # gather the 100-nt rows densely (stride 112)
    o = offs[:nrec]
    dense = torch.empty((nrec, 112), dtype=torch.uint8, device=dev)
    tg = timed(lambda: B.gather_rows(buf, o, 100, src_bytes=nbytes, out=dense), args.reps)
    gb = nrec * (100 + 112 + 8) / 1e9
    print(f"gather: {nrec} x 100 nt -> stride 112: {tg:.3f} ms, {gb / tg * 1e3:.0f} GB/s algorithmic", flush=True)
    del dense, aux, lens, offs, buf

    # slice: 50M x 150 nt (5 words) -> [10:110) (4 words)
    n, L = 50_000_000, 150
    words = torch.randint(-(1 << 62), 1 << 62, (n, 5), dtype=torch.int64, device=dev)
    out = torch.empty((n, 4), dtype=torch.int64, device=dev)
    tsl = timed(lambda: B.slice_fixed(words, L, 10, 110, out=out), args.reps)
    print(f"slice: {n} x 150 nt [10:110): {tsl:.3f} ms, {n * 72 / tsl / 1e6:.0f} GB/s algorithmic", flush=True)
    del words, out

    # all pairs: 100k UMIs of 12 nt, k = 1
    for n, L, k in ((100_000, 12, 1), (200_000, 12, 1), (50_000, 32, 2), (20_000, 96, 3)):
        w = B.encode(B.synth_reads(n, L, seed=7, device=dev), L)
        cnt_t = torch.empty(n, dtype=torch.int32, device=dev)
        tot = torch.empty(1, dtype=torch.int64, device=dev)

        def ap():
            check(L_.ss_hamming_all_pairs(w.data_ptr(), n, L, w.shape[1], k, cnt_t.data_ptr(), None, 0,
                                          tot.data_ptr(), s), "allpairs")
        ta = timed(ap, max(3, args.reps // 4))
        pairs = n * (n - 1) / 2
        print(f"all-pairs: n {n} L {L} k {k}: {ta:.3f} ms, {pairs / ta / 1e9:.2f} T pairs/s, "
              f"hits {int(tot.item())}", flush=True)


if __name__ == "__main__":
    main()
