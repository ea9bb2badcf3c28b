#!/usr/bin/env python3
"""TEST / BASELINE INFRASTRUCTURE ONLY — run in THIS container (never on the GPU box, where the
reference is absent): calibrates oracle/libcpubaseline.so (the CPU "port" bench.py times on the box)
against the reference's own compiled kernels (oracle/_ref, built by oracle/build_ref.sh), 1 core,
same process, same inputs; and measures the reference's Python API (C1: sq.pack / ShortSeqCounter,
a18: read_and_count_fastq) here, so bench.py can report those numbers labelled as container-measured.

    python3 oracle/calibrate_cpu_baseline.py   ->  profiles/r3/cpu_baseline_calibration.json

The process is pinned to one core; each kernel ratio is the median of ROUNDS interleaved rounds
(reference, then port, best of 3 each), and the speeds reported beside it are the ones of that
median round (not independently minimised), with the spread of all rounds.
"""
import contextlib
import io
import json
import os
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import cpu_baseline as cb  # noqa: E402
import oracle  # noqa: E402


def best_of(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


ROUNDS = 9


def main():
    assert oracle.ref_available(), "build the reference first (oracle/build_ref.sh)"
    core = sorted(os.sched_getaffinity(0))[-1]
    os.sched_setaffinity(0, {core})
    out = {"cpu": cb.cpu_model(), "nproc": os.cpu_count(), "pinned_core": core, "rounds": ROUNDS,
           "note": "1 pinned core, same process and inputs; ratio = port / reference (1.0 = same speed); "
                   "speeds are those of the median-ratio round"}
    p64, par = oracle.ref_kernel_ptrs()
    # this container's CPU timings wander between runs (a shared host): ROUNDS rounds, reference
    # and port interleaved; the median round is reported with the spread of all rounds
    for L, n in ((32, 4_000_000), (96, 1_500_000), (512, 300_000)):
        a = oracle.gen_reads(1, 0, n, L)
        wpr = max(1, (L + 31) // 32)
        words = np.zeros(n * wpr, np.uint64)
        ref_out = oracle.ref_encode_batch(a, n, L)
        cb.lib(1).cb_encode(a.ctypes.data, n, L, words.ctypes.data, wpr, 1)
        assert np.array_equal(ref_out.reshape(-1), words)
        rounds = []
        for _ in range(ROUNDS):
            t_ref = best_of(lambda: oracle.ref_encode_batch(a, n, L), reps=3)
            t_port = best_of(lambda: cb.lib(1).cb_encode(a.ctypes.data, n, L, words.ctypes.data, wpr, 1), reps=3)
            rounds.append((t_ref / t_port, t_ref, t_port))
        rounds.sort()
        med, t_ref, t_port = rounds[len(rounds) // 2]
        out[f"encode_{L}"] = {"reference_nt_per_s": n * L / t_ref, "port_nt_per_s": n * L / t_port,
                              "ratio": med, "ratio_min": rounds[0][0], "ratio_max": rounds[-1][0],
                              "ratio_rounds": [r[0] for r in rounds],
                              "kernel": "_marshall_bytes_64" if L <= 32 else "_marshall_bytes_array"}
        print(L, out[f"encode_{L}"], flush=True)
    sys.path.insert(0, oracle.REF_DIR)
    import shortseq.counter as ref_counter  # the reference, built from its sources (oracle/_ref)
    import shortseq.short_seq as ref_sq
    # counter: the reference ShortSeqCounter (dict of ShortSeq objects) vs the port's unordered_map
    n, U = 2_000_000, 1 << 24
    a = oracle.gen_pool_reads(5, 77, U, 0, n, 32)
    reads = [a[i * 32:(i + 1) * 32].tobytes() for i in range(n)]
    t_ref = best_of(lambda: ref_counter.ShortSeqCounter(reads), reps=3)
    import ctypes as C
    tot, fs = C.c_uint64(), C.c_uint64()
    t_port = best_of(lambda: cb.lib(1).cb_count(a.ctypes.data, n, 32, 1, C.byref(tot), C.byref(fs)), reps=3)
    out["counter_32_pool2^24"] = {"reads": n, "reference_reads_per_s": n / t_ref, "port_reads_per_s": n / t_port,
                                  "ratio": t_ref / t_port,
                                  "note": "reference: ShortSeqCounter(list of bytes) incl. object creation; "
                                          "port: encode + std::unordered_map on the packed word"}
    print(out["counter_32_pool2^24"], flush=True)
    # C3' (hamming on packed objects): the reference's hamming has no batch kernel to call -- the
    # XOR-collapse-popcount loop is inlined in each __xor__ dunder -- so its own number is the
    # per-object Python API (a ^ b over pre-built objects), beside the port's batch loop
    for L, n in ((32, 1_000_000), (96, 1_000_000), (512, 300_000)):
        a = oracle.gen_reads(6, 0, n, L)
        objs = [ref_sq.pack(a[i * L:(i + 1) * L].tobytes()) for i in range(n)]
        r0 = objs[0]
        t_ref = best_of(lambda: [r0 ^ o for o in objs], reps=3)
        pr = cb.bench_hamming_only(L, n, 1, 1.0)
        out[f"hamming_{L}"] = {"reference_api_pairs_per_s": n / t_ref, "port_pairs_per_s": pr["pairs_per_s"],
                               "note": "reference: r0 ^ obj per object (Python API; no batch kernel exists); "
                                       "port: the same loop over a packed batch (oracle/cpu_baseline.cpp cb_hamming_ref)"}
        print(out[f"hamming_{L}"], flush=True)
    # C1 (BASELINE configs[0]): the reference's own Python API on 1M x 32-nt reads, as bench.py's
    # C1 drop-in line measures the drop-in (median of 3)
    n = 1_000_000
    a = oracle.gen_reads(11, 0, n, 32)
    reads = [a[i * 32:(i + 1) * 32].tobytes() for i in range(n)]
    med = lambda fn: float(np.median([best_of(fn, reps=1) for _ in range(3)]))  # noqa: E731
    pa = oracle.gen_pool_reads(12, 13, 1 << 14, 0, n, 32)
    preads = [pa[i * 32:(i + 1) * 32].tobytes() for i in range(n)]
    out["C1_reference_api"] = {"pack_per_s": n / med(lambda: [ref_sq.pack(r) for r in reads]),
                               "counter_reads_per_s": n / med(lambda: ref_counter.ShortSeqCounter(reads)),
                               "counter_pool16k_reads_per_s": n / med(lambda: ref_counter.ShortSeqCounter(preads)),
                               "sample": "1M x 32-nt reads (seed 11; pool: 2^14 items, seeds 12/13), median of 3"}
    print(out["C1_reference_api"], flush=True)
    # a18: the reference's read_and_count_fastq on the small-RNA-like file bench.py uses
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import probe_fastq_e2e as P
    d = tempfile.mkdtemp()
    path = os.path.join(d, "smallrna.fq")
    nrec = P.write_pool_file(path)
    with contextlib.redirect_stdout(io.StringIO()):
        t = med(lambda: ref_counter.read_and_count_fastq(path))
    out["a18_reference_read_and_count_fastq"] = {"records": nrec, "file_bytes": os.path.getsize(path),
                                                 "s_per_call": t, "records_per_s": nrec / t}
    print(out["a18_reference_read_and_count_fastq"], flush=True)
    os.remove(path)
    os.makedirs(os.path.join(REPO, "profiles", "r3"), exist_ok=True)
    with open(os.path.join(REPO, "profiles", "r3", "cpu_baseline_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
