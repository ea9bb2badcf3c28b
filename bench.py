#!/usr/bin/env python3
"""Benchmark: batch 2-bit encode on MI355X (BASELINE.json configs[1]: 100M x 32-nt reads, 1 GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one ss_encode_fixed launch over one rank's batch of synthetic reads already resident in
HBM (SURVEY §8(d) generator, generated on the device).  Ranks shard the read stream by contiguous
index ranges (weak scaling, no data-path collective).  `value` = all ranks' nt / max-over-ranks
time.  The same JSON line carries the other BASELINE configs as `extra` (C3 fused encode+hamming,
C4 encode+decode round trip, C5 sharded counter with an RCCL all-to-all merge), the `roofline` of
the dominant kernel (algorithmic bytes / HIP-event kernel time vs 8 TB/s) and the `cpu_baseline`
(the reference's CPU algorithms restated in oracle/cpu_baseline.cpp, timed on 1 host core and on all
usable cores for C2-C5; the reference itself never runs on the GPU box).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

SETTLE_S = 0.1         # untimed clock-settle load before every timed region (see timed_loop)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured float4 copy
I8_PEAK_TOPS = 5000.0  # dense i8 MFMA: 2x the ~2.5 PF bf16 dense peak (MI355X_MICROARCH.md matrix cores)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def compact(x, sig: int = 4, _depth: int = 0):
    """The JSON line the driver keeps is the tail of stdout (~8.8 KB): floats to `sig` significant
    digits, explanatory strings (note / how / where / xgmi, and the kernel names of the extras'
    rooflines) dropped -- DESIGN.md section 5 and section 4 hold them; the headline keeps its kernel."""
    if isinstance(x, float):
        return float(f"{x:.{sig}g}") if x == x else None
    if isinstance(x, dict):
        drop = ("note", "how", "where", "xgmi") + (("kernel",) if _depth > 1 else ())
        return {k: compact(v, sig, _depth + 1) for k, v in x.items() if k not in drop}
    if isinstance(x, (list, tuple)):
        return [compact(v, sig, _depth + 1) for v in x]
    return x


def splitmix64(x: int) -> int:
    M = (1 << 64) - 1
    z = (x + 0x9E3779B97F4A7C15) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def known_words(seed: int, i: int, L: int) -> list:
    """The generator's words for read i = the expected encode output."""
    W = (L + 31) // 32
    out = []
    for w in range(W):
        nb = min(32, L - 32 * w)
        r = splitmix64(seed + i * W + w)
        out.append(r if nb == 32 else r & ((1 << (2 * nb)) - 1))
    return out


class Timer:
    """HIP events on the stream the kernels are launched on (torch's current stream)."""

    def __init__(self):
        self.pairs = []
        self.region_ms = float("nan")

    def __enter__(self):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        self.pairs.append((s, e))
        return self

    def __exit__(self, *exc):
        self.pairs[-1][1].record()

    def mean_ms(self) -> float:
        torch.cuda.synchronize()
        return float(np.mean([s.elapsed_time(e) for s, e in self.pairs]))


def timed_loop(step, steps, warmup, world, on_timed_start=None):
    """W untimed steps, then K steps between barrier + synchronize; returns max-over-ranks seconds
    and a Timer.  The Timer's `region` pair brackets all K steps on the launch stream, so
    region_ms / K is the per-step device time with the launch queue kept full (no host launch
    latency inside the window); per-kernel pairs are recorded by steps that time sub-kernels."""
    for _ in range(warmup):
        step(None)
    torch.cuda.synchronize()
    # clock settle: the MI355X needs ~20-30 ms of sustained load before its clocks stop ramping
    # (tools/tune_stream.hip ramp trace: first ~30 back-to-back 0.6-ms launches 2-6 % slower), so
    # untimed steps continue until SETTLE_S of load has passed, whatever W is
    # With world > 1 the ranks agree on every settle step (a step may hold collectives, e.g. the C5
    # exchange: ranks running different numbers of steps would pair one rank's exchange with another's
    # barrier and hang)
    t_s = time.perf_counter()
    while True:
        more = time.perf_counter() - t_s < SETTLE_S
        if world > 1:
            f = torch.tensor([int(more)], dtype=torch.int32, device="cuda" if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(f, op=dist.ReduceOp.MAX)
            more = bool(f.item())
        if not more:
            break
        step(None)
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if on_timed_start is not None:
        on_timed_start()      # e.g. drop the warmup steps' per-pass timings
    timer = Timer()
    r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    r0.record()
    for _ in range(steps):
        step(timer)
    r1.record()
    torch.cuda.synchronize()
    timer.region_ms = r0.elapsed_time(r1)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el, timer


def check_known_answer(words: torch.Tensor, seed: int, i0: int, L: int, n: int):
    idx = np.unique(np.linspace(0, n - 1, 257).astype(np.int64))
    got = words[torch.from_numpy(idx).to(words.device)].cpu().numpy().view(np.uint64)
    for k, i in enumerate(idx):
        exp = known_words(seed, i0 + int(i), L)
        if [int(x) for x in got[k][: len(exp)]] != exp:
            raise SystemExit(f"PARITY FAILURE: read {i0 + i} L={L}: {got[k]} != {exp}")


def load_traffic(workload: str, reads: int):
    """HBM bytes per launch from the committed PMC summary (profiles/pmc_traffic.json, written by
    tools/save_profiles.py from separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench),
    scaled to this launch's read count (the profiled launch's bytes per read x reads)."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            e = json.load(f).get(workload, {})
        per_read = e.get("hbm_bytes_per_read")
        if per_read is None and "hbm_bytes_per_launch" in e and e.get("reads"):
            per_read = e["hbm_bytes_per_launch"] / e["reads"]
        return None if per_read is None else per_read * reads
    except Exception:  # noqa: BLE001
        return None


# ------------------------------------------------------------------------------------------------
def bench_encode(B, lib, dev, rank, world, n, L, steps, warmup, seed=1):
    i0 = rank * n
    ascii = B.synth_reads(n, L, seed=seed, i0=i0, device=dev)
    wpr = B.wpr_for(L)
    words = torch.empty((n, wpr), dtype=torch.int64, device=dev)
    fb = B.first_bad_buffer(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ap, wp, fp = ascii.data_ptr(), words.data_ptr(), fb.data_ptr()

    def step(timer):
        rc = lib.ss_encode_fixed(ap, n, L, L, wp, wpr, fp, stream)
        if rc:
            raise RuntimeError(lib.ss_last_error_string())

    el, timer = timed_loop(step, steps, warmup, world)
    if int(fb.item()) != -1:
        raise SystemExit("PARITY FAILURE: synthetic batch flagged an invalid base")
    check_known_answer(words, seed, i0, L, n)
    del ascii, words
    # every step is exactly one encode launch (the first-bad reset is a 8-byte memset node)
    return el, timer.region_ms / steps


def bench_encode_hamming(B, lib, dev, rank, world, n, L, steps, warmup, seed=2):
    i0 = rank * n
    ascii = B.synth_reads(n, L, seed=seed, i0=i0, device=dev)
    wpr = B.wpr_for(L)
    words = torch.empty((n, wpr), dtype=torch.int64, device=dev)
    dist_out = torch.empty(n, dtype=torch.int32, device=dev)
    ref = torch.empty((1, wpr), dtype=torch.int64, device=dev)
    fb = B.first_bad_buffer(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    # the reference read = read 0 of the batch, packed once (the reference's __xor__ takes an already
    # packed ShortSeq); a step is one fused encode + hamming pass over the batch
    if lib.ss_encode_fixed(ascii.data_ptr(), 1, L, L, ref.data_ptr(), wpr, fb.data_ptr(), stream):
        raise RuntimeError(lib.ss_last_error_string())

    def step(_timer):
        if lib.ss_encode_hamming_ref(ascii.data_ptr(), n, L, L, words.data_ptr(), wpr, ref.data_ptr(),
                                     dist_out.data_ptr(), fb.data_ptr(), stream):
            raise RuntimeError(lib.ss_last_error_string())

    el, timer = timed_loop(step, steps, warmup, world)
    check_known_answer(words, seed, i0, L, n)
    # distances: property check against the packed words (hamming kernel on the stored words)
    d2 = B.hamming_ref(words, L, words[0])
    if not torch.equal(d2, dist_out):
        raise SystemExit("PARITY FAILURE: fused hamming != hamming on packed words")
    del ascii, words, dist_out, d2
    # the timed region holds the K fused launches back to back: region / K is the launch's duration
    return el, timer.region_ms / steps, timer.region_ms / steps


def bench_hamming_only(B, lib, dev, rank, world, n, L, steps, warmup, seed=6):
    """SURVEY §8(d) C3': hamming vs one reference on pre-packed words (ss_hamming_ref, k_ham_dense);
    the words come from a device encode of synthetic reads, the timed step is the hamming launch."""
    i0 = rank * n
    ascii = B.synth_reads(n, L, seed=seed, i0=i0, device=dev)
    words = B.encode(ascii, L)
    del ascii
    ref = words[0].clone()
    out = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    wpr = words.shape[1]
    wp, rp, op = words.data_ptr(), ref.data_ptr(), out.data_ptr()

    def step(timer):
        rc = lib.ss_hamming_ref(wp, n, L, wpr, rp, op, stream)
        if rc:
            raise RuntimeError(lib.ss_last_error_string())

    el, tr = timed_loop(step, steps, warmup, world)
    # parity: distance to read 0 == the fused encode's distance computed against read 0's words
    _, want = B.encode_hamming_ref(B.synth_reads(n, L, seed=seed, i0=i0, device=dev), L, ref, store_words=False)
    if not torch.equal(out, want):
        raise SystemExit(f"PARITY FAILURE: ss_hamming_ref L={L} != fused encode+hamming")
    del words, out, want
    return el, tr.region_ms / steps


def bench_roundtrip(B, lib, dev, rank, world, n, L, steps, warmup, seed=3):
    i0 = rank * n
    ascii = B.synth_reads(n, L, seed=seed, i0=i0, device=dev)
    wpr = B.wpr_for(L)
    words = torch.empty((n, wpr), dtype=torch.int64, device=dev)
    back = torch.empty((n, L), dtype=torch.uint8, device=dev)
    fb = B.first_bad_buffer(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    t_enc, t_dec = Timer(), Timer()

    def step(timer):
        if timer is None:
            rc = lib.ss_encode_fixed(ascii.data_ptr(), n, L, L, words.data_ptr(), wpr, fb.data_ptr(), stream)
            rc |= lib.ss_decode_fixed(words.data_ptr(), n, L, wpr, back.data_ptr(), L, stream)
        else:
            with t_enc:
                rc = lib.ss_encode_fixed(ascii.data_ptr(), n, L, L, words.data_ptr(), wpr, fb.data_ptr(), stream)
            with t_dec:
                rc |= lib.ss_decode_fixed(words.data_ptr(), n, L, wpr, back.data_ptr(), L, stream)
        if rc:
            raise RuntimeError(lib.ss_last_error_string())

    el, tr = timed_loop(step, steps, warmup, world)
    if not torch.equal(back, ascii):
        raise SystemExit("PARITY FAILURE: encode -> decode round trip")
    check_known_answer(words, seed, i0, L, n)
    del ascii, words, back
    return el, t_enc.mean_ms(), t_dec.mean_ms(), tr.region_ms / steps


def table_digest(keys, counts, first) -> str:
    """SHA-256 of the (key, count, first) uint64 rows sorted by key (tests/golden/gen_c5_digests.py)."""
    import hashlib
    k = np.asarray(keys, dtype=np.uint64)
    o = np.argsort(k, kind="stable")
    rows = np.stack([k[o], np.asarray(counts, dtype=np.uint64)[o], np.asarray(first, dtype=np.uint64)[o]], 1)
    return hashlib.sha256(np.ascontiguousarray(rows).tobytes()).hexdigest()


def c5_digest_name(U, zipf, world, n):
    """The c5_digests.json entry for this C5 run (125M reads per rank, seeds 5 / 77), or None."""
    if n != 125_000_000:
        return None
    if world == 1:
        return (f"zipf{zipf}" if zipf else "uniform") + f"_U{U.bit_length() - 1}_shard0"
    if not zipf and U == 1 << 24 and world in (2, 4, 8):
        return f"uniform_U24_job{world}"
    return None


def bench_counter(B, lib, dev, rank, world, n, L, U, steps, warmup, seed=5, pool_seed=77, zipf=None):
    """C5: per rank n reads drawn from a pool of U 32-mers (uniform, or Zipf(zipf) when given; shard =
    contiguous read-index range); shortseq_amd.dist.ShardedCounter: local HBM table -> partition by
    owner -> RCCL all-to-all of (key, count, first) -> owners merge."""
    from shortseq_amd.dist import ShardedCounter
    i0 = rank * n
    if zipf:
        ascii = B.synth_zipf_reads(n, L, seed, pool_seed, B.zipf_cdf(U, zipf), i0=i0, device=dev)
    else:
        ascii = B.synth_pool_reads(n, L, seed, pool_seed, U, i0=i0, device=dev)
    cap = 1 << max(10, int(np.ceil(np.log2(2 * U))))
    sc = ShardedCounter(cap, device=dev)

    def step(timer):
        sc.count(ascii, L, base_index=i0, check_errors=False)

    # the headline loop runs the production insert (no per-pass events: ADVICE r4); the per-pass
    # split comes from a separate short run with ss_counter_set_timing on, after it
    el, tr = timed_loop(step, steps, warmup, world)
    sc.local.set_timing(True)
    _el_p, _tr_p = timed_loop(step, max(2, steps // 2), 1, world, on_timed_start=lambda: sc.local.pass_times())
    passes = sc.local.pass_times()
    sc.local.set_timing(False)
    exch = None
    if world > 1:
        # one diagnostic count with the device synchronised around each phase:
        # local count, pack, the two all-to-alls with their host sync, merge; every rank's split
        # gathered to rank 0 as [min, max] per field, with the backend and the world size they saw
        from shortseq_amd.dist import rank_spread
        st = {}
        dist.barrier()
        sc.count(ascii, L, base_index=i0, check_errors=False, stats=st)
        allst = [None] * world
        dist.all_gather_object(allst, st)
        exch = rank_spread(allst)
    del ascii
    # parity after timing: the whole job's table gathered to rank 0 (all owners' regions), its
    # (key, count, first) rows sorted by key hashed and compared with the generator-derived digest of
    # the same job (tests/golden/c5_digests.json) when one exists for this (U, skew, world), else
    # the total count
    res = sc.gather_items(dst=0)
    sc.close()
    uniq, check = 0, "total count"
    if rank == 0:
        keys, counts, first = res
        uniq = len(keys)
        if int(counts.sum()) != n * world:
            raise SystemExit(f"PARITY FAILURE: counter total {int(counts.sum())} != {n * world}")
        name = c5_digest_name(U, zipf, world, n)
        if name is not None:
            with open(os.path.join(REPO, "tests", "golden", "c5_digests.json")) as fh:
                want = json.load(fh)[name]
            if (uniq, table_digest(keys, counts, first)) != (want["unique"], want["digest"]):
                raise SystemExit(f"PARITY FAILURE: counter table != {name}")
            check = f"digest {name}"
    return el, tr.region_ms / steps, uniq, check, passes, exch


def bench_exchange(B, dev, n=125_000_000, U=1 << 24, owners=8, reps=5):
    """The C5 exchange's device cost, rehearsed on one GPU: one rank's 125M-read
    table (pool 2^24) packs the other 7 owners' regions into 16-B records (ss_counter_pack_ranges:
    k_region_scan + k_region_pack), and folds 7 received runs into its own regions
    (ss_counter_merge_packed: k_run_bounds + k_merge_runs) -- the runs are its own part-0 records
    replicated 7 times, the size a peer's shard of the same pool sends.  The xGMI transfer between
    them (RCCL all_to_all_single) is not on one GPU.  Roofline over each step's algorithmic bytes:
    pack = the other owners' slots read (16 B each) + the records written; merge = the records read +
    the owned slices read and written once."""
    ascii = B.synth_pool_reads(n, 32, 5, 77, U, device=dev)
    cap = 1 << int(np.ceil(np.log2(2 * U)))
    gc = B.GpuCounter(cap, device=dev)
    gc.reserve(n)
    gc.insert(ascii, 32, check_errors=False)
    rec_all, parts_all = gc.pack_ranges(owners, skip=-1)
    m0 = int(parts_all[0].item())
    recv = rec_all[:m0].repeat(owners - 1, 1)
    runs = [(k * m0, (k + 1) * m0, 0) for k in range(owners - 1)]
    del rec_all
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    pk, mg = [], []
    for r in range(reps + 1):
        # as in the job, the pack follows an insert, whose aggregate leaves the regions' occupancy
        # fresh (after a merge it is stale and the pack would first recount it: k_region_occ, ~0.1 ms)
        gc.reset()            # (as ShardedCounter.count: a fresh table per count)
        gc.insert(ascii, 32, check_errors=False)
        ev[0].record()
        rec, parts = gc.pack_ranges(owners, skip=0)
        ev[1].record()
        gc.merge_packed(recv, runs, 0, owners, 32)
        ev[2].record()
        torch.cuda.synchronize()
        if r:     # the first round warms up
            pk.append(ev[0].elapsed_time(ev[1]))
            mg.append(ev[1].elapsed_time(ev[2]))
    sent = int(parts.sum().item())
    del ascii
    gc.close()
    pack_ms, merge_ms = float(np.median(pk)), float(np.median(mg))
    pack_b = cap * (owners - 1) // owners * 16 + sent * 16
    merge_b = recv.shape[0] * 16 + cap // owners * 16 * 2
    return {"owners": owners, "reads_per_owner": n, "pool": U, "records_sent": sent, "records_received": recv.shape[0],
            "pack_ms": pack_ms, "merge_ms": merge_ms,
            "roofline": {"bound": "hbm", "kernel": "k_region_scan + k_region_pack | k_run_bounds + k_merge_runs",
                         "pack_frac": pack_b / (pack_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "merge_frac": merge_b / (merge_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "pack_bytes": pack_b, "merge_bytes": merge_b, "peak": HBM_PEAK_GBS, "unit": "GB/s"},
            "xgmi": "not measured (one GPU): RCCL all_to_all_single of records_sent x 16 B per rank"}


def bench_fastq_index(B, lib, dev, n_rec=8 << 20, L=100, reps=10):
    """ss_fastq_scan + ss_fastq_index over a device-resident synthetic FASTQ text
    (n_rec records of L nt, 20-40-byte headers); checks every record's offset/length."""
    from shortseq_amd._native import check
    rng = np.random.default_rng(1)
    m = 1 << 16
    parts = []
    for i in range(m):
        seq = rng.choice(np.frombuffer(b"ACGT", np.uint8), L).tobytes()
        parts.append(b"@SYN:%08d:" % i + b"x" * int(rng.integers(8, 28)) + b"\n" + seq + b"\n+\n" + b"I" * L + b"\n")
    block = np.frombuffer(b"".join(parts), np.uint8).copy()
    reps_blk = n_rec // m
    buf = torch.from_numpy(block).to(dev).repeat(reps_blk)
    nbytes, nrec = buf.numel(), m * reps_blk
    s = torch.cuda.current_stream(dev).cuda_stream
    ws_bytes = int(lib.ss_fastq_scan_ws_bytes(nbytes))
    ws = torch.empty((ws_bytes + 7) // 8, dtype=torch.int64, device=dev)
    ws1_bytes = int(lib.ss_fastq_onepass_ws_bytes(nbytes, nrec + 2))
    ws1 = torch.empty((ws1_bytes + 7) // 8, dtype=torch.int64, device=dev)
    cnt = torch.empty(3, dtype=torch.int64, device=dev)
    offs = torch.empty(nrec + 2, dtype=torch.int64, device=dev)
    lens = torch.empty(nrec + 2, dtype=torch.int32, device=dev)
    aux = torch.empty(nrec + 2, dtype=torch.int64, device=dev)
    starts = torch.from_numpy(np.cumsum([0] + [len(p) for p in parts[:-1]]) + np.array(
        [p.index(b"\n") + 1 for p in parts])).to(dev)

    def twopass(_t):
        check(lib.ss_fastq_scan(buf.data_ptr(), nbytes, ws.data_ptr(), ws_bytes, cnt.data_ptr(), s), "scan")
        check(lib.ss_fastq_index(buf.data_ptr(), nbytes, 0, 1, ws.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                 aux.data_ptr(), nrec + 2, cnt[1:].data_ptr(), s), "index")

    def onepass(_t):
        check(lib.ss_fastq_index_onepass(buf.data_ptr(), nbytes, 0, 1, ws1.data_ptr(), ws1_bytes, offs.data_ptr(),
                                         lens.data_ptr(), aux.data_ptr(), nrec + 2, cnt.data_ptr(), s), "index1")

    def verify(what, nreads):
        if nreads != nrec or int(lens[:nrec].min()) != L or int(lens[:nrec].max()) != L:
            raise SystemExit("PARITY FAILURE: FASTQ index (%s)" % what)
        if not torch.equal(offs[:m], starts) or not torch.equal(offs[nrec - m:nrec] - offs[nrec - m], starts - starts[0]):
            raise SystemExit("PARITY FAILURE: FASTQ offsets (%s)" % what)

    el2, tr2 = timed_loop(twopass, reps, 3, 1)
    verify("two-pass", int(cnt[1]))
    offs.zero_()
    lens.zero_()
    el, tr = timed_loop(onepass, reps, 3, 1)
    if int(cnt[2]) != 0 or int(cnt[0]) != 4 * nrec:
        raise SystemExit("PARITY FAILURE: FASTQ one-pass staging / newline count")
    verify("one-pass", int(cnt[1]))
    ms = tr.region_ms / reps
    # algorithmic bytes: the file once + 12 B per sequence line out (offset u64 +
    # length u32); the kernel's own staging (2 B per line written and read back) is not counted
    algo = nbytes + nrec * 12
    staged = nrec * 4 * 2 * 2
    return {"file_bytes": nbytes, "records": nrec, "read_len": L, "ms_per_step": ms,
            "file_GB_per_s": nbytes / ms / 1e6, "records_per_s": nrec / ms * 1e3,
            "two_pass_ms_per_step": tr2.region_ms / reps,
            "roofline": {"bound": "hbm", "kernel": "k_fq_nlpos + scans + k_fq_place (whole call)",
                         "achieved": algo / ms / 1e6, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": algo / ms / 1e6 / HBM_PEAK_GBS, "algo_bytes_per_step": algo,
                         "frac_with_staging": (algo + staged) / ms / 1e6 / HBM_PEAK_GBS,
                         "traffic": load_traffic("fastq_index_onepass", nrec)},
            "note": "ss_fastq_index_onepass (file read once, newline positions staged per tile); two_pass = ss_fastq_scan + "
                    "ss_fastq_index; device-resident synthetic FASTQ, every offset / length checked"}


def bench_all_pairs(B, lib, dev, n=100_000, L=12, k=1, reps=10, method="tiles", pool=None):
    """all unordered pairs of n UMIs (L nt) within hamming k.  method "tiles" checks
    every pair on the MFMA tiles (priced against the i8 peak); "pigeonhole" / "auto" check only the
    pairs sharing one of k + 1 segments (bucketed on the device) -- same counts and total, reported
    as covered pairs per second (n (n - 1) / 2 per step), with no MFMA roofline."""
    from shortseq_amd._native import check
    code = B.ALL_PAIRS_METHODS[method]
    # pool: reads drawn from `pool` distinct items (duplicates give distance-0 hits), else all random
    a = B.synth_reads(n, L, seed=7, device=dev) if pool is None else B.synth_pool_reads(n, L, 7, 8, pool, device=dev)
    w = B.encode(a, L)
    cnt = torch.empty(n, dtype=torch.int32, device=dev)
    tot = torch.empty(1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream

    def step(_t):
        check(lib.ss_hamming_all_pairs_ex(w.data_ptr(), n, L, w.shape[1], k, cnt.data_ptr(), None, 0,
                                          tot.data_ptr(), code, s), "all_pairs")
    el, tr = timed_loop(step, reps, 2, 1)
    if int(cnt.sum().item()) != 2 * int(tot.item()):
        raise SystemExit("PARITY FAILURE: all-pairs counts")
    ms = tr.region_ms / reps
    pairs = n * (n - 1) // 2
    out = {"n": n, "read_len": L, "max_dist": k, "method": method, "pairs": pairs, "ms_per_step": ms,
           "pairs_per_s": pairs / ms * 1e3, "hits": int(tot.item())}
    if method != "tiles":
        return out
    # issued i8 MACs: one-hot codes, 8 positions (32 MACs) per k-step, ceil(min(L + 1, 32) / 8) steps
    ks = (min(L + 1, 32) + 7) // 8
    tops = pairs * 2 * 32 * ks / (ms * 1e-3) / 1e12
    # algorithmic work: L position compares per pair (one MAC each, x2 ops) against the same peak
    algo_tops = pairs * 2 * L / (ms * 1e-3) / 1e12
    out["roofline"] = {"bound": "mfma", "kernel": "k_allpairs_mfma (v_mfma_i32_32x32x32_i8)", "achieved": tops,
                       "peak": I8_PEAK_TOPS, "unit": "TOP/s", "frac": tops / I8_PEAK_TOPS,
                       "frac_algorithmic": algo_tops / I8_PEAK_TOPS,
                       "note": "frac: issued i8 MAC ops x2 (one-hot codes, 4 MACs per position, K padded to "
                               "whole k-steps); frac_algorithmic: L compares per pair x2; dense i8 peak = 2x bf16"}
    return out


def bench_ragged(B, lib, dev, reps=5, name="ragged_50M_L50-150_U20", encode=True):
    """50M ragged reads of 50-150 nt drawn from a 2^20-item pool, device-resident
    (ss_synth_ragged_*: blob + offsets + lengths).  (a) ss_encode_var over the batch (wpr 5); (b) the
    drop-in counter engine fed from device memory, ss_ingest_add_device + ss_ingest_finish: the
    length split, one table per length (multi-word keys for L > 32: k_mw_*), the first-occurrence
    rows copied back -- checked against the generator-derived digest (tests/golden/ragged_digests.json)."""
    from shortseq_amd._native import check
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    with open(os.path.join(REPO, "tests", "golden", "ragged_digests.json")) as f:
        d = json.load(f)[name]
    n = d["n"]
    blob, offs, lens = B.synth_ragged_pool_reads(n, d["seed"], d["pool_seed"], d["U"], d["Lmin"], d["Lmax"], device=dev)
    nt = int(lens.sum().item())
    wpr = B.wpr_for(d["Lmax"])
    words = torch.empty((n, wpr), dtype=torch.int64, device=dev)
    fb = B.first_bad_buffer(dev)
    s = torch.cuda.current_stream(dev).cuda_stream

    def enc(_t):
        check(lib.ss_encode_var(blob.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, words.data_ptr(), wpr,
                                fb.data_ptr(), s), "encode_var")
    enc_bytes = nt + n * (8 + 4) + n * wpr * 8        # ASCII + offset + length in, wpr words out
    if encode:
        _el, tr = timed_loop(enc, reps, 2, 1)
        if int(fb.item()) != -1:
            raise SystemExit("PARITY FAILURE: ragged encode flagged a read")
        enc_ms = tr.region_ms / reps
    del words
    eng = B.DeviceIngest(dev)
    ts = []
    try:
        for r in range(reps + 1):
            eng.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.count(blob, offs, lens)
            gl, gc, gw = eng.results(copy=False)     # the rows in the engine's pinned host buffers
            if r:
                ts.append(time.perf_counter() - t0)
        gl, gc, gw = gl.copy(), gc.copy(), gw.copy()
    finally:
        eng.close()
    import oracle as _o   # the digest helper only (numpy), after timing
    if len(gl) != d["unique"] or _o.rows_digest(gl, gc, gw) != d["digest"]:
        raise SystemExit(f"PARITY FAILURE: ragged counter rows != {name}")
    t = float(np.median(ts))
    floor = nt + n * 12
    out = {"reads": n, "nt": nt, "len_range": [d["Lmin"], d["Lmax"]], "pool": d["U"], "unique": len(gl)}
    if encode:
        out["encode_var"] = {"ms_per_step": enc_ms, "nt_per_s": nt / enc_ms * 1e3,
                             "roofline": {"bound": "hbm", "kernel": "k_encode_var_dense",
                                          "achieved": enc_bytes / enc_ms / 1e6, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                          "frac": enc_bytes / enc_ms / 1e6 / HBM_PEAK_GBS,
                                          "traffic": load_traffic("encode_var_ragged", n)}}
    return dict(out, **{
            "count": {"s_per_call": t, "reads_per_s": n / t, "nt_per_s": nt / t,
                      "floor_frac": floor / t / 1e9 / HBM_PEAK_GBS, "parity": f"digest {name}",
                      "note": "ss_ingest_add_device + ss_ingest_finish wall time (host-synchronous engine: length "
                              "split, class encode + sketch, per-class tables, rows copied back to pinned host "
                              "memory); floor_frac = one read of the blob + offsets + lengths at 8 TB/s"}})


def bench_host_staged(B, dev, n=32_000_000, L=32, reps=5):
    """PCIe-inclusive C2: the reads in pageable host memory, packed words back to host memory
    (ss_encode_host: pinned ring + H2D / kernel / D2H streams).  Never `value`: the device-resident
    number is the metric; this is what a host-side caller sees."""
    a_dev = B.synth_reads(n, L, seed=1, device=dev)
    host = a_dev.cpu().numpy()
    out = np.empty((n, 1), np.uint64)
    st = B.host_stager(dev)
    st.encode(host, out=out)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        st.encode(host, out=out)
        ts.append(time.perf_counter() - t0)
    idx = np.unique(np.linspace(0, n - 1, 257).astype(np.int64))
    for i in idx:
        if [int(out[i, 0])] != known_words(1, int(i), L):
            raise SystemExit("PARITY FAILURE: host-staged encode")
    t = float(np.median(ts))
    # the stage split of two more (timed) calls, and where the copy threads run
    st.set_timing(True)
    st.stats()
    for _ in range(2):
        st.encode(host, out=out)
    split = st.stats()
    st.set_timing(False)
    del a_dev
    place = {k: split.pop(k) for k in ("copy_threads", "affinity_cpus", "gpu_numa_node", "pinned_cpus")}
    return {"reads": n, "read_len": L, "ms_per_call": t * 1e3, "nt_per_s": n * L / t,
            "host_dev_GB_per_s": n * (L + 8) / t / 1e9, "stage_ms": split, **place,
            # the H2D copies' own time (summed over chunks) is the PCIe floor of the call
            "h2d_floor_frac": split["h2d_dev"] / (t * 1e3),
            "note": "pageable numpy in -> numpy out through ss_encode_host (64-MiB chunks, 3 slots, "
                    "12 staging threads pinned to the GPU's NUMA node within the affinity mask); stage_ms: "
                    "host copy / wait ms and device H2D / kernel / D2H ms per call (device sums overlap "
                    "across chunks); PCIe-bound, not the roofline number"}


def _median_time(fn, reps=3):
    ts, out = [], None
    for _ in range(reps):
        out = None
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), out


def bench_c1_dropin(n=1_000_000, L=32):
    """BASELINE configs[0] (C1): 1M x 32-nt synthetic reads through the drop-in Python API —
    sq.pack() per object (host codec) and ShortSeqCounter(list) (GPU batch path); median of 3
    calls each (the reference's API was timed the same way in the build container,
    oracle/calibrate_cpu_baseline.py)."""
    import shortseq_amd as sq
    import shortseq_amd.batch as B
    # the SURVEY §8(d) generator on the device, copied to host bytes objects (the API's input shape)
    a = B.synth_reads(n, L, seed=11, device="cuda").cpu().numpy().reshape(-1)
    reads = [a[i * L:(i + 1) * L].tobytes() for i in range(n)]
    t_pack, objs = _median_time(lambda: [sq.pack(r) for r in reads])
    sq.ShortSeqCounter(reads[:100_000])                    # warm the GPU path
    torch.cuda.synchronize()
    t_cnt, c = _median_time(lambda: sq.ShortSeqCounter(reads))
    if len(c) != len(set(reads)) or sum(c.values()) != n or str(objs[7]) != reads[7].decode():
        raise SystemExit("PARITY FAILURE: C1 drop-in")
    # the same API on a duplicate-heavy list (2^14-read pool): the dict the API must return is small
    pa = B.synth_pool_reads(n, L, 12, 13, 1 << 14, device="cuda").cpu().numpy().reshape(-1)
    preads = [pa[i * L:(i + 1) * L].tobytes() for i in range(n)]
    t_pool, pc = _median_time(lambda: sq.ShortSeqCounter(preads))
    if sum(pc.values()) != n:
        raise SystemExit("PARITY FAILURE: C1 drop-in (pool)")
    return {"reads": n, "read_len": L, "pack_per_s": n / t_pack, "counter_reads_per_s": n / t_cnt,
            "unique": len(c), "counter_pool16k_reads_per_s": n / t_pool, "pool_unique": len(pc),
            "note": "wall time incl. Python object creation (the reference's own API shape), median of 3"}


def bench_dropin_multidevice(n=8_000_000, L=32, U=1 << 22):
    """The drop-in counter over every visible device (only when the process sees
    >= 2 GPUs): ShortSeqCounter(list, device=[0 .. D-1]) -- one engine per device counts a contiguous
    slice, then the tree reduce over peer copies (_reduce_fill) -- against the same list on device 0;
    the dicts must be equal (keys, counts and first-occurrence order)."""
    import shortseq_amd as sq
    import shortseq_amd.batch as B
    D = min(8, torch.cuda.device_count())
    a = B.synth_pool_reads(n, L, 21, 22, U, device="cuda").cpu().numpy().reshape(-1)
    reads = [a[i * L:(i + 1) * L].tobytes() for i in range(n)]
    devs = list(range(D))
    sq.ShortSeqCounter(reads[:200_000], device=devs)          # warm every engine
    t1, c1 = _median_time(lambda: sq.ShortSeqCounter(reads, device=0))
    tD, cD = _median_time(lambda: sq.ShortSeqCounter(reads, device=devs))
    if list(cD.items())[:1000] != list(c1.items())[:1000] or len(cD) != len(c1) or sum(cD.values()) != n:
        raise SystemExit("PARITY FAILURE: multi-device drop-in counter")
    return {"devices": D, "reads": n, "read_len": L, "pool": U, "unique": len(cD), "s_one_device": t1,
            "s_all_devices": tD, "speedup": t1 / tD,
            "note": "wall time incl. building the dict; the shards reduce as a tree over peer copies"}


def _fastq_case_file(reps=128):
    """The small-RNA-like FASTQ of tools/probe_fastq_e2e.py: 8.4M ragged 18-32-nt records, 65,536
    distinct sequences each 128 times (528 MB; reps=512: the same pool 4x as long, 2.1 GB, three
    1-GiB chunks through the reader ring), written once to a temporary file."""
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import probe_fastq_e2e as P
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    path = os.path.join(d, f"smallrna_{reps}.fq")
    n = P.write_pool_file(path, reps=reps)
    return path, n


def bench_fastq_dropin(path, n):
    """a18 drop-in: sq.read_and_count_fastq(path) end to end (file read in pinned chunks, device
    index + length groups + counters, dict rebuilt in first-occurrence order)."""
    import contextlib
    import io
    import shortseq_amd as sq
    with contextlib.redirect_stdout(io.StringIO()):
        sq.read_and_count_fastq(path, device="cuda")                 # warm
        ts, c = [], None
        for _ in range(3):
            c = None          # (the previous dict's 65,536 objects are freed outside the timed call)
            t0 = time.perf_counter()
            c = sq.read_and_count_fastq(path, device="cuda")
            ts.append(time.perf_counter() - t0)
    if len(c) != 65536 or sum(c.values()) != n:
        raise SystemExit("PARITY FAILURE: read_and_count_fastq drop-in")
    t = float(np.median(ts))
    # the stage split of the last call and the PCIe floor: the file's bytes at the
    # host -> device rate the same call's H2D copies ran at
    from shortseq_amd import _shortseq
    st = (_shortseq.fastq_stage_times() or [{}])[0]
    fb = os.path.getsize(path)
    out = {"records": n, "file_bytes": fb, "s_per_call": t, "records_per_s": n / t, "unique": len(c)}
    if st.get("h2d_dev_ms"):
        rate = st["h2d_bytes"] / (st["h2d_dev_ms"] * 1e-3)
        out["stage_ms"] = {k: st[k] for k in ("read_ms", "h2d_dev_ms", "index_ms", "count_ms", "finish_ms",
                                              "reduce_and_dict_ms", "total_ms") if k in st}
        out["h2d_GB_per_s"] = rate / 1e9
        out["pcie_floor_s"] = fb / rate
        out["floor_frac"] = fb / rate / t
    out["note"] = ("wall time of the drop-in call on a 528-MB small-RNA-like FASTQ (page-cached), incl. building "
                   "the 65,536-entry dict; stage_ms of the last call (reads and H2D overlap); floor = file bytes "
                   "at the H2D rate the call's copies ran at")
    return out


def cpu_baseline(target_s=2.0):
    """The reference's per-read CPU algorithms (oracle/cpu_baseline.cpp, kind "port": table loop for
    L <= 32, PEXT blocks beyond, XOR-collapse-popcount hamming, charmap decode, a hash map for the
    counter) timed on this host over bounded samples of C2-C5 and C3': 1 core (the reference is
    single-threaded) and all the cores this process may use (OpenMP).  The reference itself never runs
    here; its own numbers (the kernels' calibration ratios, and its Python API for C1 / a18 / C3') were
    measured in the build container by oracle/calibrate_cpu_baseline.py
    (profiles/r3/cpu_baseline_calibration.json) and are attached, labelled."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import cpu_baseline as cb  # test/baseline infrastructure only — never the measured GPU path
    res = cb.run_all(target_s)
    th = res["threads_all"]
    c2 = res["C2_encode_32"]
    cfgs = {k: {"unit": v["unit"], "1_core": v["1_core"], "all_cores": v[f"{th}_cores"]}
            for k, v in res.items() if k.startswith("C")}
    out = {"value": c2["1_core"], "unit": "nt/s", "cores": 1, "kind": "port",
           "value_all_cores": c2[f"{th}_cores"], "cores_all": th,
           "sample": f"C2 {c2['sample_1_core']} (1 core); oracle/cpu_baseline.cpp on {res['cpu']}, "
                     f"nproc {res['nproc']}, {th} threads for all_cores",
           "configs": cfgs}
    cal = os.path.join(REPO, "profiles", "r3", "cpu_baseline_calibration.json")
    if os.path.exists(cal):
        with open(cal) as f:
            c = json.load(f)
        # port speed / reference speed, 1 pinned core, median of 9 interleaved rounds (min..max)
        out["calibration"] = {k: [v["ratio"], v.get("ratio_min"), v.get("ratio_max")] if "ratio_min" in v else v["ratio"]
                              for k, v in c.items() if isinstance(v, dict) and "ratio" in v}
        pick = {"C2_encode_32": "encode_32", "C3_encode_hamming_96": "encode_96",
                "C4_roundtrip_512": "encode_512", "C5_counter_32": "counter_32_pool2^24"}
        for cfg, key in pick.items():
            if cfg in cfgs and key in c:
                cfgs[cfg]["ref_equiv_1_core"] = cfgs[cfg]["1_core"] / c[key]["ratio"]
        # the counter port runs 0.59x the reference (a std::unordered_map per key vs the reference's
        # CPython dict of ShortSeq objects): C5's 1-core value is the reference-equivalent rate (port /
        # ratio), the port's own rate kept beside it
        c5 = cfgs.get("C5_counter_32")
        if c5 is not None and "ref_equiv_1_core" in c5:
            c5["port_1_core"] = c5["1_core"]
            c5["1_core"] = c5["ref_equiv_1_core"]
        api = {}
        if c.get("C1_reference_api"):
            api["C1_counter_reads_per_s"] = c["C1_reference_api"]["counter_reads_per_s"]
            api["C1_pack_per_s"] = c["C1_reference_api"]["pack_per_s"]
        if c.get("a18_reference_read_and_count_fastq"):
            api["a18_records_per_s"] = c["a18_reference_read_and_count_fastq"]["records_per_s"]
        for L in (32, 96, 512):
            if c.get(f"hamming_{L}"):
                api[f"C3p_xor_api_{L}_pairs_per_s"] = c[f"hamming_{L}"]["reference_api_pairs_per_s"]
        out["reference_api_container"] = api
    return out


def launch_ranks(n: int) -> int:
    """`python bench.py --gpus N` without a launcher: run this same command under
    torch.distributed.run with N ranks (127.0.0.1 rendezvous, a free port) and return its exit code.
    Only argv and the environment are handed on; this process never initialises the GPU."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    log(f"no launcher: starting {n} ranks ({' '.join(cmd[1:6])} ...)")
    return subprocess.call(cmd)


def dry_run(args, world: int, rank: int) -> None:
    """The contract's plumbing with no GPU work (CPU tests of the launcher): gloo rendezvous, W + K
    no-op steps between barriers, max over ranks, rank 0 prints the line (value null)."""
    if world > 1:
        dist.init_process_group("gloo")
    for _ in range(args.warmup):
        pass
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        dist.barrier()
    if rank == 0:
        print(json.dumps({"metric": "nt/sec 2-bit encode (32/96/512-nt batches) + hamming pairs/sec; % HBM roofline",
                          "value": None, "unit": "nt/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": el / max(1, args.steps) * 1e3,
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
                          "data": "dry run: no GPU work (launcher / rendezvous plumbing only)",
                          "config": {"workload": "dry run", "reads_per_gpu": args.reads_per_gpu,
                                     "parallelism": f"dp{world}"}}, separators=(",", ":")), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    # the MI355X clock needs tens of ms of sustained load to settle (tools/diag_bench.py: the first
    # ~20 back-to-back launches run ~3% slower); 50 warmup launches of the 0.6-ms kernel ~= 30 ms
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--reads-per-gpu", type=int, default=100_000_000, help="reads per GPU (C2, C3; C4 uses half)")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=2.0, help="timed seconds per CPU-baseline leg (8 legs)")
    ap.add_argument("--dist-backend", default=os.environ.get("SHORTSEQ_DIST_BACKEND", "nccl"),
                    help="nccl (= RCCL over xGMI, default) or gloo (rehearsal: several ranks on one GPU)")
    ap.add_argument("--same-device", action="store_true",
                    help="map every rank to cuda:0 (multi-rank rehearsal on a 1-GPU box)")
    ap.add_argument("--dry-run", action="store_true",
                    help="plumbing only (no GPU work): the launcher, the rendezvous, the barrier + "
                         "max-over-ranks timing around a no-op step and rank 0's JSON line (value null)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start the N ranks ourselves, in fresh child processes, before
        # anything here touches the GPU, and hand on rank 0's JSON line (the children inherit stdout)
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # never report one number under another N
        log(f"error: --gpus {args.gpus} but WORLD_SIZE {world}")
        sys.exit(2)
    if args.dry_run:
        dry_run(args, world, rank)
        return
    dev_idx = 0 if args.same_device else local_rank
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    import shortseq_amd.batch as B
    from shortseq_amd._native import lib as _lib
    lib = _lib()

    L, n = 32, args.reads_per_gpu
    log(f"rank {rank}/{world}: C2 encode {n} x {L} nt")
    el, kern_ms = bench_encode(B, lib, dev, rank, world, n, L, args.steps, args.warmup)
    ms_step = el / args.steps * 1e3
    total_nt = n * L * world
    value = total_nt / (el / args.steps)
    algo_bytes = n * (L + 8)  # 32 B ASCII in + 8 B packed word out per read
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
    result = {
        "metric": "nt/sec 2-bit encode (32/96/512-nt batches) + hamming pairs/sec; % HBM roofline",
        "value": value, "unit": "nt/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_step, "higher_is_better": True, "settle_s": SETTLE_S, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic (device-side splitmix64 reads, SURVEY §8(d))",
        "config": {"workload": f"C2: {n / 1e6:g}M x 32-nt batch encode (short_seq_64 path) per GPU",
                   "reads_per_gpu": n, "read_len": L, "global_batch": n * world,
                   "parallelism": f"dp{world} (read shards, no collective)"},
        "roofline": {"bound": "hbm", "kernel": "k_encode_g16<dense>", "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": load_traffic("encode32", n), "algo_bytes_per_launch": algo_bytes,
                     "kernel_ms": kern_ms},
    }
    log(f"C2: {value / 1e12:.3f} T nt/s, kernel {kern_ms:.3f} ms, {achieved:.0f} GB/s")

    fq_path, fq_n = None, 0
    if not args.no_extras:
        extra = {}
        L3, n3 = 96, args.reads_per_gpu
        log(f"C3 fused encode+hamming {n3} x {L3}")
        el3, k3, d3 = bench_encode_hamming(B, lib, dev, rank, world, n3, L3, args.steps, args.warmup)
        b3 = n3 * (96 + 24 + 4)
        extra["C3_encode_hamming_96"] = {
            "pairs_per_s": n3 * world / (el3 / args.steps), "nt_per_s": n3 * L3 * world / (el3 / args.steps),
            "ms_per_step": el3 / args.steps * 1e3, "kernel_ms_events": k3, "device_ms_per_step": d3,
            "roofline": {"kernel": "k_encode_ham_dense", "achieved": b3 / (k3 * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": b3 / (k3 * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "algo_bytes_per_launch": b3, "kernel_ms": k3, "traffic": load_traffic("encode_hamming96", n3),
                         "note": "HIP events around the K back-to-back fused launches of the timed region "
                                 "(the reference read packed once before it)"}}
        for Lh, nh in ((32, args.reads_per_gpu), (96, args.reads_per_gpu), (512, args.reads_per_gpu // 2)):
            log(f"C3' hamming only (pre-packed) {nh} x {Lh}")
            elh, dh = bench_hamming_only(B, lib, dev, rank, world, nh, Lh, args.steps, args.warmup)
            bh = nh * (8 * B.wpr_for(Lh) + 4)   # packed words in + u32 distance out
            extra[f"C3p_hamming_ref_{Lh}"] = {
                "pairs_per_s": nh * world / (elh / args.steps), "ms_per_step": elh / args.steps * 1e3,
                "device_ms_per_step": dh, "reads": nh,
                "roofline": {"kernel": "k_ham_dense3x" if Lh == 96 else "k_ham_dense",
                             "achieved": bh / (dh * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": bh / (dh * 1e-3) / 1e9 / HBM_PEAK_GBS, "algo_bytes_per_step": bh,
                             "traffic": load_traffic(f"hamming_ref_{Lh}", nh)}}
        L4, n4 = 512, args.reads_per_gpu // 2
        log(f"C4 encode+decode {n4} x {L4}")
        s4 = max(5, args.steps // 2)
        el4, ke, kd, d4 = bench_roundtrip(B, lib, dev, rank, world, n4, L4, s4, args.warmup)
        b4e, b4d = n4 * (512 + 128), n4 * (128 + 512)
        extra["C4_roundtrip_512"] = {
            "nt_per_s": n4 * L4 * world / (el4 / s4), "ms_per_step": el4 / s4 * 1e3,
            "encode_kernel_ms_events": ke, "decode_kernel_ms_events": kd, "device_ms_per_step": d4,
            "roofline": {"kernel": "k_encode_g16<pext> + k_decode_g16", "achieved": (b4e + b4d) / (d4 * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": (b4e + b4d) / (d4 * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "algo_bytes_per_step": b4e + b4d,
                         "traffic": (None if load_traffic("encode512", n4) is None or load_traffic("decode512", n4) is None
                                     else load_traffic("encode512", n4) + load_traffic("decode512", n4))}}

        def c5_extras():
            n5, U5 = 125_000_000, 1 << 24
            log(f"C5 counter {n5} x 32 per GPU, pool {U5}")
            s5 = max(3, args.steps // 4)
            el5, d5, uniq, chk5, pass5, exch5 = bench_counter(B, lib, dev, rank, world, n5, 32, U5, s5, 2)
            # SURVEY §8(d) prices C5 at the 32 B of ASCII per read (the problem's floor): that is the
            # headline frac.  Beside it, the partitioned pipeline's own pass bytes: coarse
            # pass 32 in + 12 out (key, read index), fine scatter 12 + 12, aggregate 12 + the whole
            # table written once (fresh slices: 16 B x 2^25 slots, amortised over the reads)
            table_b = 16 * (2 * U5) / n5
            pipe_b = 32 + 12 + 24 + 12 + table_b
            extra["C5_counter_32"] = {
                "reads_per_s": n5 * world / (el5 / s5), "ms_per_step": el5 / s5 * 1e3, "device_ms_per_step": d5,
                "reads_per_gpu": n5, "pool": U5, "unique": uniq, "parity": chk5, "passes_ms": pass5,
                "roofline": {"bound": "hbm", "kernel": "partitioned insert (k_pf_coarse, k_pf_scatter, "
                                                        "k_pc_aggregate_slice)",
                             "achieved": n5 * 32 / (d5 * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": n5 * 32 / (d5 * 1e-3) / 1e9 / HBM_PEAK_GBS, "bytes_per_read": 32,
                             "frac_pipeline": n5 * pipe_b / (d5 * 1e-3) / 1e9 / HBM_PEAK_GBS,
                             "pipeline_bytes_per_read": pipe_b,
                             "traffic": load_traffic("counter32_insert", n5),
                             "note": "frac: 32 B of ASCII per read (SURVEY 8d); frac_pipeline: the passes' own bytes"},
                "merge": (f"all_to_all_single of 16-B (key, count, first) records by owner over {dist.get_backend()}"
                          f"{' (RCCL/xGMI)' if dist.get_backend() == 'nccl' else ' (host-staged rehearsal)'}")
                         if world > 1 else "none (1 GPU)"}
            if exch5 is not None:      # per-rank [min, max] of the diagnostic count's phases
                extra["C5_counter_32"]["exchange"] = exch5
            # SURVEY §8(d) C5 variants: the smaller pool and Zipf s = 1.1 skew (same shard size)
            for name, U_, zs in (("C5_counter_32_U20", 1 << 20, None), ("C5_counter_32_zipf1.1_U24", 1 << 24, 1.1),
                                 ("C5_counter_32_zipf1.1_U20", 1 << 20, 1.1)):
                log(f"C5 counter {n5} x 32 per GPU, pool {U_}, {'zipf ' + str(zs) if zs else 'uniform'}")
                el_, d_, u_, chk_, pass_, _x = bench_counter(B, lib, dev, rank, world, n5, 32, U_, s5, 2, zipf=zs)
                # the same pipeline bytes model with this pool's table (a skewed batch moves fewer records
                # through the fine passes after deduplication: the model is then an upper bound)
                pb_ = 32 + 12 + 24 + 12 + 16 * (2 * U_) / n5
                extra[name] = {"reads_per_s": n5 * world / (el_ / s5), "ms_per_step": el_ / s5 * 1e3,
                               "device_ms_per_step": d_, "reads_per_gpu": n5, "pool": U_, "zipf_s": zs, "unique": u_,
                               "parity": chk_, "passes_ms": pass_,
                               "vs_uniform_U24": d_ / d5,
                               "roofline": {"bound": "hbm", "kernel": "partitioned insert",
                                            "achieved": n5 * 32 / (d_ * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                                            "unit": "GB/s", "frac": n5 * 32 / (d_ * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                            "bytes_per_read": 32,
                                            "frac_pipeline": n5 * pb_ / (d_ * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                            "traffic": load_traffic("counter32_insert_" + name[len("C5_counter_32_"):], n5)}}

        # C5 (and at world > 1 its RCCL exchange): an exception every rank raises alike (e.g. a backend
        # without all_to_all) is recorded in the entry instead of costing the run its JSON line;
        # parity failures (SystemExit) still end the run
        try:
            c5_extras()
        except Exception as e:  # noqa: BLE001
            log(f"C5: {type(e).__name__}: {e}")
            extra.setdefault("C5_counter_32", {"error": f"{type(e).__name__}: {e}"})
        if rank == 0 or world == 1:
            # rank-local extras (no collective): an error is recorded in its entry instead of costing
            # the run its JSON line; parity failures (SystemExit) still end the run
            def local_extra(name, fn):
                try:
                    extra[name] = fn()
                except Exception as e:  # noqa: BLE001
                    log(f"{name}: {type(e).__name__}: {e}")
                    extra[name] = {"error": f"{type(e).__name__}: {e}"}

            if world == 1:
                log("C5 exchange rehearsal (8 owners, one GPU)")
                local_extra("C5_exchange_8owners", lambda: bench_exchange(B, dev))
            log("F1 FASTQ index / F4 all-pairs")
            local_extra("F1_fastq_index_100nt", lambda: bench_fastq_index(B, lib, dev))
            local_extra("F4_all_pairs_umi12", lambda: bench_all_pairs(B, lib, dev))
            # the default entry point (auto: pigeonhole buckets for this batch), same results
            local_extra("F4_all_pairs_umi12_auto", lambda: bench_all_pairs(B, lib, dev, method="auto"))
            # multi-word reads (round 6: the pigeonhole form for L <= 128): 100k 96-nt reads of a 2^16
            # pool within distance 3, the default entry point; the tiles' time beside it
            def f4_96():
                r = bench_all_pairs(B, lib, dev, n=100_000, L=96, k=3, method="auto", pool=1 << 16)
                t = bench_all_pairs(B, lib, dev, n=100_000, L=96, k=3, method="tiles", pool=1 << 16, reps=3)
                if t["hits"] != r["hits"]:
                    raise SystemExit("PARITY FAILURE: all-pairs 96 nt (auto vs tiles)")
                return {k_: r[k_] for k_ in ("n", "read_len", "max_dist", "ms_per_step", "pairs_per_s", "hits")} | \
                    {"tiles_ms_per_step": t["ms_per_step"]}
            local_extra("F4_all_pairs_96_auto", f4_96)
            log("F2 ragged 50-150 nt")
            local_extra("F2_ragged_50_150", lambda: bench_ragged(B, lib, dev))
            # the same reads over a 2^24-item pool: ~16M distinct keys, tables past the Infinity Cache
            local_extra("F2_ragged_50_150_U24", lambda: bench_ragged(B, lib, dev, reps=3, name="ragged_50M_L50-150_U24",
                                                                     encode=False))
            log("C2 host-staged (PCIe-inclusive)")
            local_extra("C2_host_staged_32", lambda: bench_host_staged(B, dev))
            log("C1 drop-in API")
            local_extra("C1_dropin_1M_32", bench_c1_dropin)
            if world == 1 and torch.cuda.device_count() >= 2:
                log("drop-in counter over every visible device")
                local_extra("C1_dropin_multidevice", bench_dropin_multidevice)
            log("a18 read_and_count_fastq drop-in")
            fq_path, fq_n = _fastq_case_file()
            local_extra("A18_read_and_count_fastq_smallrna", lambda: bench_fastq_dropin(fq_path, fq_n))
            os.remove(fq_path)
            log("a18 read_and_count_fastq drop-in, 2.1-GB file (three chunks)")

            def a18_long():
                p4, n4 = _fastq_case_file(512)
                try:
                    r = bench_fastq_dropin(p4, n4)
                finally:
                    os.remove(p4)
                return {k: r[k] for k in ("records", "file_bytes", "s_per_call", "records_per_s", "h2d_GB_per_s",
                                          "floor_frac") if k in r}
            local_extra("A18_read_and_count_fastq_2GB", a18_long)
        result["extra"] = extra

    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline ...")
            result["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        else:
            result["cpu_baseline"] = None
        # cpu_baseline before extra, and the line compacted: the driver keeps only stdout's tail
        ex = result.pop("extra", None)
        if ex is not None:
            result["extra"] = ex
        print(json.dumps(compact(result), separators=(",", ":")), flush=True)
    if fq_path is not None:
        import shutil
        shutil.rmtree(os.path.dirname(fq_path), ignore_errors=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
