"""Drop-in API batch paths on the GPU: ShortSeqCounter(list, device="cuda") and
read_and_count_fastq(device="cuda") must equal the host path and the reference fixtures exactly
(keys, counts, dict order, exceptions)."""
import random

import pytest

import shortseq_amd as sq
from shortseq_amd import ShortSeqCounter

pytestmark = pytest.mark.gpu


def _items(c):
    return [(type(k).__name__, str(k), len(k), v) for k, v in c.items()]


def test_golden_counter_gpu(gpu, golden):
    for case in golden["counter"]:
        if "reads_str" in case:
            with pytest.raises(TypeError) as ei:
                ShortSeqCounter(case["reads_str"], device="cuda")
            assert str(ei.value) == case["message"]
            continue
        reads = [bytes.fromhex(h) for h in case["reads_hex"]]
        if "raises" in case:
            with pytest.raises(Exception) as ei:
                ShortSeqCounter(reads, device="cuda")
            assert str(ei.value) == case["message"]
            continue
        c = ShortSeqCounter(reads, device="cuda")
        exp = [(it["class"], it["str"], it["length"], it["count"]) for it in case["items"]]
        assert _items(c) == exp


def test_counter_gpu_equals_host_mixed(gpu):
    rng = random.Random(3)
    pool = []
    for L in [0, 1, 2, 5, 16, 17, 31, 32, 33, 40, 64, 96, 97, 150, 1024]:
        for _ in range(6):
            pool.append(bytes(rng.choice(b"ACGT") for _ in range(L)))
    pool.append(b"G" * 32)                 # the packed word that collides with the table's EMPTY
    pool.append(b"\x01A\x14" * 5)          # aliased bytes (table-path carry)
    reads = [rng.choice(pool) for _ in range(100_000)]
    host = ShortSeqCounter(reads, device="host")
    dev = ShortSeqCounter(reads, device="cuda")
    assert _items(dev) == _items(host)
    auto = ShortSeqCounter(reads)          # >= GPU_MIN_READS -> GPU
    assert _items(auto) == _items(host)
    assert dev[sq.pack("G" * 32)] == host[sq.pack("G" * 32)]


def test_counter_gpu_short_group(gpu):
    """Lengths 1..31 share one table (each key = the packed word with a length marker above it and
    above its table-path carry bit): a read whose last byte is aliased (\\x01 \\x03 \\x07 \\x14, whose
    carry lands on bit 2L) stays apart from the read with an 'A' there and from the read one base
    longer; ragged and dense (one-length) batches; the first rejected read is the first in input
    order across lengths."""
    rng = random.Random(41)
    pool = []
    for L in range(1, 32):
        for _ in range(3):
            s = bytes(rng.choice(b"ACGT") for _ in range(L))
            pool.append(s)
            pool += [s[:-1] + a for a in (b"\x01", b"\x03", b"\x07", b"\x14", b"A")]
            pool.append(s + b"A")
    reads = [rng.choice(pool) for _ in range(60_000)]
    host = ShortSeqCounter(reads, device="host")
    assert _items(ShortSeqCounter(reads, device="cuda")) == _items(host)
    for L in (1, 7, 20, 31):
        one = [r for r in pool if len(r) == L]
        dense = [rng.choice(one) for _ in range(20_000)]
        assert _items(ShortSeqCounter(dense, device="cuda")) == _items(ShortSeqCounter(dense, device="host")), L
    bad = list(reads)
    bad[40_000] = b"ACGTN" + b"A" * 20
    bad[30_000] = b"ACX"
    with pytest.raises(Exception) as ei_h:
        ShortSeqCounter(bad, device="host")
    with pytest.raises(Exception) as ei_d:
        ShortSeqCounter(bad, device="cuda")
    assert str(ei_d.value) == str(ei_h.value) == "Unsupported base character: X"


def test_counter_gpu_errors_first_bad(gpu):
    rng = random.Random(4)
    reads = [bytes(rng.choice(b"ACGT") for _ in range(rng.choice([8, 32, 50]))) for _ in range(70_000)]
    reads[50_000] = b"ACGTN" + b"A" * 27          # 32 nt, table path: last bad byte
    reads[60_000] = b"A" * 40 + b"N"              # 41 nt, host path group
    reads[65_000] = b"A" * 40 + b"*" * 10
    with pytest.raises(Exception) as ei_h:
        ShortSeqCounter(reads, device="host")
    with pytest.raises(Exception) as ei_d:
        ShortSeqCounter(reads, device="cuda")
    assert str(ei_d.value) == str(ei_h.value) == "Unsupported base character: N"
    reads[50_000] = b"A" * 32
    with pytest.raises(Exception) as ei_d:
        ShortSeqCounter(reads, device="cuda")
    assert str(ei_d.value) == "Unsupported base character: N"
    reads2 = list(reads)
    reads2[10] = "ACGT"
    with pytest.raises(TypeError):
        ShortSeqCounter(reads2, device="cuda")


def test_fastq_gpu(gpu, tmp_path):
    rng = random.Random(5)
    pool = [bytes(rng.choice(b"ACGT") for _ in range(rng.choice([20, 32, 33, 75]))) for _ in range(500)]
    lines = []
    for i in range(80_000):
        s = rng.choice(pool).decode()
        lines.append(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n")
    p = tmp_path / "big.fq"
    p.write_text("".join(lines))
    h = sq.read_and_count_fastq(str(p), device="host")
    d = sq.read_and_count_fastq(str(p), device="cuda")
    assert _items(d) == _items(h)
    assert sum(d.values()) == 80_000


def test_c1_dropin_reference_digest(gpu, digests, oracle):
    """BASELINE configs[0] (C1) through the drop-in API on the GPU: ShortSeqCounter(list) of the 1M x
    32-nt pool-65536 reads reproduces the reference ShortSeqCounter's own ordered digest (keys, length,
    count in dict order; tests/golden/golden_digests.json, captured from the compiled reference)."""
    import hashlib
    import numpy as np
    d = digests["counter_1000000x32_pool65536"]
    n, L = d["n"], d["L"]
    a = oracle.gen_pool_reads(d["seed"], d["pool_seed"], d["U"], 0, n, L)
    reads = [a[i * L:(i + 1) * L].tobytes() for i in range(n)]
    c = ShortSeqCounter(reads, device="cuda")
    assert len(c) == d["unique"]
    rows = np.array([(k.packed[0], len(k), v) for k, v in c.items()], dtype=np.uint64)
    assert hashlib.sha256(np.ascontiguousarray(rows).tobytes()).hexdigest() == d["ordered_sha256"]


def test_gpu_batch_path_without_torch(gpu, tmp_path):
    """ShortSeqCounter(list) and read_and_count_fastq on the GPU go Cython -> C ABI: a fresh
    interpreter runs both on the device and never imports torch; results equal the host path."""
    import subprocess
    import sys
    code = r'''
import random, sys
import shortseq_amd as sq
rng = random.Random(7)
pool = [bytes(rng.choice(b"ACGT") for _ in range(rng.choice([0, 12, 32, 33, 100]))) for _ in range(300)]
reads = [rng.choice(pool) for _ in range(120_000)]
d = sq.ShortSeqCounter(reads, device="cuda")
h = sq.ShortSeqCounter(reads, device="host")
assert [(str(k), v) for k, v in d.items()] == [(str(k), v) for k, v in h.items()]
p = sys.argv[1]
with open(p, "w") as f:
    for i, r in enumerate(reads[:50_000]):
        f.write(f"@r{i}\n{r.decode()}A\n+\n{'I' * (len(r) + 1)}\n")
fd = sq.read_and_count_fastq(p, device="cuda")
fh = sq.read_and_count_fastq(p, device="host")
assert [(str(k), v) for k, v in fd.items()] == [(str(k), v) for k, v in fh.items()]
assert "torch" not in sys.modules, "torch imported"
print("ok")
'''
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code, str(tmp_path / "x.fq")], cwd=repo, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "ok" in out.stdout


@pytest.mark.parametrize("ndev", [2, 3, 8])
def test_c1_dropin_reference_digest_multi_engine(gpu, digests, oracle, ndev):
    """The multi-GPU drop-in (counter.pyx:10-54 over a list sharded by contiguous read ranges, one
    ingest engine per device, rows merged in shard order) rehearsed with `ndev` engines on device 0:
    the reference's ordered digest of the 1M x 32 pool-65536 list, exactly as with one engine."""
    import hashlib
    import numpy as np
    d = digests["counter_1000000x32_pool65536"]
    n, L = d["n"], d["L"]
    a = oracle.gen_pool_reads(d["seed"], d["pool_seed"], d["U"], 0, n, L)
    reads = [a[i * L:(i + 1) * L].tobytes() for i in range(n)]
    c = ShortSeqCounter(reads, device=[0] * ndev)
    assert len(c) == d["unique"]
    rows = np.array([(k.packed[0], len(k), v) for k, v in c.items()], dtype=np.uint64)
    assert hashlib.sha256(np.ascontiguousarray(rows).tobytes()).hexdigest() == d["ordered_sha256"]


@pytest.mark.parametrize("ndev", [2, 3, 8])
def test_multi_engine_golden_and_mixed(gpu, golden, ndev):
    """Golden counter cases (errors too) and a mixed-length list through `ndev` engines: identical
    to the single-device and host paths (dict order across shard boundaries, the first error in list
    order)."""
    devs = [0] * ndev
    for case in golden["counter"]:
        if "reads_str" in case:
            continue
        reads = [bytes.fromhex(h) for h in case["reads_hex"]]
        if "raises" in case:
            with pytest.raises(Exception) as ei:
                ShortSeqCounter(reads, device=devs)
            assert str(ei.value) == case["message"]
            continue
        c = ShortSeqCounter(reads, device=devs)
        assert _items(c) == [(it["class"], it["str"], it["length"], it["count"]) for it in case["items"]]
    rng = random.Random(31)
    pool = [bytes(rng.choice(b"ACGT") for _ in range(L)) for L in (0, 3, 16, 32, 33, 64, 96, 97, 300, 1024)
            for _ in range(5)]
    reads = [rng.choice(pool) for _ in range(90_000)]
    assert _items(ShortSeqCounter(reads, device=devs)) == _items(ShortSeqCounter(reads, device="host"))
    reads[70_000] = b"ACGTX"
    reads[80_000] = b"ACGTN"
    with pytest.raises(Exception) as ei:
        ShortSeqCounter(reads, device=devs)
    assert str(ei.value) == "Unsupported base character: X"


@pytest.mark.parametrize("ndev", [2, 3, 8])
def test_fastq_multi_engine(gpu, golden, tmp_path, ndev):
    """read_and_count_fastq split into `ndev` byte ranges at line boundaries (ss_fastq_split: the
    lines before each range keep the j % 4 == 1 selection global), one engine each: the reference's
    FASTQ fixtures and a random file equal the host path."""
    devs = [0] * ndev
    for name, case in sorted(golden["fastq"].items()):
        p = tmp_path / (name + ".fq")
        p.write_bytes(bytes.fromhex(case["file_hex"]))
        if case["raises"]:
            with pytest.raises(Exception) as ei:
                sq.read_and_count_fastq(str(p), device=devs)
            assert str(ei.value) == case["message"], name
            continue
        c = sq.read_and_count_fastq(str(p), device=devs)
        h = sq.read_and_count_fastq(str(p), device="host")
        assert _items(c) == _items(h), name
    rng = random.Random(32)
    pool = [bytes(rng.choice(b"ACGT") for _ in range(rng.choice([18, 32, 33, 75, 151]))) for _ in range(700)]
    lines = [f"@r{i}\n{rng.choice(pool).decode()}\n+\n{'I' * 10}\n" for i in range(60_000)]
    p = tmp_path / "multi.fq"
    p.write_text("".join(lines))
    assert _items(sq.read_and_count_fastq(str(p), device=devs)) == _items(sq.read_and_count_fastq(str(p), device="host"))


def test_engines_thread_safe(gpu):
    """concurrent ShortSeqCounter calls from several Python threads (the GIL is released
    while they count) each get their own engine: every thread's dict is exact."""
    import threading
    rng = random.Random(33)
    lists = []
    for t in range(4):
        pool = [bytes(rng.choice(b"ACGT") for _ in range(rng.choice([12, 32, 40]))) for _ in range(400)]
        lists.append([rng.choice(pool) for _ in range(80_000)])
    want = [_items(ShortSeqCounter(r, device="host")) for r in lists]
    got = [None] * len(lists)

    def run(i):
        for _ in range(3):
            got[i] = _items(ShortSeqCounter(lists[i], device="cuda"))
    ts = [threading.Thread(target=run, args=(i,)) for i in range(len(lists))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert got == want


def _rows_of(counter):
    """A ShortSeqCounter's dict as the ss_ingest_results layout (lens, counts, words)."""
    import numpy as np
    lens, cnts, words = [], [], []
    for k, v in counter.items():
        lens.append(len(k))
        cnts.append(v)
        words.extend(int(w) for w in k.packed[:max(0, (len(k) + 31) // 32)])
    return np.array(lens, np.uint32), np.array(cnts, np.uint64), np.array(words, np.uint64)


@pytest.mark.parametrize("ndev", [2, 3, 5, 8])
def test_multi_engine_ragged_device_reduce(gpu, oracle, ndev):
    """a mixed 1-300-nt list through `ndev` engines reduces on the device
    (ss_ingest_export + ss_ingest_merge into the first shard's engine: single-word length tables and
    multi-word length classes alike) and the dict equals the generator-derived rows (pinned to
    oracle.count): keys, counts and first-occurrence order across every shard boundary."""
    import numpy as np
    seed, ps, U, n, lo, hi = 43, 44, 1 << 12, 60_000, 1, 300
    reads = oracle.ragged_pool_reads(seed, ps, U, 0, n, lo, hi)
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    gl, gc, gw = _rows_of(ShortSeqCounter(reads, device=[0] * ndev))
    assert gl.tolist() == el.tolist()
    assert gc.tolist() == ec.tolist()
    assert np.array_equal(gw, ew)


def test_device_ingest_export_merge(gpu, oracle):
    """The reduce at the C ABI: three DeviceIngest engines count consecutive slices of one ragged
    device batch (33-700 nt: class tables of several widths, plus 0-32 nt single-word tables in the
    second case), export, and fold into the first (ss_ingest_merge with each slice's global base);
    the first engine's rows equal the whole batch's generator-derived rows.  Merging out of order or
    an engine that was not exported is refused."""
    import shortseq_amd.batch as B
    from shortseq_amd._native import NativeError
    for seed, ps, U, n, lo, hi in ((47, 48, 3000, 150_000, 33, 700), (45, 46, 5000, 120_000, 0, 90)):
        blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
        cuts = [0, n // 5, n // 2, n]
        engs = [B.DeviceIngest(gpu) for _ in range(3)]
        try:
            for k, e in enumerate(engs):
                e.count(blob, offs[cuts[k]:cuts[k + 1]], lens[cuts[k]:cuts[k + 1]])
            with pytest.raises(NativeError, match="export"):
                engs[0].merge(engs[1], cuts[1])
            for e in engs[1:]:
                assert e.export() > 0
            with pytest.raises(NativeError, match="in order"):
                engs[0].merge(engs[2], 5)
            engs[0].merge(engs[1], cuts[1])
            engs[0].merge(engs[2], cuts[2])
            gl, gc, gw = engs[0].results()
        finally:
            for e in engs:
                e.close()
        el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
        assert gl.tolist() == el.tolist()
        assert gc.tolist() == ec.tolist()
        assert (gw == ew).all()


@pytest.mark.parametrize("ndev", [3, 6, 8])
def test_reduce_tree_equals_chain(gpu, oracle, ndev):
    """the tree reduce (adjacent pairs merged concurrently, log2(D) rounds, the
    round-2+ sources re-exported) and the serial chain into engine 0 give the same dict, equal to the
    generator-derived rows; a mixed 0-200-nt list (single-word lengths and length classes)."""
    import shortseq_amd._shortseq as S
    seed, ps, U, n, lo, hi = 51, 52, 1 << 11, 40_000, 0, 200
    reads = oracle.ragged_pool_reads(seed, ps, U, 0, n, lo, hi)
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    try:
        for mode in ("chain", "tree", "auto"):
            S._set_reduce_mode(mode)
            gl, gc, gw = _rows_of(ShortSeqCounter(reads, device=[0] * ndev))
            assert gl.tolist() == el.tolist(), mode
            assert gc.tolist() == ec.tolist(), mode
            assert (gw == ew).all(), mode
    finally:
        S._set_reduce_mode("auto")


def test_device_ingest_tree_merge_abi(gpu, oracle):
    """The tree at the C ABI: four engines on consecutive slices; 1 -> 0 and 3 -> 2 (concurrently, from
    two threads), then 2 (re-exported: it received 3) -> 0.  Merging a destination that received
    merges without exporting it again is refused."""
    import threading
    import shortseq_amd.batch as B
    from shortseq_amd._native import NativeError
    seed, ps, U, n, lo, hi = 53, 54, 4000, 160_000, 20, 180
    blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
    cuts = [0, n // 7, n // 2, 3 * n // 4, n]
    engs = [B.DeviceIngest(gpu) for _ in range(4)]
    try:
        for k, e in enumerate(engs):
            e.count(blob, offs[cuts[k]:cuts[k + 1]], lens[cuts[k]:cuts[k + 1]])
        for e in engs[1:]:
            e.export()
        ts = [threading.Thread(target=engs[0].merge, args=(engs[1], cuts[1])),
              threading.Thread(target=engs[2].merge, args=(engs[3], cuts[3] - cuts[2]))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        with pytest.raises(NativeError, match="export"):
            engs[0].merge(engs[2], cuts[2])
        engs[2].export()
        engs[0].merge(engs[2], cuts[2])
        gl, gc, gw = engs[0].results()
    finally:
        for e in engs:
            e.close()
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    assert gl.tolist() == el.tolist()
    assert gc.tolist() == ec.tolist()
    assert (gw == ew).all()


@pytest.mark.parametrize("reserve", [False, True])
def test_device_ingest_chain_reserve_abi(gpu, oracle, reserve):
    """A chain of five exported engines into engine 0, with and without ss_ingest_reserve_merge
    (engine 0's tables sized once for the union): the same rows as the generator; reserving with an
    unexported source or with the destination among the sources is refused."""
    import shortseq_amd.batch as B
    from shortseq_amd._native import NativeError
    seed, ps, U, n, lo, hi = 57, 58, 1 << 15, 300_000, 1, 200
    blob, offs, lens = B.synth_ragged_pool_reads(n, seed, ps, U, lo, hi, device=gpu)
    cuts = [0, n // 9, n // 3, n // 2, 4 * n // 5, n]
    engs = [B.DeviceIngest(gpu) for _ in range(5)]
    try:
        for k, e in enumerate(engs):
            e.count(blob, offs[cuts[k]:cuts[k + 1]], lens[cuts[k]:cuts[k + 1]])
        with pytest.raises(NativeError, match="export"):
            engs[0].reserve_merge(engs[1:])
        for e in engs[1:]:
            e.export()
        with pytest.raises(NativeError, match="distinct"):
            engs[1].reserve_merge([engs[1], engs[2]])
        if reserve:
            engs[0].reserve_merge(engs[1:])
        for k in range(1, 5):
            engs[0].merge(engs[k], cuts[k])
        gl, gc, gw = engs[0].results()
    finally:
        for e in engs:
            e.close()
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    assert gl.tolist() == el.tolist()
    assert gc.tolist() == ec.tolist()
    assert (gw == ew).all()


def test_cross_device_reduce(gpu, golden, tmp_path, oracle):
    """the xGMI path of the reduce (peer access + hipMemcpyPeerAsync on the destination's
    stream) on two real devices; skipped on a one-GPU box."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    seed, ps, U, n, lo, hi = 43, 44, 1 << 12, 60_000, 1, 300
    reads = oracle.ragged_pool_reads(seed, ps, U, 0, n, lo, hi)
    el, ec, ew = oracle.ragged_pool_rows(seed, ps, U, n, lo, hi)
    gl, gc, gw = _rows_of(ShortSeqCounter(reads, device=[0, 1]))
    assert gl.tolist() == el.tolist() and gc.tolist() == ec.tolist() and (gw == ew).all()
    for name, case in sorted(golden["fastq"].items()):
        if case["raises"]:
            continue
        p = tmp_path / (name + ".fq")
        p.write_bytes(bytes.fromhex(case["file_hex"]))
        assert _items(sq.read_and_count_fastq(str(p), device=[0, 1])) == _items(
            sq.read_and_count_fastq(str(p), device="host")), name
