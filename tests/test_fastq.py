"""FASTQ ingest: read_and_count_fastq (counter.pyx:57-70, fast_read.pyx:3-20).

Golden cases: tests/golden/golden_cases.json["fastq"], the unmodified reference's
read_and_count_fastq on each file (tests/golden/gen_golden.py --only-fastq).  The reference keys
ShortSeqVar objects by heap pointer, so equal reads > 96 nt stay separate entries
there; this build merges them by content (documented deviation), and the expected items are the
golden items merged the same way (counts summed, first occurrence kept).

CPU: the oracle's line selection (oracle/ss_oracle.c ora_fastq_index) + counter oracle reproduce
the golden items; the host front does too.  GPU: ss_fastq_index / ss_gather_rows against the
oracle on the fixtures, on random edge-case files and over random chunkings; the GPU
read_and_count_fastq against the golden items; the partitioned counter on packed keys (L not 16/32).
"""
import random

import numpy as np
import pytest

import shortseq_amd as sq

TOO_LONG = "Sequences longer than 1024 bases are not supported."


def _merged_golden(case):
    """Golden items with the reference's pointer-keyed ShortSeqVar duplicates merged (Q6)."""
    out, pos = [], {}
    for it in case["items"]:
        key = (it["length"], it["str"])
        if key in pos:
            out[pos[key]][3] += it["count"]
        else:
            pos[key] = len(out)
            out.append([it["class"], it["str"], it["length"], it["count"]])
    return [tuple(x) for x in out]


def _items(c):
    return [(type(k).__name__, str(k), len(k), v) for k, v in c.items()]


def _oracle_items(oracle, data: bytes):
    """Oracle line selection + counter oracle -> merged items, or ('raises', message)."""
    offs, lens = oracle.fastq_index(data)
    reads = []
    for o, ln in zip(offs, lens):
        if ln > 1024:
            return ("raises", TOO_LONG)
        reads.append(data[int(o):int(o) + int(ln)])
    try:
        res = oracle.count(reads)
    except ValueError as e:
        kind, ri, bo, nb = e.args[0]
        if kind == 2:
            return ("raises", TOO_LONG)
        return ("raises", "Unsupported base character: " + reads[ri][bo:bo + nb].decode("ascii"))
    items = []
    for words, L, c, _f in res:
        cls = "ShortSeq64" if L <= 32 else ("ShortSeq192" if L <= 96 else "ShortSeqVar")
        s = str(sq.from_words(list(words), L)) if L else ""
        items.append((cls, s, L, c))
    return items


def _cases(golden):
    return sorted(golden["fastq"].items())


def test_oracle_fastq_pinned_to_reference(oracle, golden):
    assert len(golden["fastq"]) >= 10
    for name, case in _cases(golden):
        data = bytes.fromhex(case["file_hex"])
        got = _oracle_items(oracle, data)
        if case["raises"]:
            assert got == ("raises", case["message"]), name
        else:
            assert got == _merged_golden(case), name


def test_host_front_fastq_golden(golden, tmp_path, capsys):
    for name, case in _cases(golden):
        p = tmp_path / (name + ".fq")
        p.write_bytes(bytes.fromhex(case["file_hex"]))
        if case["raises"]:
            with pytest.raises(Exception) as ei:
                sq.read_and_count_fastq(str(p), device="host")
            assert str(ei.value) == case["message"], name
        else:
            c = sq.read_and_count_fastq(str(p), device="host")
            assert _items(c) == _merged_golden(case), name
    assert "total seqs" in capsys.readouterr().out


def _random_fastq(rng, nrec, edge=True):
    """Random FASTQ bytes: variable headers / lengths, optional edge cases (empty seq lines, NULs,
    missing final newline)."""
    parts = []
    for i in range(nrec):
        L = rng.choice([0, 1, 15, 16, 20, 31, 32, 33, 64, 96, 100, 150]) if edge else rng.choice([20, 32, 96])
        seq = bytes(rng.choice(b"ACGT") for _ in range(L))
        if edge and rng.random() < 0.01 and L > 2:
            k = rng.randrange(L)
            seq = seq[:k] + b"\x00" + seq[k + 1:]
        hdr = b"@read_%d" % i + b"x" * rng.randrange(0, 40)
        parts.append(hdr + b"\n" + seq + b"\n+\n" + b"I" * len(seq) + b"\n")
    data = b"".join(parts)
    if edge and rng.random() < 0.5:
        data = data[:-1]          # drop the final newline
    return data


def _gpu_index(B, torch, dev, data, cuts=(), **kw):
    """Index `data` on the device in chunks ending right after the newlines at `cuts` (byte
    positions); returns global (offsets, lens)."""
    bounds = [0] + sorted(cuts) + [len(data)]
    offs_all, lens_all = [], []
    line0 = 0
    for a, b in zip(bounds[:-1], bounds[1:]):
        chunk = data[a:b]
        buf = torch.tensor(np.frombuffer(chunk, np.uint8) if chunk else np.zeros(0, np.uint8),
                           dtype=torch.uint8, device=dev)
        offs, lens, nl = B.fastq_index(buf, len(chunk), line0=line0, at_eof=(b == len(data)), **kw)
        offs_all.append(offs.cpu().numpy().astype(np.uint64) + np.uint64(a))
        lens_all.append(lens.cpu().numpy().astype(np.uint32))
        line0 += nl
    return np.concatenate(offs_all), np.concatenate(lens_all)


@pytest.mark.gpu
@pytest.mark.parametrize("onepass", [True, False])
def test_fastq_index_gpu_matches_oracle(gpu, oracle, golden, onepass):
    import torch
    import shortseq_amd.batch as B
    files = [bytes.fromhex(c["file_hex"]) for _n, c in _cases(golden)]
    rng = random.Random(11)
    files += [_random_fastq(rng, n) for n in (1, 2, 3, 7, 500, 3000)]
    files += [b"\n", b"\n\n", b"\n\n\n", b"a\nb\nc\nd\ne\nf", b"x" * 20000 + b"\n" + b"AC" * 9000 + b"\n"]
    for data in files:
        eo, el = oracle.fastq_index(data)
        go, gl = _gpu_index(B, torch, gpu, data, onepass=onepass)
        assert np.array_equal(go, eo) and np.array_equal(gl, el), data[:60]
        # chunked: random cut points right after newlines
        nls = [i + 1 for i in range(len(data)) if data[i] == 10 and i + 1 < len(data)]
        for _ in range(3):
            cuts = rng.sample(nls, min(len(nls), rng.randrange(1, 6))) if nls else []
            go, gl = _gpu_index(B, torch, gpu, data, cuts, onepass=onepass)
            assert np.array_equal(go, eo) and np.array_equal(gl, el), (data[:60], cuts)


@pytest.mark.gpu
@pytest.mark.parametrize("onepass", [True, False])
def test_fastq_index_gpu_large(gpu, oracle, onepass):
    """A multi-tile file (many 16-KiB tiles) against the oracle."""
    import torch
    import shortseq_amd.batch as B
    rng = random.Random(12)
    data = _random_fastq(rng, 40_000)
    eo, el = oracle.fastq_index(data)
    go, gl = _gpu_index(B, torch, gpu, data, onepass=onepass)
    assert len(eo) == 40_000 and np.array_equal(go, eo) and np.array_equal(gl, el)


@pytest.mark.gpu
def test_fastq_index_onepass_capacity_retry(gpu, oracle):
    """A capacity guess below the chunk's sequence lines: the one-pass call is repeated exactly."""
    import torch
    import shortseq_amd.batch as B
    rng = random.Random(14)
    data = _random_fastq(rng, 5000)
    eo, el = oracle.fastq_index(data)
    for cap in (1, 17, 4999):
        go, gl = _gpu_index(B, torch, gpu, data, max_reads=cap)
        assert np.array_equal(go, eo) and np.array_equal(gl, el), cap
    # 3 MiB of empty lines with a bound of 1: the per-shard staging regions run full (doubling path)
    data = b"\n" * (3 << 20) + b"ACGT\n"
    eo, el = oracle.fastq_index(data)
    go, gl = _gpu_index(B, torch, gpu, data, max_reads=1)
    assert np.array_equal(go, eo) and np.array_equal(gl, el)


@pytest.mark.gpu
@pytest.mark.parametrize("onepass", [True, False])
def test_fastq_index_nul_list_overflow(gpu, oracle, onepass):
    """More NUL-holding sequence lines than the NUL list holds (65,536): every line is re-measured;
    NULs at the line start (strlen 0), inside, and doubled, plus NULs outside sequence lines."""
    import torch
    import shortseq_amd.batch as B
    rng = np.random.default_rng(15)
    parts = []
    for i in range(70_000):
        L = int(rng.integers(3, 40))
        seq = bytearray(rng.choice(np.frombuffer(b"ACGT", np.uint8), L).tobytes())
        k = int(rng.integers(0, L))
        seq[k] = 0
        if i % 3 == 0:
            seq[min(L - 1, k + 1)] = 0
        hdr = b"@r\x00%d" % i if i % 5 == 0 else b"@r%d" % i
        parts.append(hdr + b"\n" + bytes(seq) + b"\n+\n" + b"I" * L + b"\n")
    data = b"".join(parts)
    eo, el = oracle.fastq_index(data)
    go, gl = _gpu_index(B, torch, gpu, data, onepass=onepass)
    assert len(eo) == 70_000 and np.array_equal(go, eo) and np.array_equal(gl, el)


@pytest.mark.gpu
def test_fastq_index_onepass_scattered_nuls(gpu, oracle):
    """~1,000 stray NULs over a 4-MB file (more than the short list, fewer than the NUL
    list holds): only the lines overlapping a 1-KiB sub-block with a NUL are byte-scanned.  NULs in
    sequence lines (first byte, inside, last byte), in headers and quality lines, and long lines that
    cross sub-block and 32-KiB tile boundaries; the result equals the oracle's, whole and chunked."""
    import torch
    import shortseq_amd.batch as B
    rng = np.random.default_rng(16)
    parts = []
    for i in range(20_000):
        L = int(rng.integers(1, 400)) if i % 97 else 3000
        seq = bytearray(rng.choice(np.frombuffer(b"ACGT", np.uint8), L).tobytes())
        qual = bytearray(b"I" * L)
        hdr = bytearray(b"@r%d" % i)
        u = rng.random()
        if u < 0.03:
            seq[int(rng.choice([0, L // 2, L - 1]))] = 0
        elif u < 0.04:
            qual[int(rng.integers(0, L))] = 0
        elif u < 0.05:
            hdr[1] = 0
        parts.append(bytes(hdr) + b"\n" + bytes(seq) + b"\n+\n" + bytes(qual) + b"\n")
    data = b"".join(parts)
    assert 100 < data.count(b"\x00") < 65_536
    eo, el = oracle.fastq_index(data)
    go, gl = _gpu_index(B, torch, gpu, data, onepass=True)
    assert np.array_equal(go, eo) and np.array_equal(gl, el)
    nls = [i + 1 for i in range(len(data)) if data[i] == 10 and i + 1 < len(data)]
    go, gl = _gpu_index(B, torch, gpu, data, sorted(random.Random(17).sample(nls, 5)), onepass=True)
    assert np.array_equal(go, eo) and np.array_equal(gl, el)


@pytest.mark.gpu
def test_gather_rows_gpu(gpu):
    import torch
    import shortseq_amd.batch as B
    rng = np.random.default_rng(13)
    blob = rng.integers(0, 256, size=100_003, dtype=np.uint8)
    src = torch.from_numpy(blob).to(gpu)
    for L in (1, 3, 15, 16, 17, 32, 33, 100, 1024):
        offs = rng.integers(0, len(blob) - L + 1, size=777).astype(np.int64)
        offs[-1] = len(blob) - L                      # a row that ends exactly at the buffer end
        sel = rng.permutation(777)[:500].astype(np.int64)
        out = B.gather_rows(src, torch.from_numpy(offs).to(gpu), L, sel=torch.from_numpy(sel).to(gpu))
        got = out.cpu().numpy()
        S = (L + 15) // 16 * 16
        assert got.shape == (500, S)
        exp = np.stack([blob[offs[s]:offs[s] + L] for s in sel])
        assert np.array_equal(got[:, :L], exp), L
        assert (got[:, L:] == ord("A")).all()


@pytest.mark.gpu
def test_fastq_golden_gpu(gpu, golden, tmp_path, capsys):
    for name, case in _cases(golden):
        p = tmp_path / (name + ".fq")
        p.write_bytes(bytes.fromhex(case["file_hex"]))
        for chunk in (0, 96):              # default chunks, and tiny ones (every chunk-boundary path)
            if chunk and len(case["file_hex"]) <= 200:
                continue
            if case["raises"]:
                with pytest.raises(Exception) as ei:
                    sq.read_and_count_fastq(str(p), device="cuda", _chunk_bytes=chunk)
                assert str(ei.value) == case["message"], (name, chunk)
                continue
            c = sq.read_and_count_fastq(str(p), device="cuda", _chunk_bytes=chunk)
            assert _items(c) == _merged_golden(case), (name, chunk)
    assert "total seqs" in capsys.readouterr().out


@pytest.mark.gpu
def test_fastq_gpu_random_vs_host(gpu, tmp_path):
    rng = random.Random(14)
    data = _random_fastq(rng, 20_000)
    data = data.replace(b"\x00", b"A")              # keep it valid
    p = tmp_path / "r.fq"
    p.write_bytes(data)
    h = sq.read_and_count_fastq(str(p), device="host")
    d = sq.read_and_count_fastq(str(p), device="cuda")
    assert _items(d) == _items(h)


@pytest.mark.gpu
@pytest.mark.parametrize("L", [20, 31, 17])
def test_counter_packed_keys_partitioned(gpu, oracle, L):
    """L not in {16, 32}: the batch is packed into the key workspace, then partitioned."""
    import torch
    import shortseq_amd.batch as B
    n = 200_000
    pool = oracle.gen_pool_reads(21, 22, 5000, 0, n, L)
    c = B.GpuCounter(1 << 14, device=gpu)
    try:
        c.insert(torch.from_numpy(pool).to(gpu).view(n, L), L, partitioned=True)
        assert int(B.lib().ss_counter_reserved(c._h)) >= n
        k, cnt, f = c.items_sorted()
    finally:
        c.close()
    reads = [pool[i * L:(i + 1) * L].tobytes() for i in range(n)]
    exp = oracle.count(reads)
    assert [int(x) for x in k] == [w[0] for (w, _L, _c, _f) in exp]
    assert [int(x) for x in cnt] == [cc for (_w, _L, cc, _f) in exp]
    assert [int(x) for x in f] == [ff for (_w, _L, _c, ff) in exp]


@pytest.mark.gpu
def test_fastq_gpu_many_lengths_many_chunks(gpu, tmp_path):
    """a multi-chunk FASTQ with many read lengths (1..300 nt, every chunk a mix) counted
    through small chunks: equals the host path; per-length tables follow each length's own share."""
    rng = random.Random(21)
    recs = []
    for i in range(30_000):
        L = rng.randint(1, 300)
        s = "".join(rng.choice("ACGT") for _ in range(L)) if rng.random() < 0.5 else "ACGT" * (L // 4) + "A" * (L % 4)
        recs.append(f"@r{i}\n{s}A\n+\n{'I' * (L + 1)}\n")
    p = tmp_path / "mix.fq"
    p.write_text("".join(recs))
    h = sq.read_and_count_fastq(str(p), device="host")
    for chunk in (1 << 16, 1 << 20):
        d = sq.read_and_count_fastq(str(p), device="cuda", _chunk_bytes=chunk)
        assert _items(d) == _items(h), chunk


@pytest.mark.gpu
def test_fastq_gpu_table_growth(gpu, tmp_path):
    """A length whose distinct keys keep arriving after the first chunk: its table (sized from the first
    chunk's rows) grows by extract + merge and keeps every count and first occurrence."""
    rng = random.Random(22)
    pool = ["".join(rng.choice("ACGT") for _ in range(20)) for _ in range(200)]
    recs = [f"@a{i}\n{rng.choice(pool)}A\n+\n{'I' * 21}\n" for i in range(3000)]          # few keys first
    recs += [f"@b{i}\n{''.join(rng.choice('ACGT') for _ in range(20))}A\n+\n{'I' * 21}\n" for i in range(150_000)]
    recs += [f"@c{i}\n{rng.choice(pool)}A\n+\n{'I' * 21}\n" for i in range(3000)]
    p = tmp_path / "grow.fq"
    p.write_text("".join(recs))
    h = sq.read_and_count_fastq(str(p), device="host")
    d = sq.read_and_count_fastq(str(p), device="cuda", _chunk_bytes=1 << 17)
    assert _items(d) == _items(h)


@pytest.mark.gpu
def test_fastq_gpu_table_growth_multiword(gpu, tmp_path):
    """an L > 32 length with a few reads near the end of the first chunk, then many
    distinct keys in later chunks: its multi-word table grows (extract_words + merge_words) instead of
    overflowing, and the dict equals the host path."""
    rng = random.Random(23)
    recs = [f"@a{i}\n{''.join(rng.choice('ACGT') for _ in range(20))}A\n+\nI\n" for i in range(2000)]
    for L in (40, 150):
        recs += [f"@x{L}_{i}\n{''.join(rng.choice('ACGT') for _ in range(L))}A\n+\nI\n" for i in range(3)]
    for L in (40, 150):
        recs += [f"@y{L}_{i}\n{''.join(rng.choice('ACGT') for _ in range(L))}A\n+\nI\n" for i in range(40_000)]
    p = tmp_path / "growmw.fq"
    p.write_text("".join(recs))
    h = sq.read_and_count_fastq(str(p), device="host")
    d = sq.read_and_count_fastq(str(p), device="cuda", _chunk_bytes=1 << 16)
    assert _items(d) == _items(h)


def test_fastq_split_host(tmp_path):
    """ss_fastq_split (host): every range starts at the file start or right after a newline, the
    ranges tile the file, and line0 = the newlines before each range."""
    import ctypes as C
    from shortseq_amd import _native
    lib = _native.lib()
    rng = random.Random(24)
    for trial in range(6):
        data = b"".join(b"@r%d\n%s\n+\n%s\n" % (i, b"ACGT" * rng.randint(0, 60), b"I" * rng.randint(0, 3))
                        for i in range(rng.choice([0, 1, 5, 2000])))
        if trial == 5:
            data += b"@last\nACG"           # no trailing newline
        p = tmp_path / f"s{trial}.fq"
        p.write_bytes(data)
        for parts in (1, 2, 3, 8, 17):
            b = (C.c_uint64 * (parts + 1))()
            l0 = (C.c_uint64 * (parts + 1))()
            assert lib.ss_fastq_split(str(p).encode(), parts, C.addressof(b), C.addressof(l0)) == 0
            bs = list(b)
            assert bs[0] == 0 and bs[-1] == len(data) and bs == sorted(bs)
            for k in range(parts):
                assert bs[k] in (0, len(data)) or data[bs[k] - 1:bs[k]] == b"\n", (trial, parts, k)
                assert l0[k] == data[:bs[k]].count(b"\n"), (trial, parts, k)


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [0, 4096])
def test_fastq_gpu_stage_split(gpu, tmp_path, chunk):
    """The engine's FASTQ stage split (ss_ingest_fastq_stages via
    _shortseq.fastq_stage_times): one entry per device, every stage timed, and the H2D copies moved
    the file once (one chunk) or once plus the carried partial lines (many chunks); the counts
    equal the host path's."""
    from shortseq_amd import _shortseq
    rng = random.Random(23)
    data = _random_fastq(rng, 5000, edge=False)
    p = tmp_path / "s.fq"
    p.write_bytes(data)
    d = sq.read_and_count_fastq(str(p), device="cuda", _chunk_bytes=chunk)
    h = sq.read_and_count_fastq(str(p), device="host")
    assert _items(d) == _items(h)
    st = _shortseq.fastq_stage_times()
    assert len(st) == 1
    s0 = st[0]
    for k in ("read_ms", "h2d_dev_ms", "index_ms", "count_ms", "finish_ms", "reduce_and_dict_ms", "total_ms"):
        assert s0[k] > 0.0, k
    if chunk == 0:
        assert s0["h2d_bytes"] == len(data)
    else:
        assert len(data) <= s0["h2d_bytes"] < 2 * len(data)


@pytest.mark.gpu
def test_fastq_gpu_reader_ring(gpu, tmp_path):
    """The reader ring (a range longer than one chunk: chunk k + 1 read and copied while chunk k is
    counted): header lines longer than the chunk (a slot grows while the other slot is in use), many
    chunks, and a rejected read early in the file (the caller stops while the reader is a chunk
    ahead): the dict, or the error, equals the host path's."""
    rng = random.Random(31)
    recs = []
    for i in range(4000):
        L = rng.randint(15, 40)
        hdr = f"@r{i}" + ("x" * rng.randint(2000, 6000) if i % 500 == 7 else "")
        s = "".join(rng.choice("ACGT") for _ in range(L))
        recs.append(f"{hdr}\n{s}\n+\n{'I' * L}\n")
    p = tmp_path / "ring.fq"
    p.write_text("".join(recs))
    h = sq.read_and_count_fastq(str(p), device="host")
    for chunk in (1024, 4096, 1 << 16):
        d = sq.read_and_count_fastq(str(p), device="cuda", _chunk_bytes=chunk)
        assert _items(d) == _items(h), chunk
    recs[300] = "@bad\nACGTZACGT\n+\nIIIIIIIII\n"
    p.write_text("".join(recs))
    with pytest.raises(Exception) as eh:
        sq.read_and_count_fastq(str(p), device="host")
    for chunk in (1024, 1 << 16):
        with pytest.raises(type(eh.value)) as ed:
            sq.read_and_count_fastq(str(p), device="cuda", _chunk_bytes=chunk)
        assert str(ed.value) == str(eh.value), chunk
