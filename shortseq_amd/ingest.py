"""Ragged read streams on the GPU: ShortSeqCounter lists and FASTQ files.

The reference counts a list of reads (counter.pyx:22-39) or the sequence lines of a FASTQ file
(counter.pyx:57-70 + fast_read.pyx:3-20) one Python object at a time.  Here the reads stay one
byte buffer in HBM plus (offsets, lens):

  * FASTQ: the file is streamed in pinned chunks that end after a newline; ss_fastq_scan /
    ss_fastq_index find the sequence lines on the device (batch.fastq_index).
  * list: the bytes objects are joined once into a pinned buffer and copied up once.

Reads are then split by length (the length is part of the dict key, short_seq_64.pyx:41-44;
short_seq_192.pyx:35-41), each length group gathered into a dense batch on the device
(ss_gather_rows) and counted by one GPU table per length (batch.GpuCounter).  The result is a list
of per-length groups (packed words, counts, global first-occurrence index) from which the Cython
front rebuilds the dict in first-occurrence order.

Errors follow the reference: the FIRST bad read in input order decides the exception (an invalid
base, or a read longer than 1024 nt), raised only after every read before it was checked.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import numpy as np
import torch

from . import batch as B

MAX_NT = B.MAX_NT
TOO_LONG_MSG = f"Sequences longer than {MAX_NT} bases are not supported."   # short_seq.pyx:74


def _pow2_at_least(x: int) -> int:
    return 1 << max(10, int(x - 1).bit_length())


class _TablePool:
    """Device counter tables kept across ShortSeqCounter / read_and_count_fastq calls, keyed by
    (device, capacity): a repeated call reuses a table and its partition workspace (reset is lazy,
    ss_counter_reset) instead of hipMalloc-ing ~100 MB per length group again.  At most
    MAX_BYTES of idle tables are kept (least recently returned are freed first)."""

    MAX_BYTES = 4 << 30

    def __init__(self):
        self.idle: list = []          # [(key, table)] in return order

    @staticmethod
    def _bytes(t: B.GpuCounter) -> int:
        return 32 * t.capacity + 20 * int(B.lib().ss_counter_reserved(t._h))

    def get(self, cap: int, device: torch.device) -> B.GpuCounter:
        key = (device.type, device.index, cap)
        for i in range(len(self.idle) - 1, -1, -1):
            if self.idle[i][0] == key:
                t = self.idle.pop(i)[1]
                t.reset()
                return t
        return B.GpuCounter(cap, device=device)

    def put(self, t: B.GpuCounter) -> None:
        if getattr(t, "_h", None) is None:
            return
        self.idle.append(((t.device.type, t.device.index, t.capacity), t))
        total = sum(self._bytes(x) for _k, x in self.idle)
        while self.idle and total > self.MAX_BYTES:
            _k, old = self.idle.pop(0)
            total -= self._bytes(old)
            old.close()


_pool = _TablePool()


class LengthGroupCounter:
    """One GpuCounter per read length over a ragged stream.  Every read gets a global index (its
    position in the stream); `first` indices returned by finish() are global."""

    MAX_TABLE = 1 << 26      # the partitioned insert's largest table (ss_counter_reserve)

    def __init__(self, device: torch.device, expected_reads: Optional[int] = None):
        self.device = device
        self.expected = expected_reads
        self.tables: dict[int, B.GpuCounter] = {}
        self.rows: dict[int, list] = {}          # L -> [global indices of the rows inserted: a
                                                 # device index tensor, or (start, count) for a range]
        self.nrows: dict[int, int] = {}
        self.empty_count = 0
        self.empty_first: Optional[int] = None
        self.bad_index: Optional[int] = None     # smallest global index of a rejected read
        self.bad_read: Optional[bytes] = None    # its bytes (None: too long)

    def _flag(self, gidx: int, read: Optional[bytes]) -> None:
        if self.bad_index is None or gidx < self.bad_index:
            self.bad_index, self.bad_read = gidx, read

    def _table(self, L: int, m: int) -> B.GpuCounter:
        t = self.tables.get(L)
        if t is None:
            want = max(m, self.expected or 0)
            t = _pool.get(min(self.MAX_TABLE, _pow2_at_least(2 * want)), self.device)
            self.tables[L] = t
            self.rows[L] = []
            self.nrows[L] = 0
        return t

    def _insert(self, t: B.GpuCounter, L: int, rows, m: int, ascii: torch.Tensor, stride: int,
                fetch_row: Callable[[int], int], fetch: Callable[[int], bytes], base: int) -> None:
        row0 = self.nrows[L]
        t.insert(ascii, L, base_index=row0, stride=stride, check_errors=False)
        fb = int(B.first_bad_buffer(self.device).item())
        if fb != -1:
            i = fetch_row(fb)
            self._flag(base + i, fetch(i))
        self.rows[L].append(rows)
        self.nrows[L] = row0 + m

    def add(self, src: torch.Tensor, src_bytes: int, offsets: torch.Tensor, lens, base: int,
            fetch: Callable[[int], bytes], dense: bool = False) -> None:
        """Count reads i (global index base + i): src[offsets[i] : + lens[i]] on the device.
        lens: int64 host array or device tensor (values > 1024, e.g. the FASTQ strlen-underflow
        marker, are rejected as too long).  fetch(i) returns read i's bytes (only called for a
        rejected read).  dense: the reads lie back to back in src (offsets = exclusive cumsum of
        lens), so a batch of one length is counted in place with no gather.

        The split by length runs on the device: a stable sort of the (clamped) lengths, a
        1026-bin histogram and the first read of every group come back in one small copy; each
        group is gathered densely (ss_gather_rows) and counted by its length's table."""
        n = int(lens.shape[0]) if isinstance(lens, torch.Tensor) else int(np.asarray(lens).size)
        if n == 0:
            return
        if self.bad_index is not None and base > self.bad_index:
            return
        d = self.device
        if isinstance(lens, torch.Tensor):
            lens_d = lens.to(d, torch.int64)
        else:
            lens_h = np.asarray(lens, dtype=np.int64)
            L0 = int(lens_h[0])
            if dense and 0 < L0 <= MAX_NT and int(lens_h.min()) == L0 == int(lens_h.max()):
                t = self._table(L0, n)
                ascii = src[:n * L0] if src.dim() == 1 else src.reshape(-1)[:n * L0]
                self._insert(t, L0, (base, n), n, ascii, L0, lambda r: r, fetch, base)
                return
            lens_d = torch.from_numpy(lens_h).to(d, non_blocking=True)
        key = torch.clamp(lens_d, max=MAX_NT + 1)                  # MAX_NT + 1 = rejected (too long)
        order = torch.sort(key, stable=True).indices
        hist = torch.bincount(key, minlength=MAX_NT + 2)
        starts = torch.cumsum(hist, 0) - hist
        nz = torch.nonzero(hist).reshape(-1)
        firsts = order[starts[nz].clamp(max=n - 1)]
        info = torch.stack([nz, hist[nz], starts[nz], firsts], 1).cpu().tolist()   # one sync
        for L, m, st, f0 in info:
            if self.bad_index is not None and base + f0 > self.bad_index:
                continue                                  # nothing here can come first any more
            if L == 0:
                self.empty_count += m
                self.empty_first = base + f0 if self.empty_first is None else min(self.empty_first, base + f0)
                continue
            if L > MAX_NT:
                self._flag(base + f0, None)
                continue
            sel = order[st:st + m]
            rows = B.gather_rows(src, offsets, L, sel=sel, src_bytes=src_bytes)
            t = self._table(L, m)
            self._insert(t, L, sel + base, m, rows, rows.shape[1], lambda r, _s=sel: int(_s[r]), fetch, base)

    def raise_if_bad(self) -> None:
        if self.bad_index is None:
            return
        if self.bad_read is None:
            e = Exception(TOO_LONG_MSG)
            e.read_index = self.bad_index
            raise e
        B.raise_read_error(self.bad_read, self.bad_index)

    def _row_index(self, L: int) -> np.ndarray:
        return np.concatenate([np.arange(r[0], r[0] + r[1], dtype=np.int64) if isinstance(r, tuple)
                               else (r.cpu().numpy() if isinstance(r, torch.Tensor) else r) for r in self.rows[L]])

    def _row_index_dev(self, L: int) -> torch.Tensor:
        d = self.device
        return torch.cat([torch.arange(r[0], r[0] + r[1], dtype=torch.int64, device=d) if isinstance(r, tuple)
                          else torch.as_tensor(r, dtype=torch.int64).to(d) for r in self.rows[L]])

    def finish(self):
        """-> (groups, empty) with groups = [(L, words u64 [m, W], counts, first_global)] in table
        order and empty = (count, first_global) of the zero-length reads (count 0 if none).  Raises
        the reference's exception first if a read was rejected."""
        try:
            self.raise_if_bad()
            groups = []
            for L, t in self.tables.items():
                words, counts, firsts = t.items_words()
                gidx = self._row_index(L)
                groups.append((L, np.ascontiguousarray(words, dtype=np.uint64), counts, gidx[firsts.astype(np.int64)]))
            return groups, (self.empty_count, self.empty_first)
        finally:
            self.close()

    def finish_ordered(self):
        """As finish(), with the dict order worked out on the device: -> (groups, empty, gseq) where
        each group's rows are sorted by global first index and gseq (int16 [total rows], None for
        one group) names the group of every key in global first-occurrence order.  The host rebuild
        then walks every array front to back (a random-order walk over 1M keys costs ~2x the dict
        inserts themselves)."""
        try:
            self.raise_if_bad()
            d = self.device
            groups, dev_firsts = [], []
            for L, t in self.tables.items():
                _, _, words, counts, first, parts = t.extract_words(1)
                m = int(parts.sum().item())
                if t.overflowed():
                    raise RuntimeError("GPU counter table overflowed; use a larger capacity")
                rows = self.rows[L]
                if len(rows) == 1 and isinstance(rows[0], tuple):      # one dense range: no upload
                    gf, perm = torch.sort(first[:m] + rows[0][0])
                else:
                    gf, perm = torch.sort(self._row_index_dev(L)[first[:m]])
                groups.append((L, words[:m][perm].cpu().numpy().view(np.uint64), counts[:m][perm].cpu().numpy(),
                               gf.cpu().numpy()))
                dev_firsts.append(gf)
            gseq = None
            if len(groups) > 1:
                allf = torch.cat(dev_firsts)
                allg = torch.cat([torch.full((f.numel(),), g, dtype=torch.int16, device=d)
                                  for g, f in enumerate(dev_firsts)])
                gseq = allg[torch.sort(allf).indices].cpu().numpy()
            return groups, (self.empty_count, self.empty_first), gseq
        finally:
            self.close()

    def close(self) -> None:
        for t in self.tables.values():
            _pool.put(t)
        self.tables = {}


_pinned: Optional[torch.Tensor] = None     # grow-only staging buffer (hipHostMalloc is not free)
_dev_bufs: dict = {}                       # device -> grow-only device staging buffer


def _device_staging(nbytes: int, device: torch.device) -> torch.Tensor:
    """Grow-only device buffer per device for the staged reads (a fresh 32-MB+ tensor per call
    measured 15-25 ms in the allocator on the MI355X box; the cached one copies in ~1 ms)."""
    buf = _dev_bufs.get(device)
    if buf is None or buf.numel() < nbytes:
        buf = _dev_bufs[device] = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
    return buf


def _staging(nbytes: int) -> torch.Tensor:
    global _pinned
    if _pinned is None or _pinned.numel() < nbytes:
        _pinned = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8).pin_memory()
    return _pinned


def count_list(reads: list, lens_np: np.ndarray, device: torch.device, staged: bool = False) -> "LengthGroupCounter":
    """ShortSeqCounter(list_of_bytes) on the GPU: the reads concatenated into pinned staging (by
    the caller when staged=True: the Cython front copies each bytes object straight into
    _staging(total)), one H2D copy."""
    gc = LengthGroupCounter(device)
    n = len(reads)
    total = int(lens_np.sum())
    if n == 0:
        return gc
    host = _staging(total)
    if total and not staged:
        host.numpy()[:total] = np.frombuffer(b"".join(reads), dtype=np.uint8)
    src = _device_staging(max(total, 1), device)[:max(total, 1)]
    src.copy_(host[:max(total, 1)], non_blocking=True)
    torch.cuda.current_stream(device).synchronize()      # the staging buffer is reused next call
    offs_np = np.zeros(n, dtype=np.int64)
    np.cumsum(lens_np[:-1], out=offs_np[1:])
    offs = torch.from_numpy(offs_np).to(device, non_blocking=True)
    gc.add(src, total, offs, lens_np, 0, lambda i: bytes(reads[i]), dense=True)
    return gc


DEFAULT_CHUNK = 1 << 30


_READ_THREADS = int(os.environ.get("SHORTSEQ_READ_THREADS", "8"))
_read_pool = None


def _pread_full(fd: int, mv: memoryview, pos: int) -> int:
    """Read len(mv) bytes at file offset pos (fewer only at EOF)."""
    got = 0
    while got < len(mv):
        k = os.preadv(fd, [mv[got:]], pos + got)
        if k == 0:
            break
        got += k
    return got


def _read_into(fd: int, mv: memoryview, pos: int, size: int) -> int:
    """Fill mv from file offset pos with up to _READ_THREADS concurrent preads (one core copies
    ~5 GB/s out of the page cache; the pinned staging buffer takes it faster).  Returns the bytes
    read = min(len(mv), size - pos)."""
    global _read_pool
    want = max(0, min(len(mv), size - pos))
    if want < (32 << 20) or _READ_THREADS <= 1:
        return _pread_full(fd, mv[:want], pos)
    if _read_pool is None:
        from concurrent.futures import ThreadPoolExecutor
        _read_pool = ThreadPoolExecutor(_READ_THREADS, thread_name_prefix="shortseq-read")
    per = ((want + _READ_THREADS - 1) // _READ_THREADS + (1 << 20) - 1) & ~((1 << 20) - 1)
    futs = [_read_pool.submit(_pread_full, fd, mv[a:min(want, a + per)], pos + a) for a in range(0, want, per)]
    got = sum(f.result() for f in futs)
    if got != want:
        raise OSError(f"short read: {got} of {want} bytes at offset {pos}")
    return got


def count_fastq(path: str, device: torch.device, chunk_bytes: int = DEFAULT_CHUNK):
    """read_and_count_fastq on the GPU: -> (LengthGroupCounter, number of sequence lines).
    The file is read in chunks of up to chunk_bytes (parallel preads into the grow-only pinned
    staging buffer) that end right after a newline; each chunk is copied up once and indexed,
    split by length and counted on the device."""
    size = os.path.getsize(path)
    cap = max(16, min(chunk_bytes, size + 16))
    if cap >= (1 << 32):
        raise ValueError("chunk_bytes must be < 4 GiB")
    pinned = _staging(cap)[:cap]
    hv = pinned.numpy()
    dbuf = _device_staging(cap, device)
    est_reads = None
    gc = LengthGroupCounter(device)
    line0 = read0 = carry = pos = 0
    fd = os.open(path, os.O_RDONLY)
    try:
        while True:
            got = _read_into(fd, memoryview(hv)[carry:], pos, size)
            pos += got
            n = carry + got
            at_eof = got == 0 or pos >= size
            if n == 0:
                break
            if at_eof:
                use = n
            else:
                use = 0
                lo = n
                while use == 0 and lo > 0:            # last newline of the chunk, searched backwards
                    a = max(0, lo - (1 << 20))
                    k = hv[a:lo].tobytes().rfind(b"\n")
                    if k >= 0:
                        use = a + k + 1
                    lo = a
                if use == 0:                          # one line fills the chunk: grow the buffers
                    if 2 * cap >= (1 << 32):
                        raise ValueError("a FASTQ line is longer than 2 GiB")
                    cap *= 2
                    grown = torch.empty(cap, dtype=torch.uint8).pin_memory()
                    grown.numpy()[:n] = hv[:n]
                    pinned, hv = grown, grown.numpy()
                    dbuf = torch.empty(cap, dtype=torch.uint8, device=device)
                    carry = n
                    continue
            dbuf[:use].copy_(pinned[:use], non_blocking=True)
            offs, lens, nl = B.fastq_index(dbuf, use, line0=line0, at_eof=at_eof)
            nrec = int(lens.shape[0])
            if est_reads is None and not at_eof:
                est_reads = int(nrec * size / max(1, use)) + 1
                gc.expected = est_reads

            def fetch(i, _o=offs, _l=lens, _d=dbuf):
                o = int(_o[i].item())
                return _d[o:o + int(_l[i].item())].cpu().numpy().tobytes()

            gc.add(dbuf, use, offs, lens, read0, fetch)
            read0 += nrec
            line0 += nl
            if at_eof or gc.bad_index is not None:
                break
            carry = n - use
            torch.cuda.current_stream(device).synchronize()   # the H2D of this chunk has left hv
            hv[:carry] = hv[use:n].copy()
    finally:
        os.close(fd)
    torch.cuda.current_stream(device).synchronize()           # the staging buffer is reused next call
    return gc, read0
