"""Batch API on the GPU — torch CUDA tensors in, torch CUDA tensors out, one HIP kernel per call.

This is the data-parallel hot path behind the C ABI in
include/shortseq_amd.h.  PyTorch only provides device memory, streams and the caching allocator;
every byte of encode / decode / hamming / counting is done by the HIP kernels in csrc/.

Packed words are returned as int64 tensors holding the raw 64-bit patterns (view them as uint64 on
the host: ``t.cpu().numpy().view(np.uint64)``).  Layout: read i -> words[i, 0:wpr], nt j in word
j // 32 at bits 2*(j % 32), codes A=0 C=1 T=2 G=3 (README.md:101-112).

Errors: a batch containing a read the reference would reject raises the reference's exception for
the FIRST such read in input order (the one ShortSeqCounter's loop, counter.pyx:22-29, would hit):
``Exception("Unsupported base character: X")`` / ``UnicodeDecodeError`` / ``Exception("Sequences
longer than 1024 bases are not supported.")``, with ``.read_index`` set.  The kernels only flag the
read; its exact message comes from re-scanning that one read with the host codec.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np
import torch

from ._native import SS_EFULL, NativeError, SsErr, check, lib

MAX_NT = 1024
_NO_BAD = -1  # UINT64_MAX viewed as int64

__all__ = ["words_for", "wpr_for", "encode", "encode_var", "decode", "decode_var", "hamming_ref",
           "hamming_pair", "encode_hamming_ref", "synth_reads", "synth_pool_reads", "synth_zipf_reads", "zipf_cdf",
           "GpuCounter",
           "raise_read_error", "first_bad_buffer", "fastq_index", "gather_rows", "slice_fixed",
           "slice_var", "hamming_all_pairs", "HostStager", "host_stager", "encode_host", "decode_host"]


def words_for(L: int) -> int:
    """ceil(L / 32): util.pyx:30-33."""
    return (L + 31) // 32


def wpr_for(L: int) -> int:
    """Words per read in batch layouts: 1 for L <= 32 (ShortSeq64 keeps one word even for L = 0)."""
    return max(1, words_for(L))


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _require_cuda(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA (HIP) tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


_first_bad_cache: dict = {}


def first_bad_buffer(dev: torch.device) -> torch.Tensor:
    """Per-device 1-word scratch the kernels atomicMin the first invalid read index into."""
    key = (dev.type, dev.index)
    t = _first_bad_cache.get(key)
    if t is None:
        t = torch.empty(1, dtype=torch.int64, device=dev)
        _first_bad_cache[key] = t
    return t


def raise_read_error(read: bytes, read_index: int) -> None:
    """Raise exactly what shortseq.pack(read) raises in the reference (SURVEY §8 error contract)."""
    if len(read) > MAX_NT:
        e = Exception(f"Sequences longer than {MAX_NT} bases are not supported.")  # short_seq.pyx:74
        e.read_index = read_index
        raise e
    buf = np.frombuffer(read, dtype=np.uint8) if read else np.zeros(1, np.uint8)
    words = np.zeros(32, dtype=np.uint64)
    err = SsErr()
    rc = lib().ss_host_encode(buf.ctypes.data, len(read), words.ctypes.data, C.byref(err))
    if rc == 0:
        raise AssertionError(f"read {read_index} was flagged by the GPU but encodes on the host")
    bad = read[err.byte_offset: err.byte_offset + err.nbytes]
    # short_seq_64.pyx:105 / util.pyx:115,137 — PyUnicode_DecodeASCII of the byte(s); a non-ASCII
    # byte makes that decode itself raise UnicodeDecodeError, as in the reference.
    e = Exception(f"Unsupported base character: {bad.decode('ascii')}")
    e.read_index = read_index
    raise e


def _check_first_bad(fb: torch.Tensor, fetch_read) -> None:
    v = int(fb.item())
    if v != _NO_BAD:
        raise_read_error(fetch_read(v), v)


def _as_rows(ascii: torch.Tensor, L: Optional[int], stride: Optional[int]):
    _require_cuda(ascii, "ascii")
    if ascii.dtype != torch.uint8:
        raise TypeError("ascii must be a uint8 tensor")
    if ascii.dim() == 2:
        n, width = ascii.shape
        L = width if L is None else L
        stride = width if stride is None else stride
        if stride != width:
            raise ValueError("for a 2-D ascii tensor the stride is its row width")
    else:
        if L is None:
            raise ValueError("L is required for a flat ascii tensor")
        stride = L if stride is None else stride
        n = ascii.numel() // stride if stride else 0
    if not (1 <= L <= MAX_NT):
        if L > MAX_NT:
            raise Exception(f"Sequences longer than {MAX_NT} bases are not supported.")
        raise ValueError("L must be >= 1 (empty reads are the empty singleton, no kernel needed)")
    if stride < L:
        raise ValueError("stride < L")
    return n, L, stride


def _fetch_row(ascii: torch.Tensor, stride: int, L: int):
    flat = ascii.reshape(-1)
    return lambda i: bytes(flat[i * stride: i * stride + L].cpu().numpy())


def encode(ascii: torch.Tensor, L: Optional[int] = None, *, stride: Optional[int] = None,
           wpr: Optional[int] = None, out: Optional[torch.Tensor] = None,
           check_errors: bool = True) -> torch.Tensor:
    """Encode a fixed-length batch (one ss_encode_fixed launch).  ascii: uint8 [n, L] or flat."""
    n, L, stride = _as_rows(ascii, L, stride)
    wpr = wpr_for(L) if wpr is None else wpr
    dev = ascii.device
    if out is None:
        out = torch.empty((n, wpr), dtype=torch.int64, device=dev)
    fb = first_bad_buffer(dev)
    check(lib().ss_encode_fixed(ascii.data_ptr(), n, L, stride, out.data_ptr(), wpr, fb.data_ptr(),
                                _stream(dev)), "ss_encode_fixed")
    if check_errors:
        _check_first_bad(fb, _fetch_row(ascii, stride, L))
    return out


def encode_var(blob: torch.Tensor, offsets: torch.Tensor, lens: torch.Tensor, *,
               wpr: Optional[int] = None, out: Optional[torch.Tensor] = None,
               check_errors: bool = True) -> torch.Tensor:
    """Encode a ragged batch: read i = blob[offsets[i] : offsets[i] + lens[i]] (0..1024 nt)."""
    for t, nm in ((blob, "blob"), (offsets, "offsets"), (lens, "lens")):
        _require_cuda(t, nm)
    if offsets.dtype != torch.int64 or lens.dtype != torch.int32 or blob.dtype != torch.uint8:
        raise TypeError("blob uint8, offsets int64, lens int32 expected")
    n = lens.numel()
    if wpr is None:
        wpr = wpr_for(min(int(lens.max().item()), MAX_NT)) if n else 1
    dev = blob.device
    if out is None:
        out = torch.empty((n, wpr), dtype=torch.int64, device=dev)
    fb = first_bad_buffer(dev)
    check(lib().ss_encode_var(blob.data_ptr(), offsets.data_ptr(), lens.data_ptr(), n, out.data_ptr(),
                              wpr, fb.data_ptr(), _stream(dev)), "ss_encode_var")
    if check_errors:
        def fetch(i):
            o, ln = int(offsets[i].item()), int(lens[i].item())
            return bytes(blob[o:o + ln].cpu().numpy())
        _check_first_bad(fb, fetch)
    return out


def decode(words: torch.Tensor, L: int, *, wpr: Optional[int] = None,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Packed words [n, wpr] -> ASCII uint8 [n, L] (one ss_decode_fixed launch)."""
    _require_cuda(words, "words")
    wpr = words.shape[1] if words.dim() == 2 else (wpr_for(L) if wpr is None else wpr)
    n = words.numel() // wpr
    dev = words.device
    if out is None:
        out = torch.empty((n, L), dtype=torch.uint8, device=dev)
    check(lib().ss_decode_fixed(words.data_ptr(), n, L, wpr, out.data_ptr(), L, _stream(dev)),
          "ss_decode_fixed")
    return out


def decode_var(words: torch.Tensor, lens: torch.Tensor, offsets: torch.Tensor,
               out_bytes: Optional[int] = None) -> torch.Tensor:
    """Ragged decode into one blob; read i lands at blob[offsets[i] : offsets[i] + lens[i]]."""
    _require_cuda(words, "words")
    n, wpr = words.shape
    dev = words.device
    total = out_bytes if out_bytes is not None else (
        int((offsets[-1] + lens[-1]).item()) if n else 0)
    out = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    check(lib().ss_decode_var(words.data_ptr(), lens.data_ptr(), n, wpr, out.data_ptr(),
                              offsets.data_ptr(), _stream(dev)), "ss_decode_var")
    return out[:total]


def hamming_ref(words: torch.Tensor, L: int, ref: torch.Tensor) -> torch.Tensor:
    """Per-read __xor__ distance to one packed reference read -> int32 [n]."""
    _require_cuda(words, "words")
    n, wpr = words.shape
    out = torch.empty(n, dtype=torch.int32, device=words.device)
    ref = ref.to(words.device).contiguous()
    check(lib().ss_hamming_ref(words.data_ptr(), n, L, wpr, ref.data_ptr(), out.data_ptr(),
                               _stream(words.device)), "ss_hamming_ref")
    return out


def hamming_pair(a: torch.Tensor, b: torch.Tensor, L: int) -> torch.Tensor:
    """Element-wise a[i] ^ b[i] (ShortSeq.__xor__) -> int32 [n]."""
    _require_cuda(a, "a")
    _require_cuda(b, "b")
    if a.shape != b.shape:
        raise ValueError("a and b must have the same shape")
    n, wpr = a.shape
    out = torch.empty(n, dtype=torch.int32, device=a.device)
    check(lib().ss_hamming_pair(a.data_ptr(), b.data_ptr(), n, L, wpr, out.data_ptr(), _stream(a.device)),
          "ss_hamming_pair")
    return out


def encode_hamming_ref(ascii: torch.Tensor, L: Optional[int], ref_words: torch.Tensor, *,
                       store_words: bool = True, wpr: Optional[int] = None,
                       check_errors: bool = True):
    """Fused encode + hamming vs one packed reference: returns (words or None, distances int32)."""
    n, L, stride = _as_rows(ascii, L, None if ascii.dim() == 2 else L)
    wpr = wpr_for(L) if wpr is None else wpr
    dev = ascii.device
    words = torch.empty((n, wpr), dtype=torch.int64, device=dev) if store_words else None
    dist = torch.empty(n, dtype=torch.int32, device=dev)
    ref = ref_words.to(dev).contiguous()
    if ref.numel() < wpr:
        ref = torch.cat([ref.reshape(-1), torch.zeros(wpr - ref.numel(), dtype=torch.int64, device=dev)])
    fb = first_bad_buffer(dev)
    check(lib().ss_encode_hamming_ref(ascii.data_ptr(), n, L, stride, _ptr(words), wpr, ref.data_ptr(),
                                      dist.data_ptr(), fb.data_ptr(), _stream(dev)),
          "ss_encode_hamming_ref")
    if check_errors:
        _check_first_bad(fb, _fetch_row(ascii, stride, L))
    return words, dist


def _host_rows(ascii, L: Optional[int], stride: Optional[int]):
    """numpy uint8 [n, >=L] (rows may be padded: stride = row pitch) or flat bytes-like + L."""
    a = np.frombuffer(ascii, dtype=np.uint8) if isinstance(ascii, (bytes, bytearray, memoryview)) else ascii
    if not isinstance(a, np.ndarray) or a.dtype != np.uint8:
        raise TypeError("host reads must be a uint8 numpy array or a bytes-like object")
    if a.ndim == 2:
        if a.strides[1] != 1 or (a.shape[0] > 1 and a.strides[0] < a.shape[1]):
            raise ValueError("rows must be contiguous bytes")
        L = a.shape[1] if L is None else L
        stride = a.strides[0] if a.shape[0] > 1 else a.shape[1]
        n = a.shape[0]
    else:
        if L is None:
            raise ValueError("L is required for a flat host buffer")
        a = np.ascontiguousarray(a).reshape(-1)
        stride = L if stride is None else stride
        n = a.size // stride if stride else 0
    if not (1 <= L <= MAX_NT):
        if L > MAX_NT:
            raise Exception(f"Sequences longer than {MAX_NT} bases are not supported.")
        raise ValueError("L must be >= 1")
    if stride < L:
        raise ValueError("stride < L")
    return a, n, L, stride


class HostStager:
    """Host-resident batches through the GPU (ss_stager_*, csrc/ss_stage.hip): numpy in, numpy out.

    A batch in host memory is streamed through a ring of pinned + device chunk slots on three HIP
    streams (H2D / kernel / D2H overlapped across neighbouring chunks).  Pageable arrays are staged
    by `copy_threads` memcpy threads; pinned arrays (torch .pin_memory().numpy()) are DMA'd
    directly.  This is the PCIe-inclusive path for data that lives on the host; for data already
    in HBM use encode()/decode() on tensors."""

    def __init__(self, device=None, chunk_bytes: int = 64 << 20, nslots: int = 3,
                 copy_threads: Optional[int] = None):
        import os
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        if copy_threads is None:
            # 12 threads pinned to the GPU's NUMA node: 20.0 ms for 32M x 32-nt reads against 21.4
            # with 8 and 20.6 with 16, the H2D copies at ~19 ms the floor (profiles/r6/probe_stage_split.log)
            copy_threads = int(os.environ.get("SHORTSEQ_STAGE_THREADS", min(12, os.cpu_count() or 1)))
        h = C.c_void_p()
        check(lib().ss_stager_create(self.device.index or 0, chunk_bytes, nslots, copy_threads, C.byref(h)),
              "ss_stager_create")
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().ss_stager_destroy(self._h)
            self._h = None

    STAGES = ("copy_in_host", "copy_out_host", "h2d_dev", "kernel_dev", "d2h_dev", "wait_host")

    def set_timing(self, on: bool = True) -> None:
        """Record the per-chunk stage split (ss_stager_set_timing)."""
        check(lib().ss_stager_set_timing(self._h, int(bool(on))), "ss_stager_set_timing")

    def stats(self) -> dict:
        """Mean ms per timed call of each stage since the last stats() (device stages are sums over
        chunks, which overlap), and the placement: copy threads, affinity CPUs, the GPU's NUMA node,
        CPUs the copy threads are pinned to (ss_stager_stats)."""
        ms = (C.c_double * 6)()
        info = (C.c_int32 * 4)()
        check(lib().ss_stager_stats(self._h, ms, info), "ss_stager_stats")
        out = {k: float(v) for k, v in zip(self.STAGES, ms)}
        out.update(copy_threads=int(info[0]), affinity_cpus=int(info[1]), gpu_numa_node=int(info[2]),
                   pinned_cpus=int(info[3]))
        return out

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 — interpreter shutdown
            pass

    @staticmethod
    def _raise_first_bad(fb: int, a: np.ndarray, stride: int, L: int) -> None:
        if fb != (1 << 64) - 1:
            row = a[fb, :L] if a.ndim == 2 else a[fb * stride: fb * stride + L]
            raise_read_error(bytes(row), fb)

    def encode(self, ascii, L: Optional[int] = None, *, stride: Optional[int] = None, wpr: Optional[int] = None,
               out: Optional[np.ndarray] = None, check_errors: bool = True) -> np.ndarray:
        """-> packed words uint64 [n, wpr] in host memory (ss_encode_host)."""
        a, n, L, stride = _host_rows(ascii, L, stride)
        wpr = wpr_for(L) if wpr is None else wpr
        if out is None:
            out = np.empty((n, wpr), dtype=np.uint64)
        fb = C.c_uint64()
        torch.cuda.current_stream(self.device).synchronize()
        check(lib().ss_encode_host(self._h, a.ctypes.data, n, L, stride, out.ctypes.data, wpr, C.byref(fb)),
              "ss_encode_host")
        if check_errors:
            self._raise_first_bad(fb.value, a, stride, L)
        return out

    def encode_hamming_ref(self, ascii, L: Optional[int], ref_words, *, check_errors: bool = True):
        """-> (words uint64 [n, wpr], distances uint32 [n]) vs one packed reference read."""
        a, n, L, stride = _host_rows(ascii, L, None)
        wpr = wpr_for(L)
        ref = torch.zeros(wpr, dtype=torch.int64, device=self.device)
        r = torch.as_tensor(np.asarray(ref_words, dtype=np.uint64).view(np.int64)).reshape(-1)[:wpr]
        ref[:r.numel()] = r.to(self.device)
        torch.cuda.current_stream(self.device).synchronize()
        words = np.empty((n, wpr), dtype=np.uint64)
        dist = np.empty(n, dtype=np.uint32)
        fb = C.c_uint64()
        check(lib().ss_encode_hamming_ref_host(self._h, a.ctypes.data, n, L, stride, words.ctypes.data, wpr,
                                               ref.data_ptr(), dist.ctypes.data, C.byref(fb)),
              "ss_encode_hamming_ref_host")
        if check_errors:
            self._raise_first_bad(fb.value, a, stride, L)
        return words, dist

    def decode(self, words: np.ndarray, L: int, *, out: Optional[np.ndarray] = None) -> np.ndarray:
        """Packed words uint64 [n, wpr] (host) -> ASCII uint8 [n, L] (host) (ss_decode_host)."""
        w = np.ascontiguousarray(words)
        if w.dtype not in (np.uint64, np.int64):
            raise TypeError("words must be uint64 / int64")
        if w.ndim == 1:
            w = w.reshape(-1, wpr_for(L))
        n, wpr = w.shape
        if out is None:
            out = np.empty((n, L), dtype=np.uint8)
        check(lib().ss_decode_host(self._h, w.ctypes.data, n, L, wpr, out.ctypes.data, out.strides[0] if n else L),
              "ss_decode_host")
        return out


_stagers: dict = {}


def host_stager(device=None) -> HostStager:
    """The process's default HostStager for a device (created on first use)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    st = _stagers.get(dev.index)
    if st is None:
        st = _stagers[dev.index] = HostStager(dev)
    return st


def encode_host(ascii, L: Optional[int] = None, **kw) -> np.ndarray:
    """Host array of reads -> host array of packed words, streamed through the GPU."""
    return host_stager(kw.pop("device", None)).encode(ascii, L, **kw)


def decode_host(words: np.ndarray, L: int, **kw) -> np.ndarray:
    return host_stager(kw.pop("device", None)).decode(words, L, **kw)


def synth_reads(n: int, L: int, seed: int, *, i0: int = 0, device=None, stride: Optional[int] = None,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Device-side synthetic reads (SURVEY §8(d) generator, bit-identical to the oracle's)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    stride = L if stride is None else stride
    if out is None:
        out = torch.empty((n, stride), dtype=torch.uint8, device=dev)
    check(lib().ss_synth_reads(out.data_ptr(), seed, i0, n, L, stride, _stream(dev)), "ss_synth_reads")
    return out


def synth_pool_reads(n: int, L: int, seed: int, pool_seed: int, U: int, *, i0: int = 0, device=None,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if out is None:
        out = torch.empty((n, L), dtype=torch.uint8, device=dev)
    check(lib().ss_synth_pool_reads(out.data_ptr(), seed, pool_seed, U, i0, n, L, L, _stream(dev)),
          "ss_synth_pool_reads")
    return out


def zipf_cdf(U: int, s: float = 1.1) -> np.ndarray:
    """Zipf(s) CDF over pool ranks 0..U-1 scaled to 2^63 (uint64 [U]; the last entry is 2^63), the
    table ss_synth_zipf_reads draws from (include/shortseq_amd.h).  Rank k has weight (k+1)^-s."""
    w = np.arange(1, U + 1, dtype=np.float64) ** (-float(s))
    c = np.cumsum(w)
    c /= c[-1]
    cdf = np.floor(c * 2.0 ** 63).astype(np.uint64)
    cdf[-1] = np.uint64(1 << 63)
    return cdf


def synth_zipf_reads(n: int, L: int, seed: int, pool_seed: int, cdf, *, i0: int = 0, device=None,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Reads drawn from a Zipf-distributed pool (SURVEY §8(d) C5 skew): read i = pool item
    rank(i) of the ss_synth_zipf_reads rule; `cdf` = zipf_cdf(U, s) (numpy) or its device copy."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if isinstance(cdf, np.ndarray):
        cdf = torch.from_numpy(cdf.view(np.int64)).to(dev)
    if out is None:
        out = torch.empty((n, L), dtype=torch.uint8, device=dev)
    check(lib().ss_synth_zipf_reads(out.data_ptr(), seed, pool_seed, cdf.data_ptr(), cdf.numel(), i0, n, L, L,
                                    _stream(dev)), "ss_synth_zipf_reads")
    return out


def synth_ragged_pool_reads(n: int, seed: int, pool_seed: int, U: int, Lmin: int, Lmax: int, *, i0: int = 0,
                            device=None):
    """Device-side ragged reads drawn from a pool of U items of lengths Lmin..Lmax (the
    ss_synth_ragged_* rule, include/shortseq_amd.h): returns (blob u8 [total + 16], offsets i64 [n],
    lens i32 [n]) with the reads back to back."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    lens = torch.empty(n, dtype=torch.int32, device=dev)
    s = _stream(dev)
    check(lib().ss_synth_ragged_lens(lens.data_ptr(), seed, pool_seed, U, i0, n, Lmin, Lmax, s), "ss_synth_ragged_lens")
    offs = torch.cumsum(lens, 0, dtype=torch.int64) - lens.to(torch.int64)   # layout only (exclusive prefix)
    total = int(offs[-1].item() + lens[-1].item()) if n else 0
    blob = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    check(lib().ss_synth_ragged_reads(blob.data_ptr(), offs.data_ptr(), seed, pool_seed, U, i0, n, Lmin, Lmax, s),
          "ss_synth_ragged_reads")
    return blob, offs, lens


class DeviceIngest:
    """The drop-in counter's engine (ss_ingest_*) fed from device memory: count(blob, offsets, lens)
    any number of times (global read indices continue), then results() -> (lens u32, counts u64,
    words u64) numpy arrays in first-occurrence order (the ShortSeqCounter dict order: row k has
    ceil(lens[k] / 32) words, one for lengths 0..32).  A rejected read raises like ShortSeqCounter."""

    def __init__(self, device=None, exact: bool = False, *, compact=True, _sizing: Optional[int] = None):
        """compact: the rows cross PCIe with u16 lengths and u32 counts (u64 when a count needs it):
        results() then returns those dtypes (ss_ingest_set_results_format)."""
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        h = C.c_void_p()
        check(lib().ss_ingest_create(dev.index or 0, C.byref(h)), "ss_ingest_create")
        self._h = h
        self.compact = int(compact)      # (2: compact with u64 counts, a test hook)
        check(lib().ss_ingest_set_results_format(h, self.compact), "ss_ingest_set_results_format")
        self._exact = exact
        self._sizing = int(exact) if _sizing is None else _sizing   # 2: test hook, undersized class tables
        self._fresh = True
        check(lib().ss_ingest_set_exact(h, self._sizing), "ss_ingest_set_exact")

    def count(self, blob: torch.Tensor, offsets: torch.Tensor, lens: torch.Tensor) -> None:
        for t, name in ((blob, "blob"), (offsets, "offsets"), (lens, "lens")):
            _require_cuda(t, name)
        if offsets.dtype != torch.int64 or lens.dtype not in (torch.int32, torch.uint32) or blob.dtype != torch.uint8:
            raise TypeError("blob u8, offsets int64, lens int32")
        torch.cuda.current_stream(self.device).synchronize()   # the engine runs on its own stream
        args = (self._h, blob.data_ptr(), blob.numel(), offsets.data_ptr(), lens.data_ptr(), lens.numel())
        rc = lib().ss_ingest_add_device(*args)
        self.retried = False
        if rc == SS_EFULL and self._fresh and not self._exact:
            # a length class's table, sized by its distinct-key sketch, ran full: the first batch of the
            # count is counted again with tables sized by their rows (later batches cannot be redone)
            check(lib().ss_ingest_reset(self._h), "ss_ingest_reset")
            check(lib().ss_ingest_set_exact(self._h, 1), "ss_ingest_set_exact")
            rc = lib().ss_ingest_add_device(*args)
            check(lib().ss_ingest_set_exact(self._h, self._sizing), "ss_ingest_set_exact")
            self.retried = True
        if rc == SS_EFULL and not self._fresh:
            raise NativeError("ss_ingest_add_device: a length class's table, sized by its distinct-key "
                                  "sketch, ran full on a later batch; the counts so far are void -- reset() "
                                  "and count every batch again with DeviceIngest(exact=True)")
        check(rc, "ss_ingest_add_device")
        self._fresh = False
        idx, kind, ln = C.c_uint64(), C.c_int(), C.c_uint64()
        check(lib().ss_ingest_error(self._h, C.byref(idx), C.byref(kind), None, 0, C.byref(ln)), "ss_ingest_error")
        if idx.value != (1 << 64) - 1:
            if kind.value == 2:
                raise Exception("Sequences longer than 1024 bases are not supported.")
            buf = (C.c_uint8 * max(1, ln.value))()
            check(lib().ss_ingest_error(self._h, C.byref(idx), C.byref(kind), buf, ln.value, C.byref(ln)),
                  "ss_ingest_error")
            raise_read_error(bytes(buf)[:ln.value], idx.value)

    def results(self, copy: bool = True):
        """(lens, counts, words u64) of the count so far, first-occurrence order: lens u32 and counts
        u64, or with compact=True lens u16 and counts u32 (u64 when a count needs it).  copy=False
        returns views of the engine's pinned result buffers, valid until the next count / reset /
        close (no host-side copy of the rows)."""
        K, NW = C.c_uint64(), C.c_uint64()
        check(lib().ss_ingest_finish(self._h, C.byref(K), C.byref(NW)), "ss_ingest_finish")
        pl, pc, pw = C.c_void_p(), C.c_void_p(), C.c_void_p()
        k, nw = K.value, NW.value
        if self.compact:
            cb = C.c_uint32()
            check(lib().ss_ingest_results_compact(self._h, C.byref(pl), C.byref(pc), C.byref(cb), C.byref(pw)),
                  "ss_ingest_results_compact")
            lt, ct = C.c_uint16, (C.c_uint32 if cb.value == 4 else C.c_uint64)
        else:
            check(lib().ss_ingest_results(self._h, C.byref(pl), C.byref(pc), C.byref(pw)), "ss_ingest_results")
            lt, ct = C.c_uint32, C.c_uint64
        lens = np.ctypeslib.as_array((lt * max(1, k)).from_address(pl.value))[:k] if k else np.zeros(0, lt)
        cnts = np.ctypeslib.as_array((ct * max(1, k)).from_address(pc.value))[:k] if k else np.zeros(0, ct)
        wds = np.ctypeslib.as_array((C.c_uint64 * max(1, nw)).from_address(pw.value))[:nw] if nw else np.zeros(0, np.uint64)
        if copy:
            lens, cnts, wds = lens.copy(), cnts.copy(), wds.copy()
        return lens, cnts, wds

    def set_row_limit(self, rows: int) -> None:
        """Test hook: re-key a length's table once its rows pass `rows` (default 2^32 - 1)."""
        check(lib().ss_ingest_set_row_limit(self._h, int(rows)), "ss_ingest_set_row_limit")

    def set_count_limit(self, reads: int) -> None:
        """Test hook: spill the tables' u32 counts into u64 row counts every `reads` reads (default 2^32 - 2)."""
        check(lib().ss_ingest_set_count_limit(self._h, int(reads)), "ss_ingest_set_count_limit")

    def export(self) -> int:
        """Extract this engine's tables for a device-side reduce (ss_ingest_export); its distinct keys."""
        k = C.c_uint64()
        check(lib().ss_ingest_export(self._h, C.byref(k)), "ss_ingest_export")
        return k.value

    def merge(self, src: "DeviceIngest", base: int) -> None:
        """Fold an exported engine whose reads follow this one's (global read index `base` onward) into
        this engine's tables on its device (ss_ingest_merge: peer copies, counts add, first = min)."""
        check(lib().ss_ingest_merge(self._h, src._h, int(base)), "ss_ingest_merge")

    def reserve_merge(self, srcs) -> None:
        """Size this engine's tables once for the union of the exported engines `srcs` it will merge
        (ss_ingest_reserve_merge): no table growth per merge."""
        arr = (C.c_void_p * max(1, len(srcs)))(*[e._h.value for e in srcs])
        check(lib().ss_ingest_reserve_merge(self._h, arr, len(srcs)), "ss_ingest_reserve_merge")

    def reset(self) -> None:
        check(lib().ss_ingest_reset(self._h), "ss_ingest_reset")
        self._fresh = True

    def close(self) -> None:
        if self._h:
            lib().ss_ingest_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def slice_fixed(words: torch.Tensor, L: int, start: Optional[int] = None, stop: Optional[int] = None,
                *, out: Optional[torch.Tensor] = None):
    """reads[start:stop] for every read of a fixed-length packed batch (Python slice bounds, step 1,
    as ShortSeq.__getitem__; short_seq.pyx:93-238) -> (words [n, max(1, ceil(len/32))], len)."""
    _require_cuda(words, "words")
    n, wpr = words.shape
    st, sp, step = slice(start, stop).indices(L)
    ln = max(0, sp - st)
    if ln == 0:
        st = 0
    ow = wpr_for(ln)
    if out is None:
        out = torch.empty((n, ow), dtype=torch.int64, device=words.device)
    check(lib().ss_slice_fixed(words.data_ptr(), n, L, wpr, st, ln, out.data_ptr(), out.shape[1],
                               _stream(words.device)), "ss_slice_fixed")
    return out, ln


def slice_var(words: torch.Tensor, starts: torch.Tensor, lens: torch.Tensor, *,
              read_lens: Optional[torch.Tensor] = None, out_wpr: Optional[int] = None) -> torch.Tensor:
    """Per-read slices of a packed batch (adapter / UMI trimming): row r = nts [starts[r],
    starts[r] + lens[r]) of read r, clamped to read_lens[r] when given (int32 tensors)."""
    for t, nm in ((words, "words"), (starts, "starts"), (lens, "lens")):
        _require_cuda(t, nm)
    n, wpr = words.shape
    if out_wpr is None:
        out_wpr = wpr
    out = torch.empty((n, out_wpr), dtype=torch.int64, device=words.device)
    check(lib().ss_slice_var(words.data_ptr(), n, wpr, _ptr(read_lens), starts.data_ptr(), lens.data_ptr(),
                             out.data_ptr(), out_wpr, _stream(words.device)), "ss_slice_var")
    return out


ALL_PAIRS_METHODS = {"auto": 0, "tiles": 1, "pigeonhole": 2}


def hamming_all_pairs(words: torch.Tensor, L: int, max_dist: int, *, counts: bool = True,
                      max_pairs: int = 0, method: str = "auto"):
    """Unordered pairs (i < j) of a packed batch within `max_dist` (the reference __xor__ distance)
    -> (neighbour counts int32 [n] or None, pairs int32 [m, 2] or None, total pairs).  Pairs are
    returned sorted; at most max_pairs are kept (0: count only).  method: "tiles" checks every pair,
    "pigeonhole" (L <= 128) only pairs sharing one of max_dist + 1 segments, "auto" picks
    (ss_hamming_all_pairs_ex); the results are the same."""
    _require_cuda(words, "words")
    n, wpr = words.shape
    dev = words.device
    cnt = torch.empty(n, dtype=torch.int32, device=dev) if counts else None
    pairs = torch.empty((max(1, max_pairs), 2), dtype=torch.int32, device=dev) if max_pairs else None
    tot = torch.empty(1, dtype=torch.int64, device=dev)
    check(lib().ss_hamming_all_pairs_ex(words.data_ptr(), n, L, wpr, max_dist, _ptr(cnt), _ptr(pairs), max_pairs,
                                        tot.data_ptr(), ALL_PAIRS_METHODS[method], _stream(dev)),
          "ss_hamming_all_pairs_ex")
    total = int(tot.item())
    if pairs is not None:
        m = min(total, max_pairs)
        p = pairs[:m].to(torch.int64)
        key = p[:, 0] * (1 << 32) + p[:, 1]
        pairs = pairs[:m][torch.argsort(key)]
    return cnt, pairs, total


LEN_UNDERFLOW = 0xFFFFFFFF   # ss_fastq_index: strlen 0 (the reference's size_t underflow -> too long)


def fastq_index(buf: torch.Tensor, nbytes: Optional[int] = None, *, line0: int = 0, at_eof: bool = True,
                onepass: bool = True, max_reads: Optional[int] = None):
    """Sequence lines of a FASTQ chunk resident on the device (fast_read.pyx:3-20 rule, see
    include/shortseq_amd.h ss_fastq_index) -> (offsets int64 [n], lens int64 [n], newlines).
    lens holds the reference's strlen - 1 (LEN_UNDERFLOW where strlen is 0).  The chunk must start
    at a line boundary and end right after a newline unless at_eof.
    onepass: ss_fastq_index_onepass (the chunk is read once; max_reads is a capacity guess, default
    nbytes / 16 + 2, and the call is repeated with the exact count if the chunk holds more lines);
    otherwise ss_fastq_scan + ss_fastq_index (two reads of the chunk, exact capacity)."""
    _require_cuda(buf, "buf")
    if buf.dtype != torch.uint8:
        raise TypeError("buf must be a uint8 tensor")
    nbytes = buf.numel() if nbytes is None else nbytes
    dev = buf.device
    L_ = lib()
    s = _stream(dev)
    if onepass:
        cnt = torch.empty(3, dtype=torch.int64, device=dev)
        cap = nbytes // 16 + 2 if max_reads is None else max_reads
        while True:
            ws_bytes = int(L_.ss_fastq_onepass_ws_bytes(nbytes, cap))
            ws = torch.empty((ws_bytes + 7) // 8, dtype=torch.int64, device=dev)
            offs = torch.empty(cap, dtype=torch.int64, device=dev)
            lens = torch.empty(cap, dtype=torch.int32, device=dev)
            aux = torch.empty(cap, dtype=torch.int64, device=dev)
            check(L_.ss_fastq_index_onepass(buf.data_ptr(), nbytes, line0, 1 if at_eof else 0, ws.data_ptr(), ws_bytes,
                                            offs.data_ptr(), lens.data_ptr(), aux.data_ptr(), cap, cnt.data_ptr(), s),
                  "ss_fastq_index_onepass")
            nl, n, full = (int(v) for v in cnt.tolist())
            if full:                  # a staging region ran full (lines far denser than the bound)
                cap *= 2
                continue
            if n <= cap:
                break
            cap = n
        return offs[:n], lens[:n].to(torch.int64) & 0xFFFFFFFF, nl
    ws_bytes = int(L_.ss_fastq_scan_ws_bytes(nbytes))
    ws = torch.empty((ws_bytes + 7) // 8, dtype=torch.int64, device=dev)
    cnt = torch.empty(2, dtype=torch.int64, device=dev)
    check(L_.ss_fastq_scan(buf.data_ptr(), nbytes, ws.data_ptr(), ws_bytes, cnt.data_ptr(), s), "ss_fastq_scan")
    nl = int(cnt[0].item())
    cap = nl // 4 + 2
    offs = torch.empty(cap, dtype=torch.int64, device=dev)
    lens = torch.empty(cap, dtype=torch.int32, device=dev)
    aux = torch.empty(cap, dtype=torch.int64, device=dev)
    check(L_.ss_fastq_index(buf.data_ptr(), nbytes, line0, 1 if at_eof else 0, ws.data_ptr(), offs.data_ptr(),
                            lens.data_ptr(), aux.data_ptr(), cap, cnt[1:].data_ptr(), s), "ss_fastq_index")
    n = int(cnt[1].item())
    if n > cap:
        raise AssertionError("FASTQ index capacity exceeded")
    return offs[:n], lens[:n].to(torch.int64) & 0xFFFFFFFF, nl


def gather_rows(src: torch.Tensor, offsets: torch.Tensor, L: int, *, sel: Optional[torch.Tensor] = None,
                src_bytes: Optional[int] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Dense [m, round_up(L, 16)] uint8 rows gathered from a ragged byte buffer on the device:
    row r = src[offsets[sel[r]] : + L] (sel None: r).  Feeds one length group of a ragged batch to the
    fixed-length kernels."""
    _require_cuda(src, "src")
    _require_cuda(offsets, "offsets")
    if offsets.dtype != torch.int64 or (sel is not None and sel.dtype != torch.int64):
        raise TypeError("offsets / sel must be int64 tensors")
    m = (sel if sel is not None else offsets).numel()
    S = (L + 15) // 16 * 16
    if out is None:
        out = torch.empty((m, S), dtype=torch.uint8, device=src.device)
    src_bytes = src.numel() if src_bytes is None else src_bytes
    check(lib().ss_gather_rows(src.data_ptr(), src_bytes, offsets.data_ptr(), _ptr(sel), m, L, out.data_ptr(),
                               out.shape[1] if out.dim() == 2 else S, _stream(src.device)), "ss_gather_rows")
    return out


class GpuCounter:
    """Dedup counter in HBM for reads of ONE length L <= 1024 (ShortSeqCounter's hot loop,
    counter.pyx:41-54).  Counts and first-occurrence indices per distinct key: the packed word for
    L <= 32, the W = ceil(L/32) packed words for longer reads (fingerprinted, compared on words)."""

    def __init__(self, capacity: int, device=None):
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().ss_counter_create(capacity, C.byref(h)), "ss_counter_create")
        self._h = h
        self.capacity = int(lib().ss_counter_capacity(h))
        self._scratch = torch.empty(2, dtype=torch.int64, device=self.device)

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().ss_counter_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 — interpreter shutdown
            pass

    @property
    def length(self) -> int:
        return int(lib().ss_counter_length(self._h))

    @property
    def words(self) -> int:
        """Words per key (1 for L <= 32); fixed by the first insert."""
        return int(lib().ss_counter_words(self._h))

    PASSES = ("coarse", "order", "scatter", "aggregate", "spill")

    def set_timing(self, on: bool = True) -> None:
        """Record HIP events between the partitioned insert's passes (ss_counter_set_timing)."""
        check(lib().ss_counter_set_timing(self._h, int(bool(on))), "ss_counter_set_timing")

    def pass_times(self) -> dict:
        """Mean ms per insert of each pass since the last call ({} when none was timed)."""
        ms = (C.c_double * 5)()
        k = C.c_uint64()
        check(lib().ss_counter_pass_times(self._h, ms, C.byref(k)), "ss_counter_pass_times")
        return dict(zip(self.PASSES, list(ms))) if k.value else {}

    def reset(self) -> None:
        check(lib().ss_counter_reset(self._h, _stream(self.device)), "ss_counter_reset")

    PARTITION_MIN_READS = 1 << 16   # batches at least this large reserve the partitioned path

    def reserve(self, max_reads: int) -> bool:
        """Workspace for the partitioned insert (20 B/read); False if this table cannot use it."""
        rc = lib().ss_counter_reserve(self._h, max_reads)
        return rc == 0

    def insert(self, ascii: torch.Tensor, L: Optional[int] = None, *, base_index: int = 0,
               stride: Optional[int] = None, check_errors: bool = True, partitioned: Optional[bool] = None) -> None:
        """partitioned: None = automatic (large batches), True = reserve workspace and use the
        partitioned insert if the table allows it, False = direct atomic insert."""
        n, L, stride = _as_rows(ascii, L, stride)
        if L > 32:   # multi-word keys: always partitioned, the library grows the workspace itself
            partitioned = None
        elif partitioned is None:
            partitioned = n >= self.PARTITION_MIN_READS
        if partitioned and n > int(lib().ss_counter_reserved(self._h)) and n < (1 << 32):
            self.reserve(n)
        if partitioned is False and int(lib().ss_counter_reserved(self._h)) >= n:
            self._drop_reservation()
        fb = first_bad_buffer(self.device)
        check(lib().ss_counter_insert_fixed(self._h, ascii.data_ptr(), n, L, stride, base_index,
                                            fb.data_ptr(), _stream(self.device)), "ss_counter_insert_fixed")
        if check_errors:
            _check_first_bad(fb, _fetch_row(ascii, stride, L))

    def _drop_reservation(self) -> None:
        torch.cuda.synchronize(self.device)
        check(lib().ss_counter_release(self._h), "ss_counter_release")

    def merge(self, keys: torch.Tensor, counts: torch.Tensor, first: torch.Tensor, L: int) -> None:
        m = keys.numel()
        check(lib().ss_counter_set_length(self._h, L), "ss_counter_set_length")
        check(lib().ss_counter_merge(self._h, keys.data_ptr(), None, counts.data_ptr(), first.data_ptr(), m,
                                     _stream(self.device)), "ss_counter_merge")

    def set_spill_limit(self, reads: int) -> None:
        """Test hook (ss_counter_set_spill_limit): move the u32 slot counts into the u64 array once more
        than `reads` reads were inserted since the last spill (default 2^32 - 1)."""
        check(lib().ss_counter_set_spill_limit(self._h, int(reads)), "ss_counter_set_spill_limit")

    def size(self) -> int:
        check(lib().ss_counter_size(self._h, self._scratch.data_ptr(), _stream(self.device)), "ss_counter_size")
        return int(self._scratch[0].item())

    def overflow_word(self) -> torch.Tensor:
        """The handle's overflow word as a 1-element device tensor (no host sync)."""
        check(lib().ss_counter_overflow(self._h, self._scratch[1:].data_ptr(), _stream(self.device)),
              "ss_counter_overflow")
        return self._scratch[1:2]

    def overflowed(self) -> bool:
        return int(self.overflow_word().item()) != 0

    def extract(self, n_parts: int = 1, cap: Optional[int] = None):
        """Occupied slots grouped by owner part -> (keys, lens, counts, first, part_counts), all on
        the device; arrays sized `cap` (default: capacity + 1), valid prefix = part_counts.sum()."""
        cap = self.capacity + 1 if cap is None else cap
        d = self.device
        keys = torch.empty(cap, dtype=torch.int64, device=d)
        lens = torch.empty(cap, dtype=torch.int32, device=d)
        counts = torch.empty(cap, dtype=torch.int64, device=d)
        first = torch.empty(cap, dtype=torch.int64, device=d)
        parts = torch.empty(n_parts, dtype=torch.int64, device=d)
        check(lib().ss_counter_extract(self._h, n_parts, keys.data_ptr(), lens.data_ptr(), counts.data_ptr(),
                                       first.data_ptr(), cap, parts.data_ptr(), _stream(d)), "ss_counter_extract")
        return keys, lens, counts, first, parts

    def geometry(self):
        """(log2 capacity, log2 slots per region) of the table (region-range ownership)."""
        a, b = C.c_uint32(), C.c_uint32()
        check(lib().ss_counter_geometry(self._h, C.byref(a), C.byref(b)), "ss_counter_geometry")
        return int(a.value), int(b.value)

    def extract_ranges(self, n_parts: int, cap: Optional[int] = None):
        """As extract, with part p = the table regions owner p holds under region-range ownership
        (include/shortseq_amd.h); each part is sorted by region, the sentinel key last."""
        cap = self.capacity + 1 if cap is None else cap
        d = self.device
        keys = torch.empty(cap, dtype=torch.int64, device=d)
        lens = torch.empty(cap, dtype=torch.int32, device=d)
        counts = torch.empty(cap, dtype=torch.int64, device=d)
        first = torch.empty(cap, dtype=torch.int64, device=d)
        parts = torch.empty(n_parts, dtype=torch.int64, device=d)
        check(lib().ss_counter_extract_ranges(self._h, n_parts, keys.data_ptr(), lens.data_ptr(), counts.data_ptr(),
                                              first.data_ptr(), cap, parts.data_ptr(), _stream(d)),
              "ss_counter_extract_ranges")
        return keys, lens, counts, first, parts

    def merge_runs(self, keys: torch.Tensor, counts: torch.Tensor, first: torch.Tensor, runs, part: int,
                   n_parts: int, L: int) -> None:
        """Fold region-sorted runs (list of (begin, end) into keys / counts / first) into the regions
        this table owns as `part` of `n_parts` (ss_counter_merge_runs)."""
        d = self.device
        m = keys.numel()
        if not runs:
            return
        offs = torch.tensor([x for be in runs for x in be], dtype=torch.int64).to(d, non_blocking=True)
        log2cap, slice_log = self.geometry()
        R = 1 << (log2cap - slice_log)
        nreg = -(-(part + 1) * R // n_parts) - (-(part * R) // n_parts)
        bounds = torch.empty(len(runs) * (nreg + 1) + 1, dtype=torch.int32, device=d)
        check(lib().ss_counter_merge_runs(self._h, keys.data_ptr(), counts.data_ptr(), first.data_ptr(),
                                          offs.data_ptr(), len(runs), m, part, n_parts, L, bounds.data_ptr(),
                                          _stream(d)), "ss_counter_merge_runs")

    def pack_ranges(self, n_parts: int, skip: int = -1, first_base: int = 0, cap: Optional[int] = None):
        """Region-range parts as packed 16-B records (ss_counter_pack_ranges) -> (rec int64 [cap, 2],
        part_counts int64 [n_parts]) on the device; rec[:, 0] = key, rec[:, 1] = count | (first -
        first_base) << 32; part `skip` is left out (count 0).  Raises if a record field overflowed."""
        cap = self.capacity + 1 if cap is None else cap
        d = self.device
        rec = torch.empty((cap, 2), dtype=torch.int64, device=d)
        parts = torch.empty(n_parts, dtype=torch.int64, device=d)
        check(lib().ss_counter_pack_ranges(self._h, n_parts, skip, first_base, rec.data_ptr(), cap, parts.data_ptr(),
                                           _stream(d)), "ss_counter_pack_ranges")
        return rec, parts

    def merge_packed(self, rec: torch.Tensor, runs, part: int, n_parts: int, L: int) -> None:
        """Fold region-sorted packed runs (list of (begin, end, first_base) into rec) into the regions
        this table owns as `part` of `n_parts` (ss_counter_merge_packed)."""
        d = self.device
        if not runs:
            return
        m = rec.shape[0]
        offs = torch.tensor([x for (b, e, _f) in runs for x in (b, e)], dtype=torch.int64).to(d, non_blocking=True)
        bases = torch.tensor([f for (_b, _e, f) in runs], dtype=torch.int64).to(d, non_blocking=True)
        log2cap, slice_log = self.geometry()
        R = 1 << (log2cap - slice_log)
        nreg = -(-(part + 1) * R // n_parts) - (-(part * R) // n_parts)
        bounds = torch.empty(len(runs) * (nreg + 1) + 1, dtype=torch.int32, device=d)
        check(lib().ss_counter_merge_packed(self._h, rec.data_ptr(), offs.data_ptr(), bases.data_ptr(), len(runs), m,
                                            part, n_parts, L, bounds.data_ptr(), _stream(d)),
              "ss_counter_merge_packed")

    def extract_words(self, n_parts: int = 1, cap: Optional[int] = None):
        """As extract, for any key length: (fps, lens, words [cap, W], counts, first, part_counts);
        fps = the multi-word fingerprints (the packed word itself for W = 1)."""
        cap = self.capacity + 1 if cap is None else cap
        d = self.device
        W = max(1, self.words)
        fps = torch.empty(cap, dtype=torch.int64, device=d)
        lens = torch.empty(cap, dtype=torch.int32, device=d)
        words = torch.empty((cap, W), dtype=torch.int64, device=d)
        counts = torch.empty(cap, dtype=torch.int64, device=d)
        first = torch.empty(cap, dtype=torch.int64, device=d)
        parts = torch.empty(n_parts, dtype=torch.int64, device=d)
        check(lib().ss_counter_extract_words(self._h, n_parts, fps.data_ptr(), lens.data_ptr(), words.data_ptr(),
                                             counts.data_ptr(), first.data_ptr(), cap, parts.data_ptr(), _stream(d)),
              "ss_counter_extract_words")
        return fps, lens, words, counts, first, parts

    def merge_words(self, words: torch.Tensor, counts: torch.Tensor, first: torch.Tensor) -> None:
        """Fold rows of packed multi-word keys (int64 [m, W], W = the handle's words) with their counts
        and global first indices into the table (ss_counter_merge_words: keys already present add
        their counts and keep the smaller first index)."""
        m = words.shape[0]
        if m == 0:
            return
        if words.dim() != 2 or words.shape[1] != self.words:
            raise ValueError("merge_words: rows of the handle's word count")
        w, c, f = (x.contiguous() for x in (words, counts.to(torch.int64), first.to(torch.int64)))
        check(lib().ss_counter_merge_words(self._h, w.data_ptr(), c.data_ptr(), f.data_ptr(), m,
                                           _stream(self.device)), "ss_counter_merge_words")

    def items_words(self):
        """Host copy of (words u64 [m, W], counts, first) in table order (unsorted)."""
        _, _, words, counts, first, parts = self.extract_words(1)
        m = int(parts.sum().item())
        if self.overflowed():
            raise RuntimeError("GPU counter table overflowed; use a larger capacity")
        return words[:m].cpu().numpy().view(np.uint64), counts[:m].cpu().numpy(), first[:m].cpu().numpy()

    def insert_words(self, words: torch.Tensor, base_index: int = 0) -> None:
        """Count rows of already-packed keys (int64 [n, W], W = 2..64, compared whole;
        ss_counter_set_words + ss_counter_insert_words).  The first call fixes W."""
        _require_cuda(words, "words")
        if words.dim() != 2 or words.dtype != torch.int64 or not words.is_contiguous():
            raise TypeError("words: contiguous int64 [n, W]")
        check(lib().ss_counter_set_words(self._h, words.shape[1]), "ss_counter_set_words")
        check(lib().ss_counter_insert_words(self._h, words.data_ptr(), words.shape[0], base_index,
                                            _stream(self.device)), "ss_counter_insert_words")

    def items_sorted_words(self):
        """Host copy of (words u64 [m, W], counts, first) sorted by first occurrence (= dict order)."""
        _, _, words, counts, first, parts = self.extract_words(1)
        m = int(parts.sum().item())
        if self.overflowed():
            raise RuntimeError("GPU counter table overflowed; use a larger capacity")
        k = words[:m].cpu().numpy().view(np.uint64)
        c = counts[:m].cpu().numpy()
        f = first[:m].cpu().numpy()
        o = np.argsort(f, kind="stable")
        return k[o], c[o], f[o]

    def items_sorted(self):
        """Host copy of (keys u64, counts, first) sorted by first occurrence (= dict order)."""
        keys, lens, counts, first, parts = self.extract(1)
        m = int(parts.sum().item())
        if self.overflowed():
            raise RuntimeError("GPU counter table overflowed; use a larger capacity")
        k = keys[:m].cpu().numpy().view(np.uint64)
        c = counts[:m].cpu().numpy()
        f = first[:m].cpu().numpy()
        o = np.argsort(f, kind="stable")
        return k[o], c[o], f[o]
