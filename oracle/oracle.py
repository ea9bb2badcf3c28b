"""TEST INFRASTRUCTURE ONLY — ctypes/numpy wrapper around oracle/liboracle.so.

The oracle is the checker: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
import this module.  shortseq_amd/ never imports it (tests/test_boundary.py enforces that).

Functions mirror oracle/ss_oracle.c (which cites the reference file:line of every rule).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_DIR = os.path.join(HERE, "_ref")


class OraErr(C.Structure):
    _fields_ = [("kind", C.c_int32), ("nbytes", C.c_int32),
                ("read_index", C.c_int64), ("byte_offset", C.c_int64)]


def build() -> None:
    """Compile liboracle.so (gcc) and, when /root/reference exists, the reference into _ref/."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if os.path.isdir("/root/reference"):
        subprocess.run([os.path.join(HERE, "build_ref.sh")], check=True,
                       stdout=subprocess.DEVNULL)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P, U64, U32, I64 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int64
        L.ora_encode.argtypes = [P, U32, P, C.POINTER(OraErr)]
        L.ora_encode.restype = C.c_int
        L.ora_words_for.argtypes = [U32]
        L.ora_words_for.restype = U32
        L.ora_decode.argtypes = [P, U32, P]
        L.ora_hamming.argtypes = [P, P, U32]
        L.ora_hamming.restype = U32
        L.ora_encode_batch.argtypes = [P, U64, U32, U64, P, U32, C.POINTER(OraErr)]
        L.ora_encode_batch.restype = C.c_int
        L.ora_decode_batch.argtypes = [P, U64, U32, U32, P, U64]
        L.ora_hamming_ref_batch.argtypes = [P, U64, U32, U32, P, P]
        L.ora_hamming_pair_batch.argtypes = [P, P, U64, U32, U32, P]
        L.ora_gen_word.argtypes = [U64, U64, U32, U32]
        L.ora_gen_word.restype = U64
        L.ora_gen_reads.argtypes = [U64, U64, U64, U32, U64, P]
        L.ora_pool_index.argtypes = [U64, U64, U64]
        L.ora_pool_index.restype = U64
        L.ora_gen_pool_reads.argtypes = [U64, U64, U64, U64, U64, U32, U64, P]
        L.ora_zipf_index.argtypes = [U64, U64, P, U64]
        L.ora_zipf_index.restype = U64
        L.ora_gen_zipf_reads.argtypes = [U64, U64, P, U64, U64, U64, U32, U64, P]
        L.ora_count.argtypes = [P, P, P, U64, P, P, P, P, C.POINTER(OraErr)]
        L.ora_count.restype = I64
        L.ora_fastq_index.argtypes = [P, U64, P, P, U64]
        L.ora_fastq_index.restype = U64
        L.ora_slice.argtypes = [P, U32, U32, U32, P]
        L.ora_slice.restype = None
        _lib = L
    return _lib


_plib = None


def plib():
    """Second handle (PyDLL: the GIL stays held) for the calls into the reference's own kernels,
    which take the GIL to raise on an invalid byte."""
    global _plib
    if _plib is None:
        lib()
        L = C.PyDLL(LIB_PATH)
        P, U64, U32 = C.c_void_p, C.c_uint64, C.c_uint32
        L.ref_encode64_batch.argtypes = [P, P, U64, U32, U64, P]
        L.ref_encode_array_batch.argtypes = [P, P, U64, U32, U64, P, U32]
        _plib = L
    return _plib


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


def words_for(L: int) -> int:
    return (L + 31) // 32


def wpr_for(L: int) -> int:
    """Words a read of length L occupies in batch layouts (1 for L <= 32, incl. L == 0)."""
    return max(1, words_for(L))


def encode_one(seq: bytes, wpr: int | None = None):
    """Encode one read like shortseq._new. Returns (words ndarray[uint64], OraErr)."""
    L = len(seq)
    n = wpr if wpr is not None else max(3 if 33 <= L <= 96 else 1, words_for(L))
    out = np.zeros(max(n, 32), dtype=np.uint64)
    buf = np.frombuffer(seq, dtype=np.uint8) if L else np.zeros(1, np.uint8)
    err = OraErr()
    lib().ora_encode(_p(buf), L, _p(out), C.byref(err))
    return out[:n], err


def encode_batch(ascii: np.ndarray, n: int, L: int, stride: int | None = None, wpr: int | None = None):
    stride = L if stride is None else stride
    wpr = wpr_for(L) if wpr is None else wpr
    out = np.zeros(n * wpr, dtype=np.uint64)
    err = OraErr()
    rc = lib().ora_encode_batch(_p(ascii), n, L, stride, _p(out), wpr, C.byref(err))
    return out.reshape(n, wpr), rc, err


def decode_batch(words: np.ndarray, n: int, L: int, wpr: int | None = None) -> np.ndarray:
    wpr = wpr_for(L) if wpr is None else wpr
    out = np.zeros(max(1, n * L), dtype=np.uint8)
    w = np.ascontiguousarray(words, dtype=np.uint64)
    lib().ora_decode_batch(_p(w), n, L, wpr, _p(out), L)
    return out[: n * L]


def hamming_ref_batch(words: np.ndarray, n: int, L: int, ref: np.ndarray, wpr: int | None = None):
    wpr = wpr_for(L) if wpr is None else wpr
    out = np.zeros(n, dtype=np.uint32)
    w = np.ascontiguousarray(words, dtype=np.uint64)
    r = np.ascontiguousarray(ref, dtype=np.uint64)
    lib().ora_hamming_ref_batch(_p(w), n, L, wpr, _p(r), _p(out))
    return out


def hamming_pair_batch(a: np.ndarray, b: np.ndarray, n: int, L: int, wpr: int | None = None):
    wpr = wpr_for(L) if wpr is None else wpr
    out = np.zeros(n, dtype=np.uint32)
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    lib().ora_hamming_pair_batch(_p(a), _p(b), n, L, wpr, _p(out))
    return out


def gen_reads(seed: int, i0: int, n: int, L: int, stride: int | None = None) -> np.ndarray:
    stride = L if stride is None else stride
    out = np.zeros(max(1, n * stride), dtype=np.uint8)
    lib().ora_gen_reads(seed, i0, n, L, stride, _p(out))
    return out[: n * stride]


def gen_words(seed: int, i0: int, n: int, L: int) -> np.ndarray:
    """Known-answer words of gen_reads (the generator's r values, masked)."""
    W = words_for(L)
    f = lib().ora_gen_word
    return np.array([[f(seed, i0 + k, L, w) for w in range(W)] for k in range(n)], dtype=np.uint64)


def gen_pool_reads(seed: int, pool_seed: int, U: int, i0: int, n: int, L: int) -> np.ndarray:
    out = np.zeros(max(1, n * L), dtype=np.uint8)
    lib().ora_gen_pool_reads(seed, pool_seed, U, i0, n, L, L, _p(out))
    return out[: n * L]


def gen_zipf_reads(seed: int, pool_seed: int, cdf: np.ndarray, i0: int, n: int, L: int) -> np.ndarray:
    out = np.zeros(max(1, n * L), dtype=np.uint8)
    c = np.ascontiguousarray(cdf, dtype=np.uint64)
    lib().ora_gen_zipf_reads(seed, pool_seed, _p(c), len(c), i0, n, L, L, _p(out))
    return out[: n * L]


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    """Vectorised ora_splitmix64 (uint64 wrap-around arithmetic)."""
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def pool_ids(pool_seed: int, i0: int, n: int, U: int, cdf: np.ndarray | None = None) -> np.ndarray:
    """Pool item of reads i0 .. i0+n-1 (ora_pool_index, or ora_zipf_index when cdf is given), vectorised."""
    i = np.arange(i0, i0 + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        r = splitmix64_np(np.uint64(pool_seed) ^ (i * np.uint64(0xD1B54A32D192ED03)))
    if cdf is None:
        return r % np.uint64(U)
    ids = np.searchsorted(np.asarray(cdf, dtype=np.uint64), r >> np.uint64(1), side="right").astype(np.uint64)
    return np.minimum(ids, np.uint64(U - 1))


def pool_counter_table(seed: int, pool_seed: int, U: int, n: int, L: int = 32, i0: int = 0,
                       cdf: np.ndarray | None = None, chunk: int = 1 << 23):
    """The counter result of n pool-drawn L <= 32 reads, derived from the generator alone: keys = the
    generator word of each drawn pool item, counts = bincount of the draw indices, first = global
    index of the first draw.  Returns (keys, counts, first) uint64 arrays sorted by key."""
    assert L <= 32
    counts = np.zeros(U, dtype=np.uint64)
    first = np.full(U, np.iinfo(np.uint64).max, dtype=np.uint64)
    for s0 in range(0, n, chunk):
        m = min(chunk, n - s0)
        ids = pool_ids(pool_seed, i0 + s0, m, U, cdf)
        counts += np.bincount(ids.astype(np.int64), minlength=U).astype(np.uint64)
        u, pos = np.unique(ids, return_index=True)
        new = first[u] == np.iinfo(np.uint64).max
        first[u[new]] = np.uint64(i0 + s0) + pos[new].astype(np.uint64)
    used = np.nonzero(counts)[0].astype(np.uint64)
    with np.errstate(over="ignore"):
        keys = splitmix64_np(np.uint64(seed) + used)
    if L < 32:
        keys &= np.uint64((1 << (2 * L)) - 1)
    o = np.argsort(keys, kind="stable")
    return keys[o], counts[used.astype(np.int64)][o], first[used.astype(np.int64)][o]


RAGGED_LEN_SALT = 0x6A09E667F3BCC909


def ragged_item_lens(seed: int, items: np.ndarray, Lmin: int, Lmax: int) -> np.ndarray:
    """Length of ragged pool items (the ss_synth_ragged_* rule, include/shortseq_amd.h)."""
    with np.errstate(over="ignore"):
        r = splitmix64_np(np.uint64(seed) ^ np.uint64(RAGGED_LEN_SALT) ^ np.asarray(items, np.uint64))
    return (np.uint64(Lmin) + r % np.uint64(Lmax - Lmin + 1)).astype(np.uint32)


def ragged_item_words(seed: int, item: int, L: int) -> list:
    """The packed words of ragged pool item `item` of length L (= the encode of its ASCII)."""
    out = []
    for w in range((L + 31) // 32):
        nb = min(32, L - 32 * w)
        with np.errstate(over="ignore"):
            r = int(splitmix64_np(np.array([seed + 32 * item + w], dtype=np.uint64))[0])
        out.append(r if nb == 32 else r & ((1 << (2 * nb)) - 1))
    return out


def ragged_pool_reads(seed: int, pool_seed: int, U: int, i0: int, n: int, Lmin: int, Lmax: int) -> list:
    """The reads (bytes) of ss_synth_ragged_* for a small n (host restatement)."""
    items = pool_ids(pool_seed, i0, n, U)
    lens = ragged_item_lens(seed, items, Lmin, Lmax)
    out = []
    for p, L in zip(items.tolist(), lens.tolist()):
        ws = ragged_item_words(seed, p, L)
        out.append(bytes(b"ACTG"[(ws[j // 32] >> (2 * (j % 32))) & 3] for j in range(L)))
    return out


def ragged_pool_rows(seed: int, pool_seed: int, U: int, n: int, Lmin: int, Lmax: int, chunk: int = 1 << 23):
    """The drop-in counter's rows for n ragged pool reads, from the generator alone: the drawn items
    in first-occurrence order, each (length, count, words), items of equal content merged.  Returns
    (lens u32 [K], counts u64 [K], words u64 [sum ceil(L/32)]) -- the ss_ingest_results layout."""
    counts = np.zeros(U, dtype=np.uint64)
    first = np.full(U, np.iinfo(np.uint64).max, dtype=np.uint64)
    for s0 in range(0, n, chunk):
        m = min(chunk, n - s0)
        ids = pool_ids(pool_seed, s0, m, U)
        counts += np.bincount(ids.astype(np.int64), minlength=U).astype(np.uint64)
        u, pos = np.unique(ids, return_index=True)
        new = first[u] == np.iinfo(np.uint64).max
        first[u[new]] = np.uint64(s0) + pos[new].astype(np.uint64)
    used = np.nonzero(counts)[0]
    used = used[np.argsort(first[used], kind="stable")]
    lens = ragged_item_lens(seed, used.astype(np.uint64), Lmin, Lmax)
    W = ((lens.astype(np.int64) + 31) // 32)
    woff = np.concatenate([[0], np.cumsum(W)])
    words = np.zeros(int(woff[-1]), dtype=np.uint64)
    for w in range(int(W.max()) if len(W) else 0):
        sel = np.nonzero(W > w)[0]
        with np.errstate(over="ignore"):
            r = splitmix64_np(np.uint64(seed) + np.uint64(32) * used[sel].astype(np.uint64) + np.uint64(w))
        nb = np.minimum(32, lens[sel].astype(np.int64) - 32 * w)
        mask = np.where(nb >= 32, np.uint64(0xFFFFFFFFFFFFFFFF),
                        (np.uint64(1) << (np.uint64(2) * nb.astype(np.uint64))) - np.uint64(1))
        words[woff[sel] + w] = r & mask
    # items of equal content (short lengths repeat: 4^L distinct reads) are one key: merged into the
    # row of their first occurrence (rows are already in first-occurrence order)
    cnt = counts[used].copy()
    keep = np.ones(len(used), dtype=bool)
    seen = {}
    wl = words.tolist()
    for k in range(len(used)):
        key = (int(lens[k]),) + tuple(wl[woff[k]:woff[k + 1]])
        j = seen.get(key)
        if j is None:
            seen[key] = k
        else:
            cnt[j] += cnt[k]
            keep[k] = False
    if keep.all():
        return lens, cnt, words
    wkeep = np.repeat(keep, W)
    return lens[keep], cnt[keep], words[wkeep]


def rows_digest(lens: np.ndarray, counts: np.ndarray, words: np.ndarray) -> str:
    """SHA-256 of the counter rows in order: per row the uint64s [length, count, words...] (the
    ss_ingest_results layout: ceil(L / 32) words per row)."""
    import hashlib
    lens = np.asarray(lens, np.uint64)
    W = (lens.astype(np.int64) + 31) // 32          # ceil(L / 32) words per row (none for L = 0)
    rl = 2 + W
    off = np.concatenate([[0], np.cumsum(rl)])
    flat = np.zeros(int(off[-1]), dtype=np.uint64)
    flat[off[:-1]] = lens
    flat[off[:-1] + 1] = np.asarray(counts, np.uint64)
    woff = np.concatenate([[0], np.cumsum(W)])
    src = np.asarray(words, np.uint64)
    for w in range(int(W.max()) if len(W) else 0):
        sel = np.nonzero(W > w)[0]
        flat[off[sel] + 2 + w] = src[woff[sel] + w]
    return hashlib.sha256(flat.tobytes()).hexdigest()


def table_digest(keys: np.ndarray, counts: np.ndarray, first: np.ndarray) -> str:
    """SHA-256 of the (key, count, first) rows sorted by key (all uint64)."""
    import hashlib
    o = np.argsort(np.asarray(keys, dtype=np.uint64), kind="stable")
    rows = np.stack([np.asarray(keys, dtype=np.uint64)[o], np.asarray(counts, dtype=np.uint64)[o],
                     np.asarray(first, dtype=np.uint64)[o]], 1)
    return hashlib.sha256(np.ascontiguousarray(rows).tobytes()).hexdigest()


def count(reads):
    """Counter oracle over a list of bytes.  Returns [(words tuple, L, count, first_index)] in
    first-occurrence order, or raises ValueError(err) on the first invalid read."""
    n = len(reads)
    lens = np.array([len(r) for r in reads], dtype=np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    if n:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    blob = np.frombuffer(b"".join(reads) or b"\0", dtype=np.uint8)
    uw = np.zeros(max(1, n) * 32, dtype=np.uint64)
    ul = np.zeros(max(1, n), dtype=np.uint32)
    uc = np.zeros(max(1, n), dtype=np.uint64)
    uf = np.zeros(max(1, n), dtype=np.uint64)
    err = OraErr()
    nu = lib().ora_count(_p(blob), _p(offs), _p(lens), n, _p(uw), _p(ul), _p(uc), _p(uf), C.byref(err))
    if nu < 0:
        raise ValueError((err.kind, err.read_index, err.byte_offset, err.nbytes))
    res = []
    for u in range(nu):
        L = int(ul[u])
        nw = 1 if L <= 32 else words_for(L)
        res.append((tuple(int(x) for x in uw[32 * u: 32 * u + nw]), L, int(uc[u]), int(uf[u])))
    return res


# --- the reference's own kernels (oracle/_ref), for validation and the CPU baseline -------------

def ref_available() -> bool:
    return os.path.isdir(os.path.join(REF_DIR, "shortseq"))


def ref_kernel_ptrs():
    """Raw function pointers of the reference's capsule-exported encode kernels."""
    import importlib
    import sys
    if REF_DIR not in sys.path:
        sys.path.insert(0, REF_DIR)
    m64 = importlib.import_module("shortseq.short_seq_64")
    util = importlib.import_module("shortseq.util")
    # the repository's own `shortseq` alias package (the drop-in under the reference's name) must
    # never stand in for the reference here
    if not os.path.abspath(m64.__file__).startswith(os.path.abspath(REF_DIR)):
        raise RuntimeError(f"'shortseq' resolved to {m64.__file__}, not the reference build in {REF_DIR}")
    get = C.pythonapi.PyCapsule_GetPointer
    get.restype = C.c_void_p
    get.argtypes = [C.py_object, C.c_char_p]
    cap64 = m64.__pyx_capi__["_marshall_bytes_64"]
    capar = util.__pyx_capi__["_marshall_bytes_array"]
    p64 = get(cap64, b"uint64_t (uint8_t *, uint8_t)")
    par = get(capar, b"void (uint64_t *, uint8_t *, size_t)")
    return p64, par


def ref_encode_batch(ascii: np.ndarray, n: int, L: int, wpr: int | None = None) -> np.ndarray:
    """Encode a valid fixed-length batch with the reference's own compiled kernels."""
    wpr = wpr_for(L) if wpr is None else wpr
    out = np.zeros(n * wpr, dtype=np.uint64)
    p64, par = ref_kernel_ptrs()
    if L <= 32:
        plib().ref_encode64_batch(p64, _p(ascii), n, L, L, _p(out))
    else:
        plib().ref_encode_array_batch(par, _p(ascii), n, L, L, _p(out), wpr)
    return out.reshape(n, wpr)


def fastq_index(data: bytes):
    """(offsets u64, lens u32) of the kept sequence lines (fast_read.pyx:3-20 rule)."""
    buf = np.frombuffer(data, dtype=np.uint8)
    n = lib().ora_fastq_index(buf.ctypes.data, len(buf), None, None, 0)
    offs = np.zeros(n, dtype=np.uint64)
    lens = np.zeros(n, dtype=np.uint32)
    lib().ora_fastq_index(buf.ctypes.data, len(buf), offs.ctypes.data, lens.ctypes.data, n)
    return offs, lens


def slice_words(words, start: int, n: int) -> list:
    """Packed words of nts [start, start + n) of a read (short_seq.pyx:93-238 restated)."""
    src = np.ascontiguousarray(words, dtype=np.uint64)
    dst = np.zeros(max(1, words_for(n)), dtype=np.uint64)
    lib().ora_slice(_p(src), len(src), start, n, _p(dst))
    return [int(x) for x in dst]
