# cython: language_level=3, boundscheck=False, wraparound=False, cdivision=True
"""Drop-in front for the reference's Python API (shortseq/__init__.py:1-14).

Per-object operations (pack / str / ^ / == / [] on single reads) run on the host C++ codec
(csrc/host_codec.h): one read is ~tens of ns of work, a kernel launch is microseconds (SURVEY §7).
Batch operations — ShortSeqCounter over a large list, read_and_count_fastq — stage the reads in a
contiguous buffer and run on the GPU through the C ABI (shortseq_amd.batch -> libshortseq_amd.so);
the GPU path raises if the HIP library cannot be used, it never degrades silently.

Object layouts match the reference so sys.getsizeof agrees (short_seq_64.pxd:11-14,
short_seq_192.pxd:11-14, short_seq_var.pxd:14-17): 32 / 48 / 32 + 8*ceil(L/32) bytes.

Documented deviations (DESIGN.md §6): hash() and the counter agree for every key (reference Q5
inserts with the raw word, so counts[pack("G"*32)] raises KeyError there); ShortSeqVar keys are
deduplicated by content (reference Q6 keys them by heap pointer).
"""
from libc.stdint cimport uint8_t, uint64_t, int64_t, int32_t, int16_t
from libc.string cimport memcmp, memcpy, memset, strlen
from libc.stdio cimport FILE, fopen, fclose
from libc.stdlib cimport free, malloc, calloc
from cpython.bytes cimport PyBytes_AS_STRING, PyBytes_GET_SIZE, PyBytes_FromStringAndSize
from cpython.mem cimport PyObject_Calloc, PyObject_Free
from cpython.unicode cimport PyUnicode_DecodeASCII
from cpython.object cimport PyObject
from cpython.list cimport PyList_GET_ITEM, PyList_GET_SIZE

import time

cdef extern from "Python.h":
    ctypedef Py_ssize_t Py_hash_t
    int _PyDict_SetItem_KnownHash(object mp, object key, object item, Py_hash_t hash) except -1
    object PyUnicode_New(Py_ssize_t size, Py_UCS4 maxchar)
    void* PyUnicode_1BYTE_DATA(object o)
    void* PyUnicode_DATA(object o)
    Py_ssize_t PyUnicode_GET_LENGTH(object o)
    bint PyUnicode_Check(object o)
    bint PyBytes_Check(object o)
    bint PyBytes_CheckExact(object o)

cdef extern from "stdio.h":
    ssize_t getline(char** lineptr, size_t* n, FILE* stream) nogil

cdef extern from "host_codec.h":
    ctypedef struct ss_err:
        int32_t kind
        int32_t nbytes
        int64_t read_index
        int64_t byte_offset
    int ssh_encode "ssh::encode"(const uint8_t* s, size_t L, uint64_t* words, ss_err* err) nogil
    void ssh_decode "ssh::decode"(const uint64_t* words, size_t L, char* out) nogil
    uint64_t ssh_hamming "ssh::hamming"(const uint64_t* a, const uint64_t* b, size_t L) nogil

# Domain constants (short_seq_64.pyx:27-28, short_seq_192.pyx:21-22, short_seq_var.pyx:8-10)
MIN_64_NT = 0
MAX_64_NT = 32
MIN_192_NT = 33
MAX_192_NT = 96
MIN_VAR_NT = 97
MAX_VAR_NT = 1024
DEF C_MAX_64 = 32
DEF C_MAX_192 = 96
DEF C_MAX_VAR = 1024
DEF MAX_REPR_LEN = 75

def get_domain_64(): return MIN_64_NT, MAX_64_NT
def get_domain_192(): return MIN_192_NT, MAX_192_NT
def get_domain_var(): return MIN_VAR_NT, MAX_VAR_NT


cdef inline size_t _nwords(size_t L) noexcept nogil:
    return (L + 31) // 32


cdef inline str _to_str(const uint64_t* words, size_t L):
    """_unmarshall_bytes_* (short_seq_64.pyx:114-121, short_seq_192.pyx:114-127,
    short_seq_var.pyx:98-120): decoded straight into a new compact ASCII str (no staging buffer,
    no ASCII re-validation; every character is one of "ACTG")."""
    cdef object s = PyUnicode_New(L, 127)
    if L:
        ssh_decode(words, L, <char*>PyUnicode_1BYTE_DATA(s))
    return s


cdef object _raise_encode_error(const uint8_t* seq, ss_err* err):
    """The reference's exception for a failed marshal (short_seq_64.pyx:105, util.pyx:115/137)."""
    if err.kind == 2:
        raise Exception(f"Sequences longer than {MAX_VAR_NT} bases are not supported.")
    # PyUnicode_DecodeASCII of the offending byte / 8-byte chunk; raises UnicodeDecodeError itself
    # for a non-ASCII byte, exactly as in the reference.
    cdef object bad = PyUnicode_DecodeASCII(<const char*>seq + err.byte_offset, err.nbytes, NULL)
    raise Exception(f"Unsupported base character: {bad}")


# ==================================================================================================
cdef class ShortSeq64:
    """0-32 nt: one packed word + length (short_seq_64.pyx:33-90)."""
    cdef uint64_t _packed
    cdef uint8_t _length

    def __hash__(self):
        return <Py_ssize_t>self._packed            # short_seq_64.pyx:35-36 (-1 -> -2 by CPython)

    def __len__(self):
        return self._length

    def __eq__(self, other):
        if type(other) is ShortSeq64:
            return self._length == (<ShortSeq64>other)._length and \
                   self._packed == (<ShortSeq64>other)._packed
        elif isinstance(other, (str, bytes)):
            return self._length == len(other) and str(self) == other
        return False

    def __ne__(self, other):
        return not self.__eq__(other)

    def __getitem__(self, item):
        return _getitem(&self._packed, self._length, item)

    def __xor__(self, ShortSeq64 other):
        if self._length != other._length:
            raise Exception(f"Hamming distance requires sequences of equal length "
                            f"({self._length} != {other._length})")
        return ssh_hamming(&self._packed, &other._packed, 1)

    def __str__(self):
        return _to_str(&self._packed, self._length)

    def __repr__(self):
        return f"<ShortSeq64 ({self._length} nt): {self}>"

    @property
    def packed(self):
        """The packed words as a tuple of ints (batch-layout interop)."""
        return (self._packed,)


cdef class ShortSeq192:
    """33-96 nt: three inline words + length (short_seq_192.pyx:27-97)."""
    cdef uint64_t _packed[3]
    cdef uint8_t _length

    def __hash__(self):
        return <Py_ssize_t>self._packed[0]         # short_seq_192.pyx:29-30

    def __len__(self):
        return self._length

    def __eq__(self, other):
        if type(other) is ShortSeq192:
            return self._length == (<ShortSeq192>other)._length and \
                   memcmp(self._packed, (<ShortSeq192>other)._packed, _nwords(self._length) * 8) == 0
        elif isinstance(other, (str, bytes)):
            return self._length == len(other) and str(self) == other
        return False

    def __ne__(self, other):
        return not self.__eq__(other)

    def __getitem__(self, item):
        return _getitem(self._packed, self._length, item)

    def __xor__(self, ShortSeq192 other):
        if self._length != other._length:
            raise Exception(f"Hamming distance requires sequences of equal length "
                            f"({self._length} != {other._length})")
        return ssh_hamming(self._packed, other._packed, self._length)

    def __str__(self):
        return _to_str(self._packed, self._length)

    def __repr__(self):
        return f"<ShortSeq192 ({self._length} nt): {self}>"

    @property
    def packed(self):
        return tuple(self._packed[i] for i in range(_nwords(self._length)))


cdef class ShortSeqVar:
    """97-1024 nt: heap words + length (short_seq_var.pyx:15-93)."""
    cdef uint64_t* _packed
    cdef size_t _length

    def __hash__(self):
        return <Py_ssize_t>self._packed[0]         # short_seq_var.pyx:16-17

    def __len__(self):
        return self._length

    def __eq__(self, other):
        if type(other) is ShortSeqVar:
            return self._length == (<ShortSeqVar>other)._length and \
                   memcmp(self._packed, (<ShortSeqVar>other)._packed, _nwords(self._length) * 8) == 0
        elif isinstance(other, (str, bytes)):
            return self._length == len(other) and str(self) == other
        return False

    def __ne__(self, other):
        return not self.__eq__(other)

    def __getitem__(self, item):
        return _getitem(self._packed, self._length, item)

    def __xor__(self, ShortSeqVar other):
        if self._length != other._length:
            raise Exception(f"Hamming distance requires sequences of equal length "
                            f"({self._length} != {other._length})")
        return ssh_hamming(self._packed, other._packed, self._length)

    def __str__(self):
        return _to_str(self._packed, self._length)

    def __repr__(self):
        cdef char buf[MAX_REPR_LEN]
        ssh_decode(self._packed, MAX_REPR_LEN, buf)   # short_seq_var.pyx:86-89
        return f"<ShortSeqVar ({self._length} nt): {PyUnicode_DecodeASCII(buf, MAX_REPR_LEN, NULL)} ... >"

    def __sizeof__(self):
        return sizeof(PyObject) + 16 + _nwords(self._length) * 8   # short_seq_var.pyx:83-84

    def __dealloc__(self):
        if self._packed is not NULL:
            PyObject_Free(self._packed)

    @property
    def packed(self):
        return tuple(self._packed[i] for i in range(_nwords(self._length)))


# Singleton (short_seq.pyx:7)
cdef ShortSeq64 empty = ShortSeq64.__new__(ShortSeq64)


# ==================================================================================================
# Construction (short_seq.pyx:13-74)
cdef object _new(const uint8_t* seq, size_t length):
    cdef ss_err err
    cdef ShortSeq64 o64
    cdef ShortSeq192 o192
    cdef ShortSeqVar ovar
    cdef uint64_t* words
    if length == 0:
        return empty
    elif length <= C_MAX_64:
        o64 = ShortSeq64.__new__(ShortSeq64)
        if ssh_encode(seq, length, &o64._packed, &err):
            _raise_encode_error(seq, &err)
        o64._length = <uint8_t>length
        return o64
    elif length <= C_MAX_192:
        o192 = ShortSeq192.__new__(ShortSeq192)
        if ssh_encode(seq, length, o192._packed, &err):
            _raise_encode_error(seq, &err)
        o192._length = <uint8_t>length
        return o192
    elif length <= C_MAX_VAR:
        words = <uint64_t*>PyObject_Calloc(_nwords(length), sizeof(uint64_t))
        if words is NULL:
            raise MemoryError(f"Error while allocating new ShortSeq of length {length}.")
        if ssh_encode(seq, length, words, &err):
            PyObject_Free(words)
            _raise_encode_error(seq, &err)
        ovar = ShortSeqVar.__new__(ShortSeqVar)
        ovar._packed = words
        ovar._length = length
        return ovar
    raise Exception(f"Sequences longer than {MAX_VAR_NT} bases are not supported.")


cdef object _from_words(const uint64_t* w, size_t length):
    """Object for already-packed words (batch results -> drop-in objects)."""
    cdef ShortSeq64 o64
    cdef ShortSeq192 o192
    cdef ShortSeqVar ovar
    if length == 0:
        return empty
    if length <= C_MAX_64:
        o64 = ShortSeq64.__new__(ShortSeq64)
        o64._packed = w[0]
        o64._length = <uint8_t>length
        return o64
    if length <= C_MAX_192:
        o192 = ShortSeq192.__new__(ShortSeq192)
        memcpy(o192._packed, w, _nwords(length) * 8)
        o192._length = <uint8_t>length
        return o192
    ovar = ShortSeqVar.__new__(ShortSeqVar)
    ovar._packed = <uint64_t*>PyObject_Calloc(_nwords(length), sizeof(uint64_t))
    if ovar._packed is NULL:
        raise MemoryError()
    memcpy(ovar._packed, w, _nwords(length) * 8)
    ovar._length = length
    return ovar


def from_words(words, size_t length):
    """Build a ShortSeq from packed words (sequence of ints)."""
    cdef uint64_t buf[32]
    cdef size_t i, n = _nwords(length)
    if length > C_MAX_VAR:
        raise Exception(f"Sequences longer than {MAX_VAR_NT} bases are not supported.")
    memset(buf, 0, sizeof(buf))
    for i in range(n):
        buf[i] = <uint64_t>(int(words[i]) & 0xFFFFFFFFFFFFFFFF)
    return _from_words(buf, length)


cdef inline object _from_py_str(str s):
    # short_seq.pyx:40-43: the raw PyUnicode buffer, length in code points (SURVEY: UCS-2 quirk kept)
    return _new(<const uint8_t*>PyUnicode_DATA(s), <size_t>PyUnicode_GET_LENGTH(s))


cdef inline object _from_py_bytes(bytes b):
    return _new(<const uint8_t*>PyBytes_AS_STRING(b), <size_t>PyBytes_GET_SIZE(b))


def pack(seq, /):
    """short_seq.pyx:13-28."""
    if PyUnicode_Check(seq):
        if not seq:
            return empty
        return _from_py_str(seq)
    elif PyBytes_Check(seq):
        if not seq:
            return empty
        return _from_py_bytes(seq)
    elif type(seq) is ShortSeq64 or type(seq) is ShortSeq192 or type(seq) is ShortSeqVar:
        return seq
    raise TypeError(f'Cannot pack objects of type "{type(seq)}"')


def from_str(str seq_str):
    if not seq_str:
        return empty
    return _from_py_str(seq_str)


def from_bytes(bytes seq_bytes):
    if not seq_bytes:
        return empty
    return _from_py_bytes(seq_bytes)


# ==================================================================================================
# Subscript / slice (short_seq.pyx:78-238, short_seq_64.pyx:53-75): bit-exact funnel-shift copy of
# nts [start, start + n), trimmed to 2n bits.
cdef object _slice_words(const uint64_t* src, size_t start, size_t n):
    cdef uint64_t buf[32]
    cdef size_t bit = 2 * start, nw = _nwords(n), i, w, o
    cdef size_t tail = (2 * n) % 64
    memset(buf, 0, sizeof(buf))
    w = bit // 64
    o = bit % 64
    for i in range(nw):
        if o == 0:
            buf[i] = src[w + i]
        else:
            buf[i] = src[w + i] >> o
            if (w + i + 1) * 32 < start + n:       # only words that hold nts of the slice
                buf[i] |= src[w + i + 1] << (64 - o)
    if tail:
        buf[nw - 1] &= (1ULL << tail) - 1
    return _from_words(buf, n)


cdef object _getitem(const uint64_t* packed, size_t length, item):
    cdef Py_ssize_t index, start, stop, step, slen
    cdef ShortSeq64 one
    if isinstance(item, slice):
        start, stop, step = item.indices(length)
        if step != 1:
            raise TypeError("Slice step not supported")
        slen = stop - start if stop > start else 0
        if slen == 0:
            return empty
        return _slice_words(packed, start, slen)
    elif isinstance(item, int):
        index = item
        if index < 0:
            index += length
        if index < 0 or index >= <Py_ssize_t>length:
            raise IndexError("Sequence index out of range")
        one = ShortSeq64.__new__(ShortSeq64)
        one._packed = (packed[index // 32] >> (2 * (index % 32))) & 3
        one._length = 1
        return one
    raise TypeError(f"Invalid index type: {type(item)}")


# ==================================================================================================
# Counter (counter.pyx:10-70)
GPU_MIN_READS = 1 << 16     # below this a list is counted on the host (launch + copy overhead)


cdef class ShortSeqCounter(dict):
    """dict subclass {ShortSeq: count} in first-occurrence order (counter.pyx:10-54).

    ShortSeqCounter(list_of_bytes, device="auto"): lists of >= GPU_MIN_READS reads are encoded and
    counted on the GPU (one hash-and-atomic-count kernel per read length <= 32); device="host"
    forces the per-object host path, device="cuda"/"cuda:N" forces the GPU.
    """

    def __init__(self, source=None, device="auto"):
        super().__init__()
        if type(source) is list:                    # counter.pyx:14: only lists are consumed
            self._count_list(source, device)

    def __setitem__(self, key, val):
        if type(key) not in (ShortSeq64, ShortSeq192, ShortSeqVar):
            raise TypeError(f"{self.__class__} does not support {type(key)} keys")
        dict.__setitem__(self, key, val)

    cdef _count_list(self, list it, device):
        cdef Py_ssize_t n = PyList_GET_SIZE(it)
        use_gpu = False
        if device != "host" and n >= (GPU_MIN_READS if device == "auto" else 0):
            if device == "auto":
                import torch
                use_gpu = torch.cuda.is_available()
            else:
                use_gpu = True
        if use_gpu:
            _count_batch_gpu(self, it, device)
        else:
            self._count_host(it)

    cdef _count_host(self, list it):
        cdef Py_ssize_t i, n = PyList_GET_SIZE(it)
        cdef object item, seq
        for i in range(n):
            item = <object>PyList_GET_ITEM(it, i)
            if not PyBytes_CheckExact(item):
                raise TypeError(f"expected bytes, {type(item).__name__} found")
            seq = _from_py_bytes(item)
            dict.__setitem__(self, seq, dict.get(self, seq, 0) + 1)


def _resolve_device(device):
    import torch
    if device in ("auto", "cuda"):
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(device)


def _count_batch_gpu(ShortSeqCounter self, list reads, device):
    """Batch path (shortseq_amd/ingest.py): the reads are joined into one pinned buffer, copied up
    once, split by length on the device (the length is part of the key, short_seq_64.pyx:41-44),
    each length group gathered densely and counted by one GPU table; the dict is rebuilt in
    first-occurrence order.  The first rejected read in list order raises the reference's error."""
    import numpy as np
    from . import ingest

    cdef Py_ssize_t i, n = PyList_GET_SIZE(reads), ln
    cdef size_t total = 0
    cdef object item
    cdef char* dst
    lens_np = np.empty(n, dtype=np.int64)
    cdef int64_t[:] lens = lens_np
    for i in range(n):
        item = <object>PyList_GET_ITEM(reads, i)
        if not PyBytes_CheckExact(item):
            # the host loop would raise here unless an earlier read is invalid: find out first
            _raise_first_error(reads, i)
            raise TypeError(f"expected bytes, {type(item).__name__} found")
        lens[i] = PyBytes_GET_SIZE(item)
        total += lens[i]
    # concatenate straight into the pinned staging buffer (no intermediate joined bytes object)
    dst = <char*><size_t>ingest._staging(total).data_ptr()
    for i in range(n):
        ln = lens[i]
        memcpy(dst, PyBytes_AS_STRING(<object>PyList_GET_ITEM(reads, i)), ln)
        dst += ln
    gc = ingest.count_list(reads, lens_np, _resolve_device(device), staged=True)
    _fill_from_groups(self, gc)


def _order_groups_host(groups):
    """finish() groups in any row order -> (groups sorted by first index, group sequence or None);
    the host-side equivalent of LengthGroupCounter.finish_ordered's device sort."""
    import numpy as np
    out, firsts = [], []
    for (Lg, w, c, f) in groups:
        f = np.asarray(f, dtype=np.int64)
        o = np.argsort(f, kind="stable")
        out.append((Lg, np.ascontiguousarray(np.asarray(w, dtype=np.uint64)[o]), np.asarray(c, dtype=np.int64)[o],
                    f[o]))
        firsts.append(f[o])
    if len(out) <= 1:
        return out, None
    allf = np.concatenate(firsts)
    allg = np.repeat(np.arange(len(out), dtype=np.int16), [len(f) for f in firsts])
    return out, allg[np.argsort(allf, kind="stable")]


cdef _fill_from_groups(ShortSeqCounter self, gc):
    """Insert the per-length GPU results into the dict in first-occurrence (= reference) order.
    The order comes from the device (gc.finish_ordered: every group sorted by first index plus the
    group of each key in global order), so this loop reads every array front to back, builds each
    key object and inserts it with its known hash: no per-key __hash__ call, tuple or sort.  (A
    presized scratch dict merged into self measured slower: the merge re-touches every key.)"""
    import numpy as np
    cdef int16_t[::1] gseq_v
    cdef Py_ssize_t i, m = 0, ng, g = 0
    cdef int64_t ef = 0
    cdef bint empty_pending, one = True
    cdef Py_hash_t h
    cdef const uint64_t* wp
    cdef int64_t[::1] cv
    cdef int64_t[::1] fv
    if hasattr(gc, "finish_ordered"):
        groups, (ecount, efirst), gseq = gc.finish_ordered()
    else:
        groups, (ecount, efirst) = gc.finish()
        groups, gseq = _order_groups_host(groups)
    if not groups:
        if ecount:
            dict.__setitem__(self, empty, ecount)
        return
    ng = len(groups)
    # per-group cursors over C pointers (the groups' arrays stay referenced by `keep`)
    keep = []
    cdef uint64_t** wps = <uint64_t**>malloc(ng * sizeof(uint64_t*))
    cdef int64_t** cps = <int64_t**>malloc(ng * sizeof(int64_t*))
    cdef int64_t** fps = <int64_t**>malloc(ng * sizeof(int64_t*))
    cdef size_t* lens = <size_t*>malloc(ng * sizeof(size_t))
    cdef size_t* wstride = <size_t*>malloc(ng * sizeof(size_t))
    cdef Py_ssize_t* cur = <Py_ssize_t*>calloc(ng, sizeof(Py_ssize_t))
    cdef uint64_t[:, ::1] kv
    if wps == NULL or cps == NULL or fps == NULL or lens == NULL or wstride == NULL or cur == NULL:
        free(wps); free(cps); free(fps); free(lens); free(wstride); free(cur)
        raise MemoryError()
    try:
        for g in range(ng):
            Lg, w, c, f = groups[g]
            w = np.ascontiguousarray(w, dtype=np.uint64)
            if w.ndim == 1:
                w = w.reshape(-1, 1)
            c = np.ascontiguousarray(c, dtype=np.int64)
            f = np.ascontiguousarray(f, dtype=np.int64)
            keep.append((w, c, f))
            kv = w
            cv = c
            fv = f
            wps[g] = &kv[0, 0] if kv.shape[0] else NULL
            cps[g] = &cv[0] if cv.shape[0] else NULL
            fps[g] = &fv[0] if fv.shape[0] else NULL
            lens[g] = Lg
            wstride[g] = kv.shape[1]
            m += kv.shape[0]
        if gseq is not None:
            one = False
            gseq_v = np.ascontiguousarray(gseq, dtype=np.int16)
        empty_pending = ecount > 0
        if empty_pending:
            ef = efirst
        for i in range(m):
            if not one:
                g = gseq_v[i]
            if empty_pending and fps[g][cur[g]] > ef:
                dict.__setitem__(self, empty, ecount)
                empty_pending = False
            wp = wps[g] + cur[g] * wstride[g]
            # the objects' own __hash__ (packed word 0; CPython maps -1 to -2), given to the dict
            # directly as the reference's counter does (counter.pyx:44-50)
            h = <Py_hash_t>wp[0]
            if h == -1:
                h = -2
            _PyDict_SetItem_KnownHash(self, _from_words(wp, lens[g]), cps[g][cur[g]], h)
            cur[g] += 1
        if empty_pending:
            dict.__setitem__(self, empty, ecount)
    finally:
        free(wps); free(cps); free(fps); free(lens); free(wstride); free(cur)


def _fill_groups(ShortSeqCounter counter, gc):
    """Fill `counter` from an object with finish() -> (groups, (empty_count, empty_first)) in the
    ingest.LengthGroupCounter format (host-side; used by the GPU paths and by the CPU tests)."""
    _fill_from_groups(counter, gc)


def _raise_first_error(list reads, Py_ssize_t upto):
    """Re-run the reference's loop on reads[0:upto] (host codec) so the first failure raises exactly
    the exception the reference raises."""
    cdef Py_ssize_t i
    cdef object item
    for i in range(upto):
        item = <object>PyList_GET_ITEM(reads, i)
        if not PyBytes_CheckExact(item):
            raise TypeError(f"expected bytes, {type(item).__name__} found")
        _from_py_bytes(item)


def read_and_count_fastq(filename, device="auto"):
    """counter.pyx:57-70 + fast_read.pyx:3-20: keep line 2 of every 4 lines; each kept line loses
    exactly its last character (strlen - 1, short_seq.pyx:50-52); prints the reference's timings.
    device "auto" (a GPU when present) / "cuda[:N]": the file is streamed to HBM in pinned chunks
    and indexed, split by length and counted there (shortseq_amd/ingest.py); "host": the
    reference's per-line loop."""
    if device != "host":
        use_gpu = True
        if device == "auto":
            import torch
            use_gpu = torch.cuda.is_available()
        if use_gpu:
            return _read_and_count_fastq_gpu(filename, device)
    cdef FILE* f
    cdef char* line = NULL
    cdef size_t cap = 0
    cdef ssize_t got
    cdef size_t count = 1
    cdef size_t ln
    seqs = []
    t1 = time.time()
    fname = filename.encode("utf-8")
    f = fopen(fname, "rb")
    if f == NULL:
        raise Exception(f"{str(fname)}: Something went wrong while reading this file.")
    try:
        while True:
            got = getline(&line, &cap, f)
            if got == -1:
                break
            if count % 2 == 0 and count % 4 != 0:
                ln = strlen(line)
                if ln == 0:   # strlen - 1 underflows in the reference -> the too-long error
                    raise Exception(f"Sequences longer than {MAX_VAR_NT} bases are not supported.")
                seqs.append(PyBytes_FromStringAndSize(line, ln - 1))
            count += 1
    finally:
        fclose(f)
        free(line)
    t2 = time.time()
    counts = ShortSeqCounter(seqs, device="host")
    t3 = time.time()
    print(f"{t2-t1:.2f}s to read {len(seqs)} total seqs, and {t3 - t2:.2f}s to count {len(counts)} unique sequences")
    return counts


def _read_and_count_fastq_gpu(filename, device):
    import os
    from . import ingest
    fname = filename.encode("utf-8")
    if not os.path.isfile(filename):
        raise Exception(f"{str(fname)}: Something went wrong while reading this file.")
    t1 = time.time()
    gc, nseqs = ingest.count_fastq(filename, _resolve_device(device))
    t2 = time.time()
    counts = ShortSeqCounter()
    _fill_from_groups(counts, gc)
    t3 = time.time()
    print(f"{t2-t1:.2f}s to read {nseqs} total seqs, and {t3 - t2:.2f}s to count {len(counts)} unique sequences")
    return counts
