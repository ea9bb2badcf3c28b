"""ctypes binding of lib/libshortseq_amd.so — the C ABI declared in include/shortseq_amd.h.

There is no fallback: if the library is missing or fails to load, every GPU entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

from .build import LIB

SS_OK = 0
SS_EINVALID_BASE = 1
SS_ETOO_LONG = 2
SS_EARG = -1
SS_EHIP = -2
SS_ENOMEM = -3
SS_EFULL = -4


class SsErr(C.Structure):
    _fields_ = [("kind", C.c_int32), ("nbytes", C.c_int32),
                ("read_index", C.c_int64), ("byte_offset", C.c_int64)]


class NativeError(RuntimeError):
    """A C-ABI call failed (argument or HIP runtime error)."""


# (name, restype, argtypes) for every exported symbol of include/shortseq_amd.h
_P, _U64, _U32, _I32, _SZ = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int32, C.c_size_t
SIGNATURES = [
    ("ss_abi_version", C.c_int, []),
    ("ss_last_error_string", C.c_char_p, []),
    ("ss_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("ss_set_device", C.c_int, [C.c_int]),
    ("ss_get_device", C.c_int, [C.POINTER(C.c_int)]),
    ("ss_pinned_alloc", C.c_int, [C.POINTER(C.c_void_p), _SZ]),
    ("ss_pinned_free", C.c_int, [_P]),
    ("ss_encode_fixed", C.c_int, [_P, _U64, _U32, _U64, _P, _U32, _P, _P]),
    ("ss_encode_var", C.c_int, [_P, _P, _P, _U64, _P, _U32, _P, _P]),
    ("ss_decode_fixed", C.c_int, [_P, _U64, _U32, _U32, _P, _U64, _P]),
    ("ss_decode_var", C.c_int, [_P, _P, _U64, _U32, _P, _P, _P]),
    ("ss_hamming_ref", C.c_int, [_P, _U64, _U32, _U32, _P, _P, _P]),
    ("ss_hamming_pair", C.c_int, [_P, _P, _U64, _U32, _U32, _P, _P]),
    ("ss_encode_hamming_ref", C.c_int, [_P, _U64, _U32, _U64, _P, _U32, _P, _P, _P, _P]),
    ("ss_counter_create", C.c_int, [_U64, C.POINTER(C.c_void_p)]),
    ("ss_counter_destroy", C.c_int, [_P]),
    ("ss_counter_reset", C.c_int, [_P, _P]),
    ("ss_counter_capacity", _U64, [_P]),
    ("ss_counter_reserve", C.c_int, [_P, _U64]),
    ("ss_counter_reserved", _U64, [_P]),
    ("ss_counter_release", C.c_int, [_P]),
    ("ss_counter_insert_fixed", C.c_int, [_P, _P, _U64, _U32, _U64, _U64, _P, _P]),
    ("ss_counter_merge", C.c_int, [_P, _P, _P, _P, _P, _U64, _P]),
    ("ss_counter_merge_words", C.c_int, [_P, _P, _P, _P, _U64, _P]),
    ("ss_counter_set_spill_limit", C.c_int, [_P, _U64]),
    ("ss_counter_set_length", C.c_int, [_P, _U32]),
    ("ss_counter_length", C.c_int, [_P]),
    ("ss_counter_set_words", C.c_int, [_P, _U32]),
    ("ss_counter_insert_words", C.c_int, [_P, _P, _U64, _U64, _P]),
    ("ss_counter_overflow", C.c_int, [_P, _P, _P]),
    ("ss_counter_size", C.c_int, [_P, _P, _P]),
    ("ss_counter_set_timing", C.c_int, [_P, C.c_int]),
    ("ss_counter_pass_times", C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    ("ss_counter_extract", C.c_int, [_P, _U32, _P, _P, _P, _P, _U64, _P, _P]),
    ("ss_counter_words", C.c_int, [_P]),
    ("ss_counter_extract_words", C.c_int, [_P, _U32, _P, _P, _P, _P, _P, _U64, _P, _P]),
    ("ss_counter_geometry", C.c_int, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    ("ss_counter_extract_ranges", C.c_int, [_P, _U32, _P, _P, _P, _P, _U64, _P, _P]),
    ("ss_counter_merge_runs", C.c_int, [_P, _P, _P, _P, _P, _U32, _U64, _U32, _U32, _U32, _P, _P]),
    ("ss_counter_pack_ranges", C.c_int, [_P, _U32, _I32, _U64, _P, _U64, _P, _P]),
    ("ss_counter_merge_packed", C.c_int, [_P, _P, _P, _P, _U32, _U64, _U32, _U32, _U32, _P, _P]),
    ("ss_synth_reads", C.c_int, [_P, _U64, _U64, _U64, _U32, _U64, _P]),
    ("ss_synth_pool_reads", C.c_int, [_P, _U64, _U64, _U64, _U64, _U64, _U32, _U64, _P]),
    ("ss_synth_zipf_reads", C.c_int, [_P, _U64, _U64, _P, _U64, _U64, _U64, _U32, _U64, _P]),
    ("ss_synth_ragged_lens", C.c_int, [_P, _U64, _U64, _U64, _U64, _U64, C.c_uint32, C.c_uint32, _P]),
    ("ss_synth_ragged_reads", C.c_int, [_P, _P, _U64, _U64, _U64, _U64, _U64, C.c_uint32, C.c_uint32, _P]),
    ("ss_slice_fixed", C.c_int, [_P, _U64, _U32, _U32, _U32, _U32, _P, _U32, _P]),
    ("ss_slice_var", C.c_int, [_P, _U64, _U32, _P, _P, _P, _P, _U32, _P]),
    ("ss_hamming_all_pairs", C.c_int, [_P, _U64, _U32, _U32, _U32, _P, _P, _U64, _P, _P]),
    ("ss_hamming_all_pairs_ex", C.c_int, [_P, _U64, _U32, _U32, _U32, _P, _P, _U64, _P, _U32, _P]),
    ("ss_fastq_scan_ws_bytes", _U64, [_U64]),
    ("ss_fastq_scan", C.c_int, [_P, _U64, _P, _U64, _P, _P]),
    ("ss_fastq_index", C.c_int, [_P, _U64, _U64, C.c_int, _P, _P, _P, _P, _U64, _P, _P]),
    ("ss_fastq_onepass_ws_bytes", _U64, [_U64, _U64]),
    ("ss_fastq_index_onepass", C.c_int, [_P, _U64, _U64, C.c_int, _P, _U64, _P, _P, _P, _U64, _P, _P]),
    ("ss_gather_rows", C.c_int, [_P, _U64, _P, _P, _U64, _U32, _P, _U64, _P]),
    ("ss_ingest_create", C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    ("ss_ingest_destroy", C.c_int, [_P]),
    ("ss_ingest_reset", C.c_int, [_P]),
    ("ss_ingest_set_exact", C.c_int, [_P, C.c_int]),
    ("ss_ingest_set_row_limit", C.c_int, [_P, _U64]),
    ("ss_ingest_set_count_limit", C.c_int, [_P, _U64]),
    ("ss_ingest_staging", C.c_int, [_P, _U64, C.POINTER(C.c_void_p)]),
    ("ss_ingest_add_blob", C.c_int, [_P, _P, _P, _U64]),
    ("ss_ingest_add_fastq", C.c_int, [_P, C.c_char_p, _U64, C.POINTER(C.c_uint64)]),
    ("ss_fastq_split", C.c_int, [C.c_char_p, C.c_uint32, _P, _P]),
    ("ss_ingest_add_fastq_range", C.c_int, [_P, C.c_char_p, _U64, _U64, _U64, _U64, C.POINTER(C.c_uint64)]),
    ("ss_ingest_add_device", C.c_int, [_P, _P, _U64, _P, _P, _U64]),
    ("ss_ingest_error", C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_int), _P, _U64, C.POINTER(C.c_uint64)]),
    ("ss_ingest_finish", C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("ss_ingest_fastq_stages", C.c_int, [_P, _P, _P]),
    ("ss_ingest_results", C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    ("ss_ingest_set_results_format", C.c_int, [_P, C.c_int]),
    ("ss_ingest_results_compact", C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                            C.POINTER(C.c_uint32), C.POINTER(C.c_void_p)]),
    ("ss_ingest_export", C.c_int, [_P, C.POINTER(C.c_uint64)]),
    ("ss_ingest_merge", C.c_int, [_P, _P, _U64]),
    ("ss_ingest_reserve_merge", C.c_int, [_P, _P, _U32]),
    ("ss_stager_create", C.c_int, [C.c_int, _U64, _U32, _U32, C.POINTER(C.c_void_p)]),
    ("ss_stager_destroy", C.c_int, [_P]),
    ("ss_stager_set_timing", C.c_int, [_P, C.c_int]),
    ("ss_stager_stats", C.c_int, [_P, _P, _P]),
    ("ss_encode_host", C.c_int, [_P, _P, _U64, _U32, _U64, _P, _U32, C.POINTER(C.c_uint64)]),
    ("ss_encode_hamming_ref_host", C.c_int, [_P, _P, _U64, _U32, _U64, _P, _U32, _P, _P, C.POINTER(C.c_uint64)]),
    ("ss_decode_host", C.c_int, [_P, _P, _U64, _U32, _U32, _P, _U64]),
    ("ss_host_encode", C.c_int, [_P, _U64, _P, C.POINTER(SsErr)]),
    ("ss_host_decode", None, [_P, _U64, _P]),
    ("ss_host_hamming", _U64, [_P, _P, _U64]),
]

_lib = None


def lib():
    """Load the HIP library (building it first if this is a dev checkout without it)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            from .build import build_hip
            build_hip()
        L = C.CDLL(LIB)
        # A/B runs of an older library build (scripts/gpu.sh libab) may lack symbols added since
        lenient = os.environ.get("SHORTSEQ_AMD_LENIENT_ABI") == "1"
        for name, res, args in SIGNATURES:
            if lenient and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.ss_abi_version() != 1:
            raise NativeError("libshortseq_amd ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != SS_OK:
        msg = lib().ss_last_error_string().decode(errors="replace")
        raise NativeError(f"{what} failed (status {rc}): {msg}")
