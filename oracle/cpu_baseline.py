"""TEST / BASELINE INFRASTRUCTURE ONLY — times oracle/libcpubaseline.so (the reference's per-read CPU
algorithms restated in C++, oracle/cpu_baseline.cpp) on bounded samples of the BASELINE workloads,
on 1 host core and on all the cores this process may use (OpenMP).  bench.py's cpu_baseline leg is
the only caller besides the calibration script; nothing under shortseq_amd/ imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libcpubaseline.so")
_lib = None


_lib1 = None


def lib(threads: int = 0):
    """The port.  threads == 1: a PyDLL handle (the GIL stays held, as when Python calls the
    reference's kernels), so the port's per-read error checks (cpu_baseline.cpp err_check) take the
    GIL the way the compiled reference does; otherwise a CDLL handle (GIL released for the OpenMP
    legs)."""
    global _lib, _lib1
    if threads == 1:
        if _lib1 is None:
            lib()
            _lib1 = _bind(C.PyDLL(LIB_PATH))
        return _lib1
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            oracle.build()
        _lib = _bind(C.CDLL(LIB_PATH))
    return _lib


def _bind(L):
    P, U64, U32, I = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
    L.cb_encode.argtypes = [P, U64, U32, P, U32, I]
    L.cb_encode.restype = U64
    L.cb_encode_hamming.argtypes = [P, U64, U32, P, U32, P, P, I]
    L.cb_encode_hamming.restype = U64
    L.cb_hamming_ref.argtypes = [P, U64, U32, U32, P, P, I]
    L.cb_hamming_ref.restype = None
    L.cb_roundtrip.argtypes = [P, U64, U32, P, U32, P, I]
    L.cb_roundtrip.restype = U64
    L.cb_count.argtypes = [P, U64, U32, I, C.POINTER(U64), C.POINTER(U64)]
    L.cb_count.restype = U64
    L.cb_max_threads.restype = I
    L.cb_set_gil_checks.argtypes = [I]
    L.cb_gil_api.restype = I
    return L


def host_threads() -> int:
    """The cores this process may use: OMP_NUM_THREADS when set (the GPU box pins it to the box's
    CPU share), else the affinity mask."""
    v = os.environ.get("OMP_NUM_THREADS")
    if v and v.isdigit() and int(v) > 0:
        return int(v)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _time(fn, target_s: float):
    fn()  # warm (page-faults the outputs)
    passes, t0 = 0, time.perf_counter()
    while True:
        fn()
        passes += 1
        el = time.perf_counter() - t0
        if el >= target_s:
            return passes, el


def _p(a):
    return a.ctypes.data


def bench_encode(L: int, n: int, threads: int, target_s: float, seed: int = 1) -> dict:
    ascii = oracle.gen_reads(seed, 0, n, L)
    wpr = max(1, (L + 31) // 32)
    words = np.zeros(n * wpr, np.uint64)
    assert lib(threads).cb_encode(_p(ascii), n, L, _p(words), wpr, threads) == 0
    assert np.array_equal(words.reshape(n, wpr)[:64], oracle.gen_words(seed, 0, 64, L))
    passes, el = _time(lambda: lib(threads).cb_encode(_p(ascii), n, L, _p(words), wpr, threads), target_s)
    return {"nt_per_s": passes * n * L / el, "reads_per_s": passes * n / el, "sample": f"{passes} x {n} reads x {L} nt"}


def bench_encode_hamming(L: int, n: int, threads: int, target_s: float, seed: int = 2) -> dict:
    ascii = oracle.gen_reads(seed, 0, n, L)
    wpr = max(1, (L + 31) // 32)
    words = np.zeros(n * wpr, np.uint64)
    dist = np.zeros(n, np.uint32)
    ref = oracle.gen_words(seed, 0, 1, L)[0].astype(np.uint64)
    ref = np.ascontiguousarray(np.concatenate([ref, np.zeros(wpr - len(ref), np.uint64)]))
    assert lib(threads).cb_encode_hamming(_p(ascii), n, L, _p(words), wpr, _p(ref), _p(dist), threads) == 0
    exp = oracle.hamming_ref_batch(words.reshape(n, wpr)[:4096], 4096, L, ref)
    assert np.array_equal(dist[:4096], exp)
    passes, el = _time(lambda: lib(threads).cb_encode_hamming(_p(ascii), n, L, _p(words), wpr, _p(ref), _p(dist), threads),
                       target_s)
    return {"pairs_per_s": passes * n / el, "nt_per_s": passes * n * L / el, "sample": f"{passes} x {n} reads x {L} nt"}


def bench_hamming_only(L: int, n: int, threads: int, target_s: float, seed: int = 6) -> dict:
    """C3': hamming vs read 0 on pre-packed words (the XOR-collapse-popcount loop alone)."""
    W = (L + 31) // 32
    words = oracle.splitmix64_np(np.uint64(seed) + np.arange(n * W, dtype=np.uint64)).reshape(n, W)
    if L % 32:
        words[:, -1] &= np.uint64((1 << (2 * (L % 32))) - 1)
    assert np.array_equal(words[:4], oracle.gen_words(seed, 0, 4, L))   # the generator's known answer
    wpr = words.shape[1]
    ref = np.ascontiguousarray(words[0].copy())
    dist = np.zeros(n, np.uint32)
    lib(threads).cb_hamming_ref(_p(words), n, L, wpr, _p(ref), _p(dist), threads)
    assert np.array_equal(dist[:4096], oracle.hamming_ref_batch(words[:4096], 4096, L, ref))
    passes, el = _time(lambda: lib(threads).cb_hamming_ref(_p(words), n, L, wpr, _p(ref), _p(dist), threads), target_s)
    return {"pairs_per_s": passes * n / el, "sample": f"{passes} x {n} pairs x {L} nt"}


def bench_roundtrip(L: int, n: int, threads: int, target_s: float, seed: int = 3) -> dict:
    ascii = oracle.gen_reads(seed, 0, n, L)
    wpr = max(1, (L + 31) // 32)
    words = np.zeros(n * wpr, np.uint64)
    back = np.zeros(n * L, np.uint8)
    assert lib(threads).cb_roundtrip(_p(ascii), n, L, _p(words), wpr, _p(back), threads) == 0
    assert np.array_equal(back, ascii)
    passes, el = _time(lambda: lib(threads).cb_roundtrip(_p(ascii), n, L, _p(words), wpr, _p(back), threads), target_s)
    return {"nt_per_s": passes * n * L / el, "reads_per_s": passes * n / el, "sample": f"{passes} x {n} reads x {L} nt"}


def bench_count(n: int, U: int, threads: int, target_s: float, seed: int = 5, pool_seed: int = 77) -> dict:
    L = 32
    ascii = oracle.gen_pool_reads(seed, pool_seed, U, 0, n, L)
    tot, fs = C.c_uint64(), C.c_uint64()
    uniq = lib(threads).cb_count(_p(ascii), n, L, threads, C.byref(tot), C.byref(fs))
    k, c, f = oracle.pool_counter_table(seed, pool_seed, U, n, L)
    assert uniq == len(k) and tot.value == n and fs.value == int(f.sum()), (uniq, len(k))
    passes, el = _time(lambda: lib(threads).cb_count(_p(ascii), n, L, threads, C.byref(tot), C.byref(fs)), target_s)
    return {"reads_per_s": passes * n / el, "unique": int(uniq), "sample": f"{passes} x {n} reads (pool {U})"}


WORKLOADS = {
    # name: (callable(threads, target_s), unit key)
    "C2_encode_32": (lambda th, s: bench_encode(32, 4_000_000, th, s), "nt_per_s"),
    "C3_encode_hamming_96": (lambda th, s: bench_encode_hamming(96, 2_000_000, th, s), "pairs_per_s"),
    "C3p_hamming_ref_32": (lambda th, s: bench_hamming_only(32, 8_000_000, th, s), "pairs_per_s"),
    "C3p_hamming_ref_96": (lambda th, s: bench_hamming_only(96, 4_000_000, th, s), "pairs_per_s"),
    "C3p_hamming_ref_512": (lambda th, s: bench_hamming_only(512, 1_000_000, th, s), "pairs_per_s"),
    "C4_roundtrip_512": (lambda th, s: bench_roundtrip(512, 400_000, th, s), "nt_per_s"),
    "C5_counter_32": (lambda th, s: bench_count(8_000_000, 1 << 24, th, s), "reads_per_s"),
}


def run_all(target_s: float = 2.0, threads_all: int | None = None) -> dict:
    """Every workload on 1 core and on all usable cores; ~8 x target_s of CPU time plus setup."""
    threads_all = host_threads() if threads_all is None else threads_all
    out = {"cpu": cpu_model(), "nproc": os.cpu_count(), "threads_all": threads_all}
    for name, (fn, unit) in WORKLOADS.items():
        one = fn(1, target_s)
        many = fn(threads_all, target_s) if threads_all > 1 else one
        out[name] = {"unit": unit, "1_core": one[unit], f"{threads_all}_cores": many[unit],
                     "sample_1_core": one["sample"], f"sample_{threads_all}_cores": many["sample"]}
    return out
