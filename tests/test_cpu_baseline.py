"""The CPU-baseline port (oracle/cpu_baseline.cpp, bench.py's cpu_baseline leg) computes what the
oracle computes: encode (table path and PEXT blocks), fused hamming, round trip and the counter, on
1 thread (GIL held, the reference's per-read error checks restated) and on 2 OpenMP threads.  Each
bench_* function asserts its own results against the oracle before it times anything."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import cpu_baseline as cb  # noqa: E402  (test infrastructure)
import oracle  # noqa: E402


@pytest.mark.parametrize("threads", [1, 2])
@pytest.mark.parametrize("L", [32, 96, 100, 512])
def test_port_encode_matches_oracle(threads, L):
    n = 2000
    a = oracle.gen_reads(3, 0, n, L)
    wpr = max(1, (L + 31) // 32)
    words = np.zeros(n * wpr, np.uint64)
    assert cb.lib(threads).cb_encode(a.ctypes.data, n, L, words.ctypes.data, wpr, threads) == 0
    assert np.array_equal(words.reshape(n, wpr), oracle.gen_words(3, 0, n, L))


def test_port_rejects_invalid_bases():
    L, n = 96, 64
    a = oracle.gen_reads(4, 0, n, L).copy()
    a[5 * L + 40] = ord("N")
    a[9 * L + 3] = ord("a")
    words = np.zeros(n * 3, np.uint64)
    assert cb.lib(1).cb_encode(a.ctypes.data, n, L, words.ctypes.data, 3, 1) == 2


@pytest.mark.parametrize("threads", [1, 2])
def test_port_workloads_self_check(threads):
    # the bench functions assert words / distances / round trip / counter against the oracle
    cb.bench_encode(32, 20_000, threads, 0.001)
    cb.bench_encode_hamming(96, 20_000, threads, 0.001)
    cb.bench_roundtrip(512, 4_000, threads, 0.001)
    cb.bench_count(50_000, 1 << 12, threads, 0.001)


def test_gil_checks_toggle_keeps_results():
    L, n = 512, 500
    a = oracle.gen_reads(6, 0, n, L)
    out = []
    for on in (1, 0):
        cb.lib(1).cb_set_gil_checks(on)
        w = np.zeros(n * 16, np.uint64)
        assert cb.lib(1).cb_encode(a.ctypes.data, n, L, w.ctypes.data, 16, 1) == 0
        out.append(w)
    cb.lib(1).cb_set_gil_checks(1)
    assert np.array_equal(out[0], out[1])
    assert cb.lib(1).cb_gil_api() == 1     # inside Python the C-API calls are the ones made
