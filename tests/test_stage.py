"""Host-resident batches through the GPU (ss_stager_* / batch.HostStager): numpy in, numpy out,
bit-exact against the oracle; chunk boundaries, slot reuse, pageable and pinned buffers, padded
rows, first-bad reporting across chunks, decode round trip, fused hamming."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _reads(rng, n, L, p_alias=0.0):
    a = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=n * L)]
    if p_alias:
        m = rng.random(n * L) < p_alias
        a = np.where(m, np.array([1, 3, 7, 20], np.uint8)[rng.integers(0, 4, size=n * L)], a)
    return a.astype(np.uint8).reshape(n, L)


@pytest.mark.parametrize("chunk,nslots", [(4096, 2), (4096, 3), (1 << 16, 4), (64 << 20, 3)])
def test_encode_host_chunks(gpu, oracle, chunk, nslots):
    import shortseq_amd.batch as B
    st = B.HostStager(gpu, chunk_bytes=chunk, nslots=nslots, copy_threads=3)
    rng = np.random.default_rng(chunk + nslots)
    try:
        for L in (1, 17, 31, 32, 33, 64, 96, 100, 128, 512, 1000, 1024):
            n = 3001
            a = _reads(rng, n, L, p_alias=0.02)
            exp, rc, _ = oracle.encode_batch(a.reshape(-1), n, L)
            assert rc == 0
            got = st.encode(a)
            assert got.dtype == np.uint64 and np.array_equal(got, exp), (L, chunk, nslots)
            back = st.decode(exp, L)
            assert np.array_equal(back.reshape(-1), oracle.decode_batch(exp, n, L)), (L, chunk)
    finally:
        st.close()


def test_encode_host_pinned_and_padded(gpu, oracle):
    import shortseq_amd.batch as B
    st = B.HostStager(gpu, chunk_bytes=1 << 16, nslots=3, copy_threads=2)
    rng = np.random.default_rng(5)
    n, L = 20000, 96
    a = _reads(rng, n, L)
    exp, _, _ = oracle.encode_batch(a.reshape(-1), n, L)
    # pinned input and output: DMA'd directly, no staging copies
    pin_in = torch.from_numpy(a.reshape(-1)).pin_memory()
    pin_out = torch.empty(n * 3, dtype=torch.int64).pin_memory()
    outv = pin_out.numpy().view(np.uint64).reshape(n, 3)
    got = st.encode(pin_in.numpy(), L, out=outv)
    assert np.array_equal(got, exp)
    # padded rows: a view of a wider array (stride 112)
    wide = np.zeros((n, 112), np.uint8)
    wide[:, :L] = a
    assert np.array_equal(st.encode(wide[:, :L]), exp)
    # flat bytes with an explicit stride
    assert np.array_equal(st.encode(wide.tobytes(), L, stride=112), exp)
    st.close()


def test_encode_host_first_bad_across_chunks(gpu, oracle):
    import shortseq_amd.batch as B
    st = B.HostStager(gpu, chunk_bytes=8192, nslots=2, copy_threads=0)
    rng = np.random.default_rng(9)
    n, L = 5000, 32
    a = _reads(rng, n, L)
    a[4100, 7] = ord("N")       # chunk 16 (256 reads per 8-KiB chunk)
    a[4700, 0] = ord("x")       # a later chunk: must not win
    with pytest.raises(Exception) as ei:
        st.encode(a)
    assert str(ei.value) == "Unsupported base character: N" and ei.value.read_index == 4100
    # check_errors=False: every other read is still encoded
    got = st.encode(a, check_errors=False)
    fixed = a.copy()
    fixed[4100, 7] = fixed[4700, 0] = ord("A")
    exp, _, _ = oracle.encode_batch(fixed.reshape(-1), n, L)     # the oracle stops at a bad read
    ok = np.ones(n, bool)
    ok[[4100, 4700]] = False
    assert np.array_equal(got[ok], exp[ok])
    st.close()


def test_encode_hamming_ref_host(gpu, oracle):
    import shortseq_amd.batch as B
    st = B.HostStager(gpu, chunk_bytes=1 << 15, nslots=3, copy_threads=2)
    rng = np.random.default_rng(21)
    for L in (12, 32, 96, 150):
        n = 7000
        a = _reads(rng, n, L, p_alias=0.01)
        exp, _, _ = oracle.encode_batch(a.reshape(-1), n, L)
        words, dist = st.encode_hamming_ref(a, L, exp[3])
        assert np.array_equal(words, exp)
        assert np.array_equal(dist, oracle.hamming_ref_batch(exp, n, L, exp[3])), L
    st.close()


def test_encode_host_default_stager_large(gpu, oracle):
    """The module default stager over a multi-chunk batch (64-MiB chunks): generator words."""
    import shortseq_amd.batch as B
    n, L = 3_000_000, 32
    a = B.synth_reads(n, L, seed=4, device=gpu).cpu().numpy()
    got = B.encode_host(a)
    assert np.array_equal(got[::997], oracle.gen_words(4, 0, n, L).reshape(n, 1)[::997])
    back = B.decode_host(got, L)
    assert np.array_equal(back, a)


@pytest.mark.parametrize("pin", ["1", "0"])
def test_stager_stage_split_and_placement(gpu, oracle, monkeypatch, pin):
    """ss_stager_set_timing / ss_stager_stats: the split of timed calls is
    reported per call (host copies for pageable buffers, device H2D / kernel / D2H > 0), untimed
    calls leave nothing, a stats call resets it, and the placement fields are consistent (the copy
    threads pinned only with SHORTSEQ_STAGE_PIN != 0, to at most the CPUs the process may use); the
    words stay the oracle's with timing on."""
    import shortseq_amd.batch as B
    monkeypatch.setenv("SHORTSEQ_STAGE_PIN", pin)
    st = B.HostStager(gpu, chunk_bytes=1 << 20, nslots=3, copy_threads=4)
    rng = np.random.default_rng(7)
    try:
        n, L = 200_000, 32
        a = _reads(rng, n, L)
        exp, rc, _ = oracle.encode_batch(a.reshape(-1), n, L)
        st.encode(a)
        first = st.stats()
        assert all(first[k] == 0.0 for k in B.HostStager.STAGES)       # nothing timed yet
        st.set_timing(True)
        for _ in range(2):
            got = st.encode(a)
        sp = st.stats()
        assert np.array_equal(got.reshape(-1).view(np.uint64), exp.reshape(-1))
        for k in ("copy_in_host", "copy_out_host", "h2d_dev", "kernel_dev", "d2h_dev"):
            assert sp[k] > 0.0, k
        assert st.stats()["h2d_dev"] == 0.0                              # reset by the previous call
        assert sp["copy_threads"] == 4 and sp["affinity_cpus"] >= 1 and sp["gpu_numa_node"] >= -1
        if pin == "0" or sp["gpu_numa_node"] < 0:
            assert sp["pinned_cpus"] == 0
        else:
            assert 0 <= sp["pinned_cpus"] <= sp["affinity_cpus"]
        st.set_timing(False)
    finally:
        st.close()
