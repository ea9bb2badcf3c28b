"""The C-ABI boundary: the library loads on a CPU-only host, exports every symbol declared in
include/shortseq_amd.h, the host codec matches the oracle, and the product never touches oracle/."""
import ctypes as C
import os
import re

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(REPO, "include", "shortseq_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ss_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    from shortseq_amd import _native
    lib = _native.lib()
    names = declared_symbols()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), n
    bound = {s[0] for s in _native.SIGNATURES}
    assert set(names) == bound, set(names) ^ bound
    assert lib.ss_abi_version() == 1


_NO_DEVICE_CHILD = r"""
import ctypes as C, sys
sys.path.insert(0, sys.argv[1])
from shortseq_amd import _native
lib = _native.lib()
n = C.c_int(-1)
lib.ss_device_count(C.byref(n))
assert n.value == 0, ("device visible", n.value)
fb = C.c_uint64(0)
assert lib.ss_encode_fixed(None, 10, 32, 32, None, 1, C.addressof(fb), None) != 0
import shortseq_amd as sq
try:
    sq.ShortSeqCounter([b"ACGT"] * 10, device="cuda")
except Exception as e:
    print("RAISED", type(e).__name__)
else:
    raise SystemExit("counted a batch without a device")
"""


def test_no_device_is_an_error_not_a_fallback():
    """Without a GPU the device entry points fail loudly (SS_EHIP/EARG) and a batch forced onto the
    GPU raises: nothing computes on a silent fallback.  Runs in a child that sees no device
    (HIP_VISIBLE_DEVICES=-1), so it checks the same thing on a GPU box as on a CPU-only host."""
    import subprocess
    import sys
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1")
    r = subprocess.run([sys.executable, "-c", _NO_DEVICE_CHILD, REPO], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "RAISED" in r.stdout, r.stdout


def test_product_does_not_import_oracle():
    """Only tests/, smoke() and bench.py's cpu_baseline may use oracle/ (the checker)."""
    pat = re.compile(r"\bimport\s+oracle|\bfrom\s+oracle|liboracle|\bora_[a-z_]+\s*\(|oracle/_ref")
    pkg = os.path.join(REPO, "shortseq_amd")
    for root, _dirs, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".pyx", ".pxd", ".hip", ".h", ".cpp")):
                text = open(os.path.join(root, f), encoding="utf-8", errors="replace").read()
                assert not pat.search(text), f


def test_host_codec_matches_oracle(oracle, golden):
    from shortseq_amd import _native
    lib = _native.lib()
    rng = np.random.default_rng(3)
    alphabet = np.frombuffer(b"ACGT\x01\x03\x07\x14NacgU*\n\xc1\x81\xff", np.uint8)
    for L in list(range(0, 100)) + [127, 128, 129, 500, 1023, 1024, 1025]:
        for rep in range(20):
            p_bad = [0.0, 0.01, 0.2][rep % 3]
            codes = np.where(rng.random(L) < p_bad, rng.integers(4, len(alphabet), L), rng.integers(0, 7, L))
            seq = alphabet[codes].astype(np.uint8).tobytes()
            wo, eo = oracle.encode_one(seq, 32)
            wh = np.zeros(32, np.uint64)
            eh = _native.SsErr()
            buf = np.frombuffer(seq, np.uint8) if L else np.zeros(1, np.uint8)
            rc = lib.ss_host_encode(buf.ctypes.data, L, wh.ctypes.data, C.byref(eh))
            assert rc == eo.kind, (L, seq)
            if rc == 1:
                assert (eh.byte_offset, eh.nbytes) == (eo.byte_offset, eo.nbytes)
            elif rc == 0:
                nw = max(1, (L + 31) // 32)
                assert np.array_equal(wh[:nw], wo[:nw]), (L, seq)
    # decode + hamming on the golden vectors
    for v in golden["vectors"]:
        L = v["L"]
        wa = np.array([int(h, 16) for h in v["words_a"]] + [0] * 32, np.uint64)
        wb = np.array([int(h, 16) for h in v["words_b"]] + [0] * 32, np.uint64)
        out = C.create_string_buffer(max(L, 1))
        lib.ss_host_decode(wa.ctypes.data, L, out)
        assert out.raw[:L].decode() == v["str_a"]
        assert lib.ss_host_hamming(wa.ctypes.data, wb.ctypes.data, L) == v["hamming"]


_AUTO_NO_LIB_CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
import shortseq_amd as sq
reads = [b"ACGT" * 8, b"GATTACA"] * 40_000          # >= GPU_MIN_READS: "auto" would pick a GPU
c = sq.ShortSeqCounter(reads)                        # no HIP library here: the host path, not an error
assert [(str(k), v) for k, v in c.items()] == [("ACGT" * 8, 40_000), ("GATTACA", 40_000)], list(c.items())
for dev in ("cuda", "cuda:0", "all", [0, 0]):
    try:
        sq.ShortSeqCounter(reads, device=dev)
    except ImportError:
        pass
    else:
        raise SystemExit(f"device={dev!r} counted without the HIP library")
print("AUTO OK")
"""


def test_auto_without_hip_library_takes_host_path(tmp_path):
    """with device="auto" a host without a usable HIP library counts on the host (the
    reference's behaviour) instead of raising ImportError; explicit GPU choices still raise.  The
    package is copied without lib/libshortseq_amd.so into a scratch directory."""
    import shutil
    import subprocess
    import sys
    dst = tmp_path / "shortseq_amd"
    shutil.copytree(os.path.join(REPO, "shortseq_amd"), dst, ignore=shutil.ignore_patterns("lib", "__pycache__"))
    r = subprocess.run([sys.executable, "-c", _AUTO_NO_LIB_CHILD, str(tmp_path)], capture_output=True, text=True,
                       timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0 and "AUTO OK" in r.stdout, r.stdout + r.stderr
