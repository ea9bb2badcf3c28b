"""In-tree build of the native pieces (no pip install; the built files travel with the repo).

  lib/libshortseq_amd.so   hipcc --offload-arch=gfx950: kernels + C ABI (include/shortseq_amd.h)
  _shortseq*.so            Cython front (per-object drop-in types, host C++ codec compiled in); binds
                           lib/libshortseq_amd.so's batch engine (ss_ingest_*) at the first batch call

`python -m shortseq_amd.build` rebuilds whatever is stale.
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(PKG, "lib", "libshortseq_amd.so")
HIP_SOURCES = ["ss_codec.hip", "ss_counter.hip", "ss_fastq.hip", "ss_allpairs.hip", "ss_runtime.hip", "ss_ingest.hip",
               "ss_stage.hip"]
HIP_DEPS = HIP_SOURCES + ["ss_device.h", "ss_internal.h", "host_codec.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SHORTSEQ_AMD_ARCH", "gfx950")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_hip(force: bool = False, verbose: bool = False) -> str:
    deps = [os.path.join(CSRC, f) for f in HIP_DEPS] + [os.path.join(INCLUDE, "shortseq_amd.h"), os.path.abspath(__file__)]
    if force or _stale(LIB, deps):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        tmp = LIB + ".tmp"
        # -amdgpu-mfma-vgpr-form: MFMA results in VGPRs (no v_accvgpr_read before the all-pairs hit
        # test; tools/tune_allpairs.hip, 100k-200k x 12 nt: 14.1 -> 14.6 T pairs/s, same hits)
        cmd = [HIPCC, "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared",
               "-mllvm", "-amdgpu-mfma-vgpr-form=1",
               "-Xarch_host", "-mbmi2", "-Xarch_host", "-mpopcnt", "-I" + INCLUDE,
               *[os.path.join(CSRC, f) for f in HIP_SOURCES], "-o", tmp]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(tmp, LIB)
    return LIB


def _ext_path(name: str) -> str:
    return os.path.join(PKG, name + sysconfig.get_config_var("EXT_SUFFIX"))


def build_cython(force: bool = False, verbose: bool = False) -> str:
    pyx = os.path.join(CSRC, "_shortseq.pyx")
    out = _ext_path("_shortseq")
    deps = [pyx, os.path.join(CSRC, "host_codec.h"), os.path.join(INCLUDE, "shortseq_amd.h"), LIB]
    if not os.path.exists(pyx):
        return out
    if force or _stale(out, deps):
        build_dir = os.path.join(REPO, "build", "cython")
        os.makedirs(build_dir, exist_ok=True)
        cpp = os.path.join(build_dir, "_shortseq.cpp")
        subprocess.run([sys.executable, "-m", "cython", "-3", "--cplus", "--module-name", "shortseq_amd._shortseq",
                        "-I", CSRC, pyx, "-o", cpp],
                       check=True, stdout=None if verbose else subprocess.DEVNULL)
        inc = sysconfig.get_paths()["include"]
        tmp = out + ".tmp"
        # the HIP C ABI library (ss_ingest_* batch engine) is dlopen'ed at the first batch call
        cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-mbmi2", "-mpopcnt", "-march=x86-64-v3",
               "-fno-strict-aliasing", "-w", "-I" + inc, "-I" + CSRC, "-I" + INCLUDE, cpp, "-ldl", "-o", tmp]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(tmp, out)
    return out


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_hip(force, verbose)
    build_cython(force, verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, verbose=True)
