"""Shared fixtures.  `-m gpu` tests need an MI355X (run through gpurun); everything else runs on CPU."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
# SHORTSEQ_TEST_ROOT: import the package and the oracle from another build of them (scripts/
# sanitize_cpu.sh points it at build/asan); data files still come from this checkout
_ROOT = os.environ.get("SHORTSEQ_TEST_ROOT", REPO)
for p in (_ROOT, os.path.join(_ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    import oracle as o  # test infrastructure only
    o.lib()
    return o


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "golden_cases.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def digests():
    with open(os.path.join(GOLDEN, "golden_digests.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected without a HIP device (run -m 'not gpu' on CPU-only hosts)")
    import shortseq_amd.batch as B
    B.lib()
    return torch.device("cuda", 0)
