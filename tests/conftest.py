import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "better-search-rag-rust_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")
    config.addinivalue_line("markers", "slow: large sizes (still bounded to a few seconds of oracle time)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def bsr_mod():
    # One HIP runtime per process: PyTorch bundles its own libamdhip64, so it is loaded
    # before libbsr.so pulls in /opt/rocm's (torch imported after the library has used HIP
    # reports no GPUs; tools/diag/torch_after_graph.py).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    import bsr
    bsr.lib()  # raises if libbsr.so is missing: no fallback
    return bsr


@pytest.fixture(scope="session")
def gpu(bsr_mod):
    if bsr_mod.device_count() < 1:
        pytest.fail("gpu-marked test run without a visible GPU (the engine has no CPU path)")
    return 0
