import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

# Environment of a subprocess that injects faults: the testing library (the same
# kernels and host code plus fault injection and test probes) instead of the release
# library, which reads no SPFFT_FAULT_* switch.
TESTING_LIB = os.path.join(REPO, "spfft_amd", "_native", "libspfft_amd_testing.so")
TESTING_ENV = {"SPFFT_AMD_LIBRARY": TESTING_LIB}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not _gpu_available():
        pytest.skip("no GPU")
    import torch
    torch.cuda.set_device(0)
    return torch.device("cuda:0")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    """Build the native library once if it is missing (CPU container or GPU box)."""
    from spfft_amd.ops._lib import library_path
    if not os.path.exists(library_path()):
        from spfft_amd.build import build
        build()
