import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    # build the in-tree native libraries if they are missing (no-op when present)
    need = [os.path.join(ROOT, "lpcnet_amd", "liblpcnet_mi355x.so"), os.path.join(ROOT, "oracle", "liblpcnet_oracle.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.run(["make", "-C", ROOT, "-j4"], check=True, capture_output=True)


def gpu_available() -> bool:
    import lpcnet_amd
    return lpcnet_amd.device_count() > 0


@pytest.fixture(scope="session")
def require_gpu():
    if not gpu_available():
        pytest.fail("no HIP device visible: -m gpu tests need an MI355X")
