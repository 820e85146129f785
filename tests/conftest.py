import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sorting-fhe_amd", "python"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP product library)")
    config.addinivalue_line("markers", "slow: long-running")


def _build(target_dir):
    import subprocess
    subprocess.run(["make", "-C", target_dir, "-j8"], check=True, stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def oracle_lib():
    """CPU oracle build (test infrastructure)."""
    import sfhe
    if not os.path.exists(sfhe.ORACLE_LIB):
        _build(os.path.join(ROOT, "oracle"))
    return sfhe.load("oracle")


@pytest.fixture(scope="session")
def hip_lib():
    """The product library; GPU tests fail loudly if it is missing."""
    import sfhe
    if not os.path.exists(sfhe.PRODUCT_LIB):
        _build(os.path.join(ROOT, "sorting-fhe_amd"))
    return sfhe.load("hip")
