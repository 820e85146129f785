import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sorting-fhe_amd", "python"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP product library)")
    config.addinivalue_line("markers", "slow: long-running CPU-oracle runs at the reference's full rings "
                            "(skipped unless SFHE_SLOW=1 or -m slow; the GPU tests cover the same paths)")


def pytest_collection_modifyitems(config, items):
    """The default CPU suite stays a few minutes long: oracle runs of whole
    k-way / bitonic / bootstrapping sorts at ring 2^17 are opt-in."""
    if os.environ.get("SFHE_SLOW") == "1" or "slow" in (config.getoption("-m") or ""):
        return
    skip = pytest.mark.skip(reason="slow oracle run (SFHE_SLOW=1 or -m slow to run)")
    for item in items:
        if "slow" in item.keywords and "gpu" not in item.keywords:
            item.add_marker(skip)


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
