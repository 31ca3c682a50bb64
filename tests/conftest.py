"""pytest setup: import paths, the `gpu` marker, and GPU detection without torch."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bipartite-link-prediction_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def _has_gpu():
    try:
        import blp

        return blp.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    """Device 0 is present; GPU tests fail loudly if the engine cannot load."""
    import blp

    blp.lib()  # raises BLPUnavailable if libblp.so is missing -- never skip silently
    if not _has_gpu():
        pytest.skip("no GPU visible")
    return 0
