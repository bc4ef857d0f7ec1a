import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "gpu-gmres_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

FIXTURES = os.path.join(REPO, "tests", "golden", "fixtures")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")
    config.addinivalue_line("markers", "slow: full-size (1M-row) checks")


def fixture_path(name):
    return os.path.join(FIXTURES, name)


@pytest.fixture(scope="session")
def ggmres_lib():
    """The built C-ABI library (built on demand, never faked)."""
    import ggmres
    if not os.path.exists(ggmres.LIB_PATH):
        import subprocess
        subprocess.check_call(["make", "-s", "-j8", "-C", PKG])
    return ggmres.lib()
