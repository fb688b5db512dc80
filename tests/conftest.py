import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
# the reverse-slot index's carried entries are verified before each write in the test suite
# (k_patch_rev<VERIFY>; a stale entry is repaired and counted in stats()["rev_fallbacks"])
os.environ.setdefault("WHARF_REV_VERIFY", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")


@pytest.fixture(autouse=True)
def _free_gpu_handles(request):
    """After every GPU test, free the device memory of any handle still alive (a failed
    test's handle stays referenced by its traceback and would starve the next tests)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    mod = sys.modules.get("dynamicgraphrepresentationlearning_amd.wharfmh")
    if mod is not None:
        mod.WharfMH.destroy_all()
