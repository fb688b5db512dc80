"""The C++ drop-in (include/wharfmh.hpp) running the reference's own
integration-test assertions (tests/wharfmh.cpp, tests/sampler.cpp) on the GPU."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.gpu
def test_cpp_dropin_reference_assertions():
    exe = os.path.join(HERE, "cpp", "build", "wharfmh_test")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(HERE, "cpp")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


def test_cpp_dropin_builds():
    """host-only compile of the drop-in header against the C ABI (no device calls)"""
    r = subprocess.run(["make", "-s", "-C", os.path.join(HERE, "cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert os.path.exists(os.path.join(HERE, "cpp", "build", "wharfmh_test"))
