"""CPU sanitizer builds: the C oracle under ASan + UBSan and under
TSan with several OpenMP threads (clang + libomp + the Archer tool, so TSan
sees OpenMP's synchronisation; reports inside the uninstrumented libomp are
ignored, reports in our code fail), and the host IO / compat-layer helpers
under ASan + UBSan.  The reference's own races (wharfmh.h:524-536) are what
the oracle's lazily initialised anchor cache must not repeat."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(REPO, "oracle")
CPP = os.path.join(REPO, "tests", "cpp")
LLVM_LIB = "/opt/rocm/llvm/lib"


def _make(path, target):
    r = subprocess.run(["make", "-s", "-C", path, target], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def _run(exe, env=None):
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run([exe], capture_output=True, text=True, env=e, timeout=300)
    return r.returncode, r.stdout + r.stderr


def test_oracle_asan_ubsan():
    _make(ORACLE, "asan")
    rc, out = _run(os.path.join(ORACLE, "build", "sanitize_asan"),
                   {"OMP_NUM_THREADS": "4", "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0"})
    assert rc == 0 and "sanitize OK" in out, out[-4000:]
    assert "runtime error" not in out and "ERROR: AddressSanitizer" not in out


@pytest.mark.skipif(not os.path.exists(os.path.join(LLVM_LIB, "libarcher.so")), reason="no libarcher (ROCm llvm)")
def test_oracle_tsan_openmp():
    _make(ORACLE, "tsan")
    rc, out = _run(os.path.join(ORACLE, "build", "sanitize_tsan"),
                   {"OMP_NUM_THREADS": "4", "OMP_TOOL_LIBRARIES": os.path.join(LLVM_LIB, "libarcher.so"),
                    "TSAN_OPTIONS": "ignore_noninstrumented_modules=1 exitcode=66"})
    assert rc == 0 and "sanitize OK" in out, out[-4000:]
    assert "WARNING: ThreadSanitizer" not in out


def test_host_io_and_compat_asan_ubsan():
    _make(CPP, "sanitize")
    rc, out = _run(os.path.join(CPP, "build", "io_sanitize"), {"ASAN_OPTIONS": "detect_leaks=1"})
    assert rc == 0 and "io sanitize OK" in out, out[-4000:]
