"""CPU-only checks of the drop-in boundary: the HIP library loads, exports every
symbol include/wharf_gpu.h declares, and the Python mirror's struct layouts
match the C header.  No device calls."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "wharf_gpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(wharf_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_walk_path():
    names = declared_functions()
    for must in ("wharf_create", "wharf_generate", "wharf_insert_edges", "wharf_delete_edges", "wharf_walk",
                 "wharf_export_index", "wharf_destroy", "wharf_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from dynamicgraphrepresentationlearning_amd import _lib as L
    lib = C.CDLL(L.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes table binds exactly the declared set
    assert sorted(L.SIGNATURES) == declared_functions()


def test_library_is_gfx950_code():
    from dynamicgraphrepresentationlearning_amd import _lib as L
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", L.LIB_PATH], capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("llvm-readelf unavailable")
    assert ".hip_fatbin" in out.stdout
    blob = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_struct_layout_matches_header():
    from dynamicgraphrepresentationlearning_amd import _lib as L
    prog = r"""
#include <stdio.h>
#include <stddef.h>
#include "wharf_gpu.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu\n", sizeof(wharf_config), offsetof(wharf_config, seed), offsetof(wharf_config, shard_hi),
         sizeof(wharf_stats), offsetof(wharf_stats, last_walk_kernel_ms));
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(prog)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), c, "-o", exe], check=True)
        got = [int(x) for x in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    exp = [C.sizeof(L.wharf_config), L.wharf_config.seed.offset, L.wharf_config.shard_hi.offset,
           C.sizeof(L.wharf_stats), L.wharf_stats.last_walk_kernel_ms.offset]
    assert got == exp


def test_config_defaults_mirror_reference_globals():
    from dynamicgraphrepresentationlearning_amd import _lib as L
    from dynamicgraphrepresentationlearning_amd import WharfConfig
    c = L.wharf_config()
    L.lib.wharf_config_default(C.byref(c))
    py = WharfConfig().to_c()
    for f, _ in L.wharf_config._fields_:
        assert getattr(c, f) == getattr(py, f), f
    # config/globals.h:7-29
    assert (c.walks_per_vertex, c.walk_length, c.sampler_init, c.deterministic) == (10, 80, 2, 1)
    assert (c.paramP, c.paramQ) == (4.0, 1.0)
    assert c.model == L.WHARF_NODE2VEC            # config::random_walk_model = NODE2VEC (globals.h:13)


def test_errors_without_a_device_are_reported_not_crashed():
    from dynamicgraphrepresentationlearning_amd import _lib as L
    h = C.c_void_p()
    cfg = L.wharf_config()
    L.lib.wharf_config_default(C.byref(cfg))
    cfg.walk_length = 1000   # invalid: rejected before any device call
    off = np.zeros(4, np.uint64)
    rc = L.lib.wharf_create(C.byref(cfg), 4, 0, off.ctypes.data_as(C.c_void_p), None, 0, C.byref(h))
    assert rc == -1 and "walk_length" in L.last_error()


def test_balanced_shards():
    from dynamicgraphrepresentationlearning_amd.distributed import balanced_shards
    deg = np.array([0, 3, 0, 0, 1, 1, 2, 0, 5, 1], dtype=np.int64)
    sh = balanced_shards(deg, 3)
    assert sh[0][0] == 0 and sh[-1][1] == len(deg)
    assert all(a[1] == b[0] for a, b in zip(sh, sh[1:]))
    act = [int((deg[a:b] > 0).sum()) for a, b in sh]
    assert max(act) - min(act) <= 1 and sum(act) == 6
