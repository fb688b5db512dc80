"""The C++ drop-ins over the C ABI: include/wharfmh.hpp running the reference's
own integration-test assertions (tests/wharfmh.cpp, tests/sampler.cpp), and a
restated reference experiment driver (experiments/src/throughput-latency.cpp)
built unchanged against include/compat/wharfmh.h."""
import os
import re
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")


def _exe(name):
    exe = os.path.join(CPP, "build", name)
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", CPP], check=True)
    return exe


@pytest.mark.gpu
def test_cpp_dropin_reference_assertions():
    r = subprocess.run([_exe("wharfmh_test")], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


def test_cpp_dropin_builds():
    """host-only compile of both drop-in headers against the C ABI (no device calls)"""
    r = subprocess.run(["make", "-s", "-C", CPP], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    for exe in ("wharfmh_test", "throughput_latency"):
        assert os.path.exists(os.path.join(CPP, "build", exe))


def test_reference_driver_needs_only_the_include_path():
    """the restated driver includes <wharfmh.h> like a reference driver does and
    names only reference API (dygrl::, config::, types::, utility::, pbbs::)"""
    src = open(os.path.join(CPP, "throughput_latency.cpp")).read()
    includes = re.findall(r"^#include\s*[<\"]([^>\"]+)[>\"]", src, re.M)
    assert includes == ["wharfmh.h"]
    assert "wharf_" not in src.replace("wharfmh.h", "") and "wharf::" not in src
    make = open(os.path.join(CPP, "Makefile")).read()
    assert "-I../../include/compat" in make


def _write_adjacency_graph(path, off, adj):
    with open(path, "w") as f:
        f.write("AdjacencyGraph\n%d\n%d\n" % (len(off) - 1, len(adj)))
        f.write("\n".join(str(int(x)) for x in off[:-1]) + "\n")
        f.write("\n".join(str(int(x)) for x in adj) + "\n")


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["-model", "deepwalk"],
                                  ["-model", "node2vec", "-paramP", "0.5", "-paramQ", "2", "-det", "false"]])
def test_reference_driver_runs(tmp_path, args):
    from oracle import oracle as O
    base = O.generate_batch_of_edges(20000, 1 << 11, 5, False, False)
    off, adj = O.csr_from_edges(1 << 11, base)
    g = tmp_path / "rmat11.adj"
    _write_adjacency_graph(str(g), off, adj)
    r = subprocess.run([_exe("throughput_latency"), "-f", str(g), "-s", "-w", "2", "-l", "20", "-trials", "2",
                        "-maxbatch", "50", *args], capture_output=True, text=True, timeout=300)
    out = r.stdout
    assert r.returncode == 0, out + r.stderr
    assert "Vertices: %d Edges: %d" % (len(off) - 1, len(adj)) in out
    assert out.count("Batch size = ") == 2
    aff = [float(x) for x in re.findall(r"Average number of walks affected = ([0-9.e+-]+)", out)]
    assert len(aff) == 4 and all(a > 0 for a in aff)
    walk_t = [float(x) for x in re.findall(r"Average walk update insert time = ([0-9.e+-]+)", out)]
    assert len(walk_t) == 2 and all(t > 0 for t in walk_t)   # the config.h timers are fed
    m = re.search(r"Deferred walk update: (\d+) rewalk points, (\d+) walks updated \(match\)", out)
    assert m and int(m.group(1)) > 0
    assert "Average time to generate random walks from scratch" in out
