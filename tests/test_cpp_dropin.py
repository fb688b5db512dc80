"""The C++ drop-ins over the C ABI: include/wharfmh.hpp running the reference's
own integration-test assertions (tests/wharfmh.cpp, tests/sampler.cpp), and the
reference's own experiment drivers (experiments/src/*.cpp) compiled where they
lie against include/compat/wharfmh.h.  (Round 4 removed the restated
throughput-latency driver of tests/cpp/: the reference's own file builds in
place and runs below.)"""
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
    """host-only compile of the C++ drop-in header against the C ABI (no device calls)"""
    r = subprocess.run(["make", "-s", "-C", CPP], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert os.path.exists(os.path.join(CPP, "build", "wharfmh_test"))


def _write_adjacency_graph(path, off, adj):
    with open(path, "w") as f:
        f.write("AdjacencyGraph\n%d\n%d\n" % (len(off) - 1, len(adj)))
        f.write("\n".join(str(int(x)) for x in off[:-1]) + "\n")
        f.write("\n".join(str(int(x)) for x in adj) + "\n")


# ---------------------------------------------------------------------------
# The reference's OWN experiment drivers (experiments/src/*.cpp), compiled where
# they lie against include/compat/wharfmh.h (oracle/Makefile `drivers`; the
# binaries live in the git-ignored oracle/_ref/drivers/ and travel to the GPU
# box with the tree, the reference itself does not).
# ---------------------------------------------------------------------------
REFERENCE = "/root/reference"
REF_DRIVERS = ("throughput-latency", "memory-throughput-latency", "memory-footprint", "vertex-classification")
DRV = os.path.join(os.path.dirname(HERE), "oracle", "_ref", "drivers")


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="the reference is only present in the build container")
def test_reference_drivers_build_in_place():
    """`-I include/compat -I include` in place of the reference's include dirs is
    the whole change: every driver compiles from the reference's own file and
    links libwharf_gpu.so (vertex-classification.cpp needs the <fstream> /
    <sstream> / namespace-std the reference's headers pull in)."""
    r = subprocess.run(["make", "-s", "-B", "-C", os.path.join(os.path.dirname(HERE), "oracle"), "drivers"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    for d in REF_DRIVERS:
        exe = os.path.join(DRV, d)
        assert os.access(exe, os.X_OK), d
        ldd = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
        assert "libwharf_gpu.so" in ldd and "not found" not in ldd.split("libwharf_gpu.so")[1].splitlines()[0], ldd


def _ref_driver(name):
    exe = os.path.join(DRV, name)
    if not os.access(exe, os.X_OK):
        pytest.skip(f"{exe} not built (make -C oracle drivers needs the reference)")
    return exe


def _rmat_graph(tmp_path, scale=11, samples=20000, seed=5):
    from oracle import oracle as O
    n = 1 << scale
    base = O.generate_batch_of_edges(samples, 2 * n, seed, False, False)
    off, adj = O.csr_from_edges(n, base)
    g = tmp_path / "rmat.adj"
    _write_adjacency_graph(str(g), off, adj)
    return str(g), off, adj


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["throughput-latency", "memory-throughput-latency"])
@pytest.mark.parametrize("args", [["-model", "deepwalk"],
                                  ["-model", "node2vec", "-paramP", "0.5", "-paramQ", "2", "-det", "false"]])
def test_reference_throughput_drivers_run(tmp_path, name, args):
    """The reference's throughput/latency drivers, unchanged, over the GPU engine:
    directed RMAT batches of 5 / 50 / 500 edges inserted and deleted
    (throughput-latency.cpp:87-150), the config.h update timers fed, walks
    regenerated from scratch (:178-191)."""
    g, off, adj = _rmat_graph(tmp_path)
    r = subprocess.run([_ref_driver(name), "-f", g, "-s", "-w", "2", "-l", "20", "-trials", "2", *args],
                       capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    out = r.stdout
    assert r.returncode == 0, out + r.stderr
    assert "Vertices: %d Edges: %d" % (len(off) - 1, len(adj)) in out
    sizes = [2 * b for b in ((5, 50, 500) if name == "throughput-latency" else (500,))]
    assert [int(x) for x in re.findall(r"Batch size = (\d+)", out)] == sizes
    aff = [float(x) for x in re.findall(r"Average number of walks affected = ([0-9.e+-]+)", out)]
    assert len(aff) == 2 * len(sizes) and all(a > 0 for a in aff)
    walk_t = [float(x) for x in re.findall(r"Average walk update insert time = ([0-9.e+-]+)", out)]
    assert len(walk_t) == len(sizes) and all(t > 0 for t in walk_t)     # fed by the device timers
    assert "Average time to generate random walks from scratch" in out


@pytest.mark.gpu
def test_reference_memory_footprint_driver_runs(tmp_path):
    g, off, adj = _rmat_graph(tmp_path)
    r = subprocess.run([_ref_driver("memory-footprint"), "-f", g, "-s", "-w", "2", "-l", "20"],
                       capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Vertices: %d Edges: %d" % (len(off) - 1, len(adj)) in r.stdout


@pytest.mark.gpu
def test_reference_vertex_classification_driver_corpus(tmp_path):
    """vertex-classification.cpp, the only caller of the corpus readout: it builds
    WharfMH(n, m) over isolated vertices, streams the edge file in partitions of
    -eps (both directions, :5-38), re-walks incrementally, then regenerates from
    scratch after each partition (static learning, :300-350) and writes every
    walk with WharfMH::walk(i) to walks.txt (:142-150,309-312).  The yskip / perl /
    python steps it shells out to are outside the walk path (logged, not run).
    Deterministic mode (the default): the final walks.txt equals the oracle's
    corpus of the final graph, line for line."""
    from oracle import oracle as O
    n = 600
    e = O.generate_batch_of_edges(3000, 1024, 3, False, True)
    e = e[(e[:, 0] < n) & (e[:, 1] < n) & (e[:, 0] != e[:, 1])]
    stream = tmp_path / "stream"
    with open(stream, "w") as f:
        f.write("".join(f"{u} {v}\n" for u, v in e))
    _write_adjacency_graph(str(tmp_path / "stream.adj"), np.zeros(n + 1, np.uint64), np.zeros(0, np.uint32))
    r = subprocess.run([_ref_driver("vertex-classification"), "-f", str(stream), "-w", "2", "-l", "10",
                        "-eps", "400"], capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "[downstream step not run]" in r.stderr and "yskip" in r.stderr
    assert r.stdout.count("Total") >= 2
    # final graph: every stream edge, both directions (create_edge_stream), as a set
    both = np.unique(np.concatenate([e, e[:, ::-1]]), axis=0)
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(np.bincount(both[:, 0], minlength=n), out=off[1:])
    ref = O.Engine(off, both[:, 1].astype(np.uint32), wpv=2, L=10)
    ref.generate()
    want = "".join(" ".join(str(int(x)) for x in row if x != O.SENT) + " \n" for row in ref.walks())
    assert open(tmp_path / "walks.txt").read() == want
