"""MH mode: the CPU oracle's Philox restatement against the reference's own
seed x sampler-init x (p, q) statistics (`golden.json` `mh_matrix_reference`,
produced by the reference through oracle/_ref/ref_harness, 8 seeds per cell).

The GPU path is bit-exact to the oracle under the same Philox semantics
(test_gpu_parity.py), and tests/test_gpu_parity.py::test_mh_matrix_vs_reference
runs the same matrix through the HIP library; this file pins the oracle itself.
Tolerance: Z_TOL standard errors derived from the reference's seed spread
(tests/mh_stats.py)."""
import json
import os

import numpy as np
import pytest

import mh_stats as S
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")
MATRIX = json.load(open(os.path.join(G, "golden.json")))["mh_matrix_reference"]
INITS = {"random": O.INIT_RANDOM, "burnin": O.INIT_BURNIN, "weight": O.INIT_WEIGHT}


@pytest.fixture(scope="module")
def wiki():
    z = np.load(os.path.join(G, "wiki_csr.npz"))
    return z["off"], z["adj"]


def test_matrix_covers_every_cell():
    keys = [c[0] for c in S.cells(MATRIX)]
    assert len(keys) == 10                      # 3 inits x 3 (p, q) + DeepWalk
    for k in keys:
        assert len(MATRIX[k]["return"]["per_seed"]) == len(MATRIX["seeds"]) == 8


@pytest.mark.parametrize("cell", S.cells(MATRIX), ids=lambda c: c[0])
def test_oracle_mh_cell_vs_reference(wiki, cell):
    key, model, p, q, init = cell
    off, adj = wiki
    ours = []
    for s in MATRIX["seeds"]:
        e = O.Engine(off, adj, wpv=MATRIX["wpv"], L=MATRIX["L"], model=O.NODE2VEC if model == "node2vec" else O.DEEPWALK,
                     p=p, q=q, init=INITS[init], deterministic=False, seed=s)
        e.generate()
        ours.append(S.class_fractions(e.walks(), off, adj))
    bad = S.check_cell(MATRIX[key], np.array(ours), key)
    assert not bad, bad


STREAM = json.load(open(os.path.join(G, "golden.json")))["mh_stream_matrix_reference"]


def test_stream_matrix_covers_directed_and_undirected_cells():
    cells = STREAM["cells"]
    assert len(cells) == 21                       # wiki: 3 (p, q) x 3 inits x {undirected, directed}; RMAT: 3
    assert sum(c["directed"] for c in cells.values()) == 10
    rmat = [k for k, c in cells.items() if c["graph"] == "rmat12c"]
    assert sorted(rmat) == ["rmat_directed_p0.5_q2.0_weight", "rmat_undirected_p0.5_q2.0_random",
                            "rmat_undirected_p0.5_q2.0_weight"]
    for c in cells.values():
        assert len(c["return"]["per_seed"]) == len(STREAM["seeds"]) == len(c["batches"]) == 8


@pytest.mark.parametrize("cell", S.stream_cells(STREAM), ids=lambda c: c[0])
def test_oracle_mh_stream_vs_reference(wiki, cell):
    """After an insert and a delete batch (re-walks, sampler resets of batch
    sources): class fractions of the final corpus on the final graph, against
    the reference's 8 seeds (`mh_stream_matrix_reference`).  Undirected RMAT
    batches on wiki, and the reference driver's directed insert/delete pairs of
    one batch (throughput-latency.cpp:121,126,135) on wiki without isolated
    vertices — the batches where the prev-row anchor reset of DESIGN.md §4
    departs from the reference's keep-first-anchor samplers — and insert/delete
    pairs (undirected: the anchor carry; directed) on an RMAT graph with hubs."""
    key, p, q, init = cell
    c = STREAM["cells"][key]
    off, adj = S.stream_graph(c, *wiki)
    n = len(off) - 1
    ours = []
    for i, s in enumerate(STREAM["seeds"]):
        e = O.Engine(off, adj, wpv=STREAM["wpv"], L=STREAM["L"], model=O.NODE2VEC, p=p, q=q, init=INITS[init],
                     deterministic=False, seed=s)
        e.generate()
        for ins, b in S.stream_batches(c, i, n, O.generate_batch_of_edges):
            e.update(ins, b)
        o2, a2 = e.csr()
        ours.append(S.class_fractions(e.walks(), o2, a2))
    bad = S.check_cell(c, np.array(ours), key)
    assert not bad, bad
