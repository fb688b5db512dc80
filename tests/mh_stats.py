"""Shared helpers for the MH-mode statistical link to the reference.

The reference's MH mode draws from one global RNG (`config::random`,
`config/globals.h:26`), so its corpus is reproducible only serially and only for
its own RNG; our Philox streams give different walks.  What must agree is the
*distribution*: per (model, p, q, sampler init) cell, the fractions of node2vec
transition classes — return (next == prev), triangle (edge prev-next) and
outward — that the frozen-anchor MH sampler produces
(`walks/metropolis_hastings_sampler.h:69-122`, `walks/models/node2vec.h:74-119`).

`tests/golden/make_golden.py mh-matrix` ran the reference over seeds 1..8 per
cell on wiki-graph and committed the mean and sample sd per fraction
(`golden.json` `mh_matrix_reference`).  A build run over the same number of
seeds passes a cell when each fraction's mean lies within
`Z_TOL` standard errors of the reference mean, the standard error of the
difference being sqrt(sd_ref^2/k_ref + sd_ours^2/k_ours) — the tolerance comes
from the reference's own seed-to-seed spread, not from a hand-picked band.
"""
from __future__ import annotations

import numpy as np

SENT = 0xFFFFFFFE
Z_TOL = 4.0
CLASSES = ("return", "triangle", "outward")
SD_FLOOR = 5e-5     # guards cells whose 8 seeds happen to agree to 4 digits


def cells(matrix: dict):
    """(key, model, p, q, init name) of every cell in mh_matrix_reference."""
    out = []
    for key, c in sorted(matrix.items()):
        if not isinstance(c, dict) or "return" not in c:
            continue
        if key == "deepwalk":
            out.append((key, "deepwalk", 1.0, 1.0, "weight"))
        else:
            _, ps, qs, init = key.split("_")
            out.append((key, "node2vec", float(ps[1:]), float(qs[1:]), init))
    return out


def class_fractions(walks: np.ndarray, off: np.ndarray, adj: np.ndarray) -> np.ndarray:
    """[return, triangle, outward] over every transition walk[pos] -> walk[pos+1],
    pos >= 1, classified against walk[pos-1] (the same count as make_golden.py's
    mh_class_fractions)."""
    a = walks[:, :-2].ravel().astype(np.int64)
    c = walks[:, 2:].ravel().astype(np.int64)
    k = c != SENT
    a, c = a[k], c[k]
    ret = a == c
    n = len(off) - 1
    src = np.repeat(np.arange(n, dtype=np.int64), np.diff(off.astype(np.int64)))
    ekeys = src * n + adj.astype(np.int64)
    q = a * n + c
    j = np.minimum(np.searchsorted(ekeys, q), max(len(ekeys) - 1, 0))
    tri = (ekeys[j] == q) & ~ret
    t = len(a)
    r, e = ret.sum() / t, tri.sum() / t
    return np.array([r, e, 1.0 - r - e])


def check_cell(ref_cell: dict, ours: np.ndarray, label: str) -> list[str]:
    """ours: [k_seeds, 3] fractions.  Returns the failures (empty = pass)."""
    k = ours.shape[0]
    mu = ours.mean(0)
    sd = ours.std(0, ddof=1) if k > 1 else np.zeros(3)
    bad = []
    for i, cl in enumerate(CLASSES):
        rm = ref_cell[cl]["mean"]
        rs = max(ref_cell[cl]["sd"], SD_FLOOR)
        kr = len(ref_cell[cl]["per_seed"])
        se = np.sqrt(rs ** 2 / kr + max(sd[i], SD_FLOOR) ** 2 / k)
        z = (mu[i] - rm) / se
        if abs(z) > Z_TOL:
            bad.append(f"{label} {cl}: ours {mu[i]:.5f} ref {rm:.5f} (sd {rs:.5f}) z={z:.1f}")
    return bad


def wiki_compact(off: np.ndarray, adj: np.ndarray):
    """wiki-graph without its isolated vertices, ids renumbered in order: the
    graph of the directed stream cells.  A directed batch edge into an isolated
    vertex makes a sink, where the reference evaluates lrand() % 0
    (utility.h:220, via node2vec.h:97-105) and dies of SIGFPE."""
    return compact_graph(off, adj)


def compact_graph(off: np.ndarray, adj: np.ndarray):
    """A CSR without its isolated vertices, ids renumbered in order."""
    off = off.astype(np.int64)
    deg = np.diff(off)
    keep = np.nonzero(deg > 0)[0]
    remap = np.full(len(deg), -1, dtype=np.int64)
    remap[keep] = np.arange(len(keep))
    src = remap[np.repeat(np.arange(len(deg)), deg)]
    tgt = remap[adj.astype(np.int64)]
    n2 = len(keep)
    off2 = np.zeros(n2 + 1, dtype=np.uint64)
    np.cumsum(np.bincount(src, minlength=n2), out=off2[1:])
    return off2, tgt.astype(np.uint32)


def stream_batch_seeds(off: np.ndarray, adj: np.ndarray, count: int, edges: int):
    """The first `count` batch seeds b = 1, 2, ... whose directed batch
    generate_batch_of_edges(edges, n, b, false, true), inserted and then
    deleted, leaves every vertex with an out-edge (a vertex left without one
    would crash the reference, see wiki_compact)."""
    from oracle import oracle as O
    off = off.astype(np.int64)
    n = len(off) - 1
    deg = np.diff(off)
    src = np.repeat(np.arange(n, dtype=np.int64), deg)
    ekeys = src * n + adj.astype(np.int64)
    out, b = [], 0
    while len(out) < count:
        b += 1
        e = O.generate_batch_of_edges(edges, n, b, False, True).astype(np.int64)
        # after insert + delete of the same batch every batch edge is gone
        present = np.isin(e[:, 0] * n + e[:, 1], ekeys)
        lost = np.bincount(e[present, 0], minlength=n)
        if not ((deg - lost) == 0).any():
            out.append(b)
    return out


def stream_batches(cell: dict, i: int, n: int, gen_batch):
    """The (insert?, pairs) batches of stream cell `cell` for its i-th seed;
    gen_batch = generate_batch_of_edges(edges, n, seed, self_loops, directed)."""
    return [(b["insert"], gen_batch(b["edges"], n, b["seed"], False, b["directed"])) for b in cell["batches"][i]]


def stream_graph(cell: dict, off: np.ndarray, adj: np.ndarray):
    """The cell's base graph: wiki's CSR (off, adj), wiki without isolated
    vertices, or a graph committed beside golden.json (tests/golden/<name>_csr.npz:
    the RMAT hub graph of the rmat_* cells)."""
    if cell["graph"] == "wiki_compact":
        return wiki_compact(off, adj)
    if cell["graph"] == "wiki":
        return off, adj
    import os
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"{cell['graph']}_csr.npz"))
    return z["off"], z["adj"]


def stream_cells(matrix: dict):
    """(key, p, q, init name) of every stream cell."""
    return [(k, c["p"], c["q"], c["init"]) for k, c in sorted(matrix["cells"].items())]
