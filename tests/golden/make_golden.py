#!/usr/bin/env python3
"""Regenerate the golden vectors under tests/golden/ from the *reference itself*.

Runs oracle/_ref/ref_harness (the reference's header-only WharfMH compiled by
``make -C oracle ref`` from /root/reference, unmodified) and packages its dumps
as small fixtures.  Only runs in the build container (the reference is not on
the GPU box); the committed outputs are data: inputs and the reference's
outputs for them.

    python tests/golden/make_golden.py            # writes tests/golden/*
    python tests/golden/make_golden.py mh-matrix  # only the MH statistics matrices (merged into golden.json)
    python tests/golden/make_golden.py mh-stream  # only the MH stream cells (wiki)
    python tests/golden/make_golden.py mh-stream-rmat  # only the MH stream cells on the RMAT hub graph
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
WIKI = "/root/reference/experiments/data/wiki-graph"   # SNAP edge list shipped with the reference
SENT = 0xFFFFFFFE


def run(args, env_threads=1):
    env = dict(os.environ, NUM_THREADS=str(env_threads))
    r = subprocess.run([HARNESS] + [str(a) for a in args], env=env, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"harness failed ({r.returncode}): {r.stderr[-2000:]}")
    return r.stdout


def snap_to_csr(path):
    """SNAPtoAdj -s equivalent: symmetrise, sort, drop duplicates and self loops
    (reproduces the 2405 V / 23192 E the survey measured for wiki-graph)."""
    e = np.loadtxt(path, dtype=np.int64).reshape(-1, 2)
    s = np.concatenate([e, e[:, ::-1]])
    s = s[s[:, 0] != s[:, 1]]
    u = np.unique(s, axis=0)
    n = int(u.max()) + 1
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(np.bincount(u[:, 0], minlength=n), out=off[1:])
    return off, u[:, 1].astype(np.uint32)


def write_csr(path, off, adj):
    with open(path, "wb") as f:
        np.array([len(off) - 1, len(adj)], dtype=np.uint64).tofile(f)
        off[:-1].astype(np.uint64).tofile(f)
        adj.astype(np.uint32).tofile(f)


def read_walks(d, tag, L):
    return np.fromfile(os.path.join(d, f"walks_{tag}.bin"), dtype=np.uint32).reshape(-1, L)


def read_index(d, tag):
    raw = open(os.path.join(d, f"index_{tag}.bin"), "rb").read()
    n = int(np.frombuffer(raw[:8], dtype=np.uint64)[0])
    cnt = np.frombuffer(raw[8:8 + 8 * n], dtype=np.uint64).copy()
    body = np.frombuffer(raw[8 + 8 * n:], dtype=np.uint32).reshape(-1, 2)
    return cnt, body[:, 0].copy(), body[:, 1].copy()


def read_graph(d, tag):
    raw = open(os.path.join(d, f"graph_{tag}.bin"), "rb").read()
    n = int(np.frombuffer(raw[:8], dtype=np.uint64)[0])
    off = np.frombuffer(raw[8:8 + 8 * (n + 1)], dtype=np.uint64).copy()
    adj = np.frombuffer(raw[8 + 8 * (n + 1):], dtype=np.uint32).copy()
    return off, adj


def rd(d, name, dt=np.uint32):
    return np.fromfile(os.path.join(d, name), dtype=dt)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def mh_class_fractions(walks, off, adj):
    """Per-transition class of walk[pos+1] given (walk[pos-1], walk[pos]), pos >= 1:
    return (== prev), triangle (edge prev-next), outward (otherwise)."""
    ret = tri = out = 0
    adjset = {}
    for v in range(len(off) - 1):
        adjset[v] = set(adj[off[v]:off[v + 1]].tolist())
    for w in walks:
        for pos in range(1, len(w) - 1):
            a, b, c = int(w[pos - 1]), int(w[pos]), int(w[pos + 1])
            if c == SENT:
                break
            if c == a:
                ret += 1
            elif c in adjset[a]:
                tri += 1
            else:
                out += 1
    t = ret + tri + out
    return {"return": ret / t, "triangle": tri / t, "outward": out / t, "transitions": t}


MH_SEEDS = tuple(range(1, 9))
MH_INITS = ("random", "burnin", "weight")
MH_PQ = ((0.5, 2.0), (4.0, 1.0), (2.0, 0.5))


def _mh_cell(args):
    """One reference MH run (serial, config::random.reinit(seed)) on wiki: the
    transition-class fractions of its corpus."""
    tmp, csr, model, p, q, init, seed = args
    d = os.path.join(tmp, f"mhm_{model}_{p}_{q}_{init}_{seed}")
    os.makedirs(d, exist_ok=True)
    run(["out", d, "cfg", 10, 80, model, p, q, init, 0, seed, "graph-csr", csr, "gen"])
    wm = read_walks(d, "0_gen", 80)
    shutil.rmtree(d, ignore_errors=True)
    return wm


def mh_matrix(tmp, woff, wadj):
    """Reference MH-mode statistics over seeds x sampler init x (p, q) on wiki
    (metropolis_hastings_sampler.h:69-122, node2vec.h:74-119): per cell the
    mean and sample sd over the seeds of the return / triangle / outward
    fractions, so a test can derive its tolerance from the reference's own
    seed-to-seed spread.  DeepWalk: the same fractions (uniform walk)."""
    from concurrent.futures import ThreadPoolExecutor
    csr = os.path.join(tmp, "wiki_mh.csr")
    write_csr(csr, woff, wadj)
    jobs = [(tmp, csr, "node2vec", p, q, init, s) for (p, q) in MH_PQ for init in MH_INITS for s in MH_SEEDS]
    jobs += [(tmp, csr, "deepwalk", 1.0, 1.0, "weight", s) for s in MH_SEEDS]
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        walks = list(ex.map(_mh_cell, jobs))
    cells = {}
    for j, wm in zip(jobs, walks):
        _, _, model, p, q, init, s = j
        key = f"{model}_p{p}_q{q}_{init}" if model == "node2vec" else "deepwalk"
        cells.setdefault(key, []).append(mh_class_fractions(wm, woff, wadj))
    out = {"seeds": list(MH_SEEDS), "graph": "wiki (tests/golden/wiki_csr.npz)", "wpv": 10, "L": 80,
           "generator": "ref_harness cfg 10 80 <model> <p> <q> <init> 0 <seed> graph-csr wiki gen, NUM_THREADS=1"}
    for key, fr in cells.items():
        c = {"transitions": fr[0]["transitions"]}
        for k in ("return", "triangle", "outward"):
            v = np.array([f[k] for f in fr])
            c[k] = {"mean": float(v.mean()), "sd": float(v.std(ddof=1)), "per_seed": [float(x) for x in v]}
        out[key] = c
    return out


# MH stream cells (wharfmh.h:439-923 in MH mode: re-walks draw from config::random,
# sampler resets of batch sources at :504,539,652,689).  Per cell: graph, batch
# pattern, (p, q), sampler init.
#   undirected: insert 5000 undirected RMAT samples (batch seed s), then delete
#     3000 (batch seed s + 100), on wiki;
#   directed: the reference driver's own pattern (throughput-latency.cpp:121,126,135):
#     insert a directed batch, then delete the same batch, on wiki without its 42
#     isolated vertices (wiki_compact: a directed edge into an isolated vertex makes
#     a sink, where the reference evaluates lrand() % 0, utility.h:220, and dies of
#     SIGFPE).  Batch seeds whose delete would leave a vertex without out-edges are
#     skipped for the same reason (stream_batch_seeds).
MH_STREAM_UNDIRECTED = ((True, 5000, 0), (False, 3000, 100))   # (insert?, edges, batch-seed offset)
MH_STREAM_DIRECTED_EDGES = 5000


def stream_cell_specs():
    """(key, graph, directed, p, q, init) of every stream cell."""
    out = []
    for (p, q) in MH_PQ:
        for init in MH_INITS:
            out.append((f"undirected_p{p}_q{q}_{init}", "wiki", False, p, q, init))
    for (p, q) in MH_PQ:
        for init in MH_INITS:
            out.append((f"directed_p{p}_q{q}_{init}", "wiki_compact", True, p, q, init))
    return out


def _mh_stream_cell(args):
    """One reference MH run through the cell's two batches: the class fractions
    of the final corpus on the final graph."""
    tmp, csr, key, batches, p, q, init, seed = args
    d = os.path.join(tmp, f"mhs_{key}_{seed}")
    os.makedirs(d, exist_ok=True)
    cmd = ["out", d, "cfg", 10, 80, "node2vec", p, q, init, 0, seed, "graph-csr", csr, "gen"]
    for b in batches:
        cmd += ["ins" if b["insert"] else "del", b["edges"], b["seed"], int(b["directed"])]
    cmd += ["dump-graph"]
    run(cmd)
    wm = read_walks(d, f"{len(batches)}_{'ins' if batches[-1]['insert'] else 'del'}", 80)
    off, adj = read_graph(d, str(len(batches)))
    shutil.rmtree(d, ignore_errors=True)
    return mh_class_fractions(wm, off, adj)


def mh_stream_matrix(tmp, woff, wadj):
    """Reference MH statistics of the corpus after an insert and a delete batch,
    classified against the final graph, per stream cell (stream_cell_specs), 8
    seeds each: pins the re-walk path and the sampler resets of batch sources
    statistically, for undirected batches and for the directed insert/delete
    pairs of the reference's own driver."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.dirname(HERE))   # tests/ (mh_stats)
    sys.path.insert(0, REPO)                    # oracle/ (generate_batch_of_edges, bit-exact with the reference's)
    import mh_stats
    graphs = {"wiki": (woff, wadj), "wiki_compact": mh_stats.wiki_compact(woff, wadj)}
    paths = {}
    for gname, (o, a) in graphs.items():
        paths[gname] = os.path.join(tmp, f"{gname}_mhs.csr")
        write_csr(paths[gname], o, a)
    dseeds = mh_stats.stream_batch_seeds(*graphs["wiki_compact"], len(MH_SEEDS), MH_STREAM_DIRECTED_EDGES)
    jobs, cells = [], {}
    for key, gname, directed, p, q, init in stream_cell_specs():
        per_seed = []
        for i, s in enumerate(MH_SEEDS):
            if directed:
                b = dseeds[i]
                batches = [{"insert": True, "edges": MH_STREAM_DIRECTED_EDGES, "seed": b, "directed": True},
                           {"insert": False, "edges": MH_STREAM_DIRECTED_EDGES, "seed": b, "directed": True}]
            else:
                batches = [{"insert": ins, "edges": e, "seed": s + off, "directed": False}
                           for (ins, e, off) in MH_STREAM_UNDIRECTED]
            per_seed.append(batches)
            jobs.append((tmp, paths[gname], key, batches, p, q, init, s))
        cells[key] = {"graph": gname, "directed": directed, "p": p, "q": q, "init": init, "batches": per_seed}
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = list(ex.map(_mh_stream_cell, jobs))
    fr_by = {}
    for j, fr in zip(jobs, res):
        fr_by.setdefault(j[2], []).append(fr)
    for key, fr in fr_by.items():
        c = cells[key]
        c["transitions"] = [f["transitions"] for f in fr]
        for k in ("return", "triangle", "outward"):
            v = np.array([f[k] for f in fr])
            c[k] = {"mean": float(v.mean()), "sd": float(v.std(ddof=1)), "per_seed": [float(x) for x in v]}
    return {"seeds": list(MH_SEEDS), "wpv": 10, "L": 80, "cells": cells,
            "graphs": {"wiki": "tests/golden/wiki_csr.npz",
                       "wiki_compact": "wiki_csr.npz without its isolated vertices (tests/mh_stats.py wiki_compact)"},
            "generator": "ref_harness cfg 10 80 node2vec <p> <q> <init> 0 <seed> graph-csr <graph> gen "
                         "<ins|del> <edges> <batch seed> <directed> x2 dump-graph, NUM_THREADS=1 (remove_dups=true)"}


# RMAT stream cells (the prev-row reset and the anchor carry act per hub row, and
# wiki has no hubs): an RMAT scale-12 graph (generate_batch_of_edges(40000, 8192, 5, false,
# undirected) on n = 4096: max degree 421 against a mean of 18), without its isolated vertices
# (a directed edge into one makes a sink, see wiki_compact), saved as rmat12c_csr.npz.
#   undirected pairs: insert batch b, delete batch b, insert b + 50, delete b + 50
#     (generate_batch_of_edges(600, n, ., false, undirected), throughput-latency.cpp:126,135), at
#     (p, q) = (0.5, 2) with WEIGHT and with RANDOM inits;
#   directed pair: insert a directed batch, delete it (throughput-latency.cpp:121,126,135), WEIGHT.
RMAT_CELL_GRAPH = ("rmat12c", 40000, 8192, 5, 4096)   # name, samples, vertices_number, seed, n
RMAT_PAIR_EDGES = 600
RMAT_DIRECTED_EDGES = 1000


def rmat_stream_cell_specs():
    return [("rmat_undirected_p0.5_q2.0_weight", False, 0.5, 2.0, "weight"),
            ("rmat_undirected_p0.5_q2.0_random", False, 0.5, 2.0, "random"),
            ("rmat_directed_p0.5_q2.0_weight", True, 0.5, 2.0, "weight")]


def rmat_cell_graph(tmp):
    """The reference's own RMAT base graph (ref_harness graph-rmat + dump-graph),
    isolated vertices removed."""
    sys.path.insert(0, os.path.dirname(HERE))
    import mh_stats
    name, samples, vn, seed, n = RMAT_CELL_GRAPH
    d = os.path.join(tmp, "rmatcell")
    os.makedirs(d, exist_ok=True)
    run(["out", d, "cfg", 1, 2, "deepwalk", 1, 1, "weight", 1, 1, "graph-rmat", samples, vn, seed, n, "gen", "dump-graph"])
    off, adj = read_graph(d, "0")
    return mh_stats.compact_graph(off, adj)


def mh_stream_rmat_cells(tmp):
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, REPO)
    import mh_stats
    off, adj = rmat_cell_graph(tmp)
    np.savez_compressed(os.path.join(HERE, f"{RMAT_CELL_GRAPH[0]}_csr.npz"), off=off, adj=adj)
    csr = os.path.join(tmp, "rmat12c.csr")
    write_csr(csr, off, adj)
    dseeds = mh_stats.stream_batch_seeds(off, adj, len(MH_SEEDS), RMAT_DIRECTED_EDGES)
    jobs, cells = [], {}
    for key, directed, p, q, init in rmat_stream_cell_specs():
        per_seed = []
        for i, s in enumerate(MH_SEEDS):
            if directed:
                b = dseeds[i]
                batches = [{"insert": True, "edges": RMAT_DIRECTED_EDGES, "seed": b, "directed": True},
                           {"insert": False, "edges": RMAT_DIRECTED_EDGES, "seed": b, "directed": True}]
            else:
                batches = [{"insert": ins, "edges": RMAT_PAIR_EDGES, "seed": s + o, "directed": False}
                           for o in (0, 50) for ins in (True, False)]
            per_seed.append(batches)
            jobs.append((tmp, csr, key, batches, p, q, init, s))
        cells[key] = {"graph": RMAT_CELL_GRAPH[0], "directed": directed, "p": p, "q": q, "init": init,
                      "batches": per_seed}
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = list(ex.map(_mh_stream_cell, jobs))
    fr_by = {}
    for j, fr in zip(jobs, res):
        fr_by.setdefault(j[2], []).append(fr)
    for key, fr in fr_by.items():
        c = cells[key]
        c["transitions"] = [f["transitions"] for f in fr]
        for k in ("return", "triangle", "outward"):
            v = np.array([f[k] for f in fr])
            c[k] = {"mean": float(v.mean()), "sd": float(v.std(ddof=1)), "per_seed": [float(x) for x in v]}
    return cells


def main_mh_stream_rmat():
    """Adds the RMAT stream cells to golden.json's mh_stream_matrix_reference."""
    if not os.path.exists(HARNESS):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    tmp = tempfile.mkdtemp(prefix="golden_mhr_")
    try:
        cells = mh_stream_rmat_cells(tmp)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    path = os.path.join(HERE, "golden.json")
    meta = json.load(open(path))
    ms = meta["mh_stream_matrix_reference"]
    ms["cells"].update(cells)
    ms["graphs"][RMAT_CELL_GRAPH[0]] = (f"tests/golden/{RMAT_CELL_GRAPH[0]}_csr.npz: the reference's "
                                        f"generate_batch_of_edges({RMAT_CELL_GRAPH[1]}, {RMAT_CELL_GRAPH[2]}, "
                                        f"{RMAT_CELL_GRAPH[3]}, false, undirected) on n = {RMAT_CELL_GRAPH[4]} "
                                        "(ref_harness graph-rmat), isolated vertices removed")
    with open(path, "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("RMAT stream cells written to", path)


def main_mh_matrix(stream_only=False):
    if not os.path.exists(HARNESS):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    z = np.load(os.path.join(HERE, "wiki_csr.npz"))
    tmp = tempfile.mkdtemp(prefix="golden_mh_")
    try:
        mm = None if stream_only else mh_matrix(tmp, z["off"], z["adj"])
        ms = mh_stream_matrix(tmp, z["off"], z["adj"])
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    path = os.path.join(HERE, "golden.json")
    meta = json.load(open(path))
    if mm is not None:
        meta["mh_matrix_reference"] = mm
    meta["mh_stream_matrix_reference"] = ms
    with open(path, "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("mh_matrix_reference written to", path)


def main():
    if not os.path.exists(HARNESS):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    tmp = tempfile.mkdtemp(prefix="golden_")
    meta = {"generator": "tests/golden/make_golden.py via oracle/_ref/ref_harness (reference headers, unmodified)"}
    try:
        # ---- 1. known answers: RNG, hashes, Szudzik, RMAT batches ---------------
        batches = [(8, 64, 0, 1), (100, 1024, 3, 1), (500, 2048, 5, 0), (5000, 2405, 0, 1), (2000, 4096, 11, 0)]
        args = ["out", tmp, "kat"]
        for b in batches:
            args += ["batch"] + list(b)
        run(args)
        shutil.copy(os.path.join(tmp, "kat.txt"), os.path.join(HERE, "kat.txt"))
        bz = {}
        for (M, V, s, d) in batches:
            bz[f"b_{M}_{V}_{s}_{d}"] = rd(tmp, f"batch_gen_{M}_{V}_{s}_{d}.bin").reshape(-1, 2)
        np.savez_compressed(os.path.join(HERE, "rmat_batches.npz"), **bz)

        # ---- 2. six-vertex graph (tests/sampler.cpp:24-35) -------------------------
        six = {0: [1, 2], 1: [0, 2, 3], 2: [0, 1, 3, 4, 5], 3: [1, 2, 5], 4: [2, 5], 5: [2, 3, 4]}
        off = np.zeros(7, dtype=np.uint64)
        adj = []
        for v in range(6):
            adj += six[v]
            off[v + 1] = len(adj)
        adj = np.array(adj, dtype=np.uint32)
        write_csr(os.path.join(tmp, "six.csr"), off, adj)
        d6 = os.path.join(tmp, "six")
        os.makedirs(d6)
        run(["out", d6, "cfg", 2, 5, "deepwalk", 4, 1, "weight", 1, 7, "graph-csr", os.path.join(tmp, "six.csr"),
             "gen", "dump-index", "walkstr", 0, "walkstr", 11])
        d6n = os.path.join(tmp, "six_n2v")
        os.makedirs(d6n)
        run(["out", d6n, "cfg", 2, 5, "node2vec", 0.5, 2, "weight", 1, 7, "graph-csr", os.path.join(tmp, "six.csr"), "gen"])
        cnt, keys, nexts = read_index(d6, "0")
        np.savez_compressed(os.path.join(HERE, "six.npz"), off=off, adj=adj, walks=read_walks(d6, "0_gen", 5),
                            walks_node2vec=read_walks(d6n, "0_gen", 5), index_counts=cnt, index_keys=keys,
                            index_nexts=nexts)
        meta["six_walkstr"] = {"0": open(os.path.join(d6, "walkstr_0.txt")).read(),
                               "11": open(os.path.join(d6, "walkstr_11.txt")).read()}

        # ---- 3. RMAT scale-10 streaming case (wpv=2, L=20) --------------------------
        # base: generate_batch_of_edges(12800, 2048, seed 1, undirected) on n = 1024
        for model in ("deepwalk", "node2vec"):
            dr = os.path.join(tmp, f"rmat10_{model}")
            os.makedirs(dr)
            out = run(["out", dr, "cfg", 2, 20, model, 0.5, 2, "weight", 1, 7, "graph-rmat", 12800, 2048, 1, 1024,
                       "gen", "dump-index", "dump-graph",
                       "ins", 500, 5, 0, "dump-index", "dump-graph",
                       "del", 500, 5, 0, "dump-index", "dump-graph",
                       "ins", 300, 9, 0, "dump-graph",
                       "del", 200, 2, 0, "dump-graph"])
            meta[f"rmat10_{model}_log"] = out
        dr = os.path.join(tmp, "rmat10_deepwalk")
        z = {}
        for tag in ("0", "1", "2", "3", "4"):
            o, a = read_graph(dr, tag)
            z[f"off_{tag}"], z[f"adj_{tag}"] = o, a
        for tag, name in (("0_gen", "gen"), ("1_ins", "ins1"), ("2_del", "del2"), ("3_ins", "ins3"), ("4_del", "del4")):
            z[f"walks_{name}"] = read_walks(dr, tag, 20)
        for tag in ("1_ins", "2_del", "3_ins", "4_del"):
            z[f"batch_{tag}"] = rd(dr, f"batch_{tag}_in.bin").reshape(-1, 2)
            z[f"affected_{tag}"] = rd(dr, f"affected_{tag}.bin")
        for tag in ("0", "1", "2"):
            c, k, nx = read_index(dr, tag)
            z[f"index_counts_{tag}"], z[f"index_keys_{tag}"], z[f"index_nexts_{tag}"] = c, k, nx
        drn = os.path.join(tmp, "rmat10_node2vec")
        for tag, name in (("0_gen", "gen"), ("1_ins", "ins1"), ("2_del", "del2")):
            z[f"n2v_walks_{name}"] = read_walks(drn, tag, 20)
        np.savez_compressed(os.path.join(HERE, "rmat10.npz"), **z)

        # ---- 4. directed batches (throughput-latency.cpp:121 pattern) ----------------
        dd = os.path.join(tmp, "rmat10_dir")
        os.makedirs(dd)
        try:
            out = run(["out", dd, "cfg", 2, 20, "deepwalk", 4, 1, "weight", 1, 7, "graph-rmat", 12800, 2048, 1, 1024,
                       "gen", "ins", 50, 0, 1, "del", 50, 0, 1])
            zd = {"walks_gen": read_walks(dd, "0_gen", 20), "walks_ins": read_walks(dd, "1_ins", 20),
                  "walks_del": read_walks(dd, "2_del", 20),
                  "batch_ins": rd(dd, "batch_1_ins_in.bin").reshape(-1, 2),
                  "affected_ins": rd(dd, "affected_1_ins.bin"), "affected_del": rd(dd, "affected_2_del.bin")}
            np.savez_compressed(os.path.join(HERE, "rmat10_directed.npz"), **zd)
            meta["rmat10_directed_log"] = out
        except RuntimeError as ex:
            meta["rmat10_directed_error"] = str(ex)

        # ---- 5. wiki-graph (experiments/data/wiki-graph, SNAPtoAdj -s) ------------------
        woff, wadj = snap_to_csr(WIKI)
        np.savez_compressed(os.path.join(HERE, "wiki_csr.npz"), off=woff, adj=wadj)
        write_csr(os.path.join(tmp, "wiki.csr"), woff, wadj)
        dw = os.path.join(tmp, "wiki")
        os.makedirs(dw)
        out = run(["out", dw, "cfg", 10, 80, "deepwalk", 4, 1, "weight", 1, 7, "graph-csr", os.path.join(tmp, "wiki.csr"),
                   "gen", "ins", 5000, 0, 0, "del", 5000, 0, 0, "walkstr", 12345])  # serial: the rewalk-point min-update races at >1 thread (wharfmh.h:524-536)
        w, wz = {}, {}
        for tag in ("0_gen", "1_ins", "2_del"):
            wm = read_walks(dw, tag, 80)
            w[tag] = {"sha256": sha(wm)}
            wz[f"first64_{tag}"] = wm[:64]
        for tag in ("1_ins", "2_del"):
            a = rd(dw, f"affected_{tag}.bin")
            w[f"affected_{tag}"] = {"count": int(len(a)), "sha256": sha(a)}
            wz[f"batch_{tag}"] = rd(dw, f"batch_{tag}_in.bin").reshape(-1, 2)
        np.savez_compressed(os.path.join(HERE, "wiki_golden.npz"), **wz)
        w["walkstr_12345"] = open(os.path.join(dw, "walkstr_12345.txt")).read()
        w["log"] = out
        meta["wiki"] = w

        # ---- 6. MH-mode statistics (reference, serial, config::random.reinit(42)) -------
        mh = {}
        for model, p, q in (("node2vec", 0.5, 2.0), ("deepwalk", 1.0, 1.0)):
            dm = os.path.join(tmp, f"mh_{model}")
            os.makedirs(dm)
            run(["out", dm, "cfg", 10, 80, model, p, q, "weight", 0, 42, "graph-csr", os.path.join(tmp, "wiki.csr"), "gen"])
            wm = read_walks(dm, "0_gen", 80)
            st = mh_class_fractions(wm, woff, wadj)
            # DeepWalk: uniform-neighbour check, per-(cur) next-vertex chi-square
            if model == "deepwalk":
                cnt = {}
                for row in wm:
                    for a, b in zip(row[:-1], row[1:]):
                        if b == SENT:
                            break
                        cnt[(int(a), int(b))] = cnt.get((int(a), int(b)), 0) + 1
                chi, dof = 0.0, 0
                for v in range(len(woff) - 1):
                    d = int(woff[v + 1] - woff[v])
                    if d < 2:
                        continue
                    nb = wadj[woff[v]:woff[v + 1]]
                    obs = np.array([cnt.get((v, int(x)), 0) for x in nb], dtype=np.float64)
                    tot = obs.sum()
                    if tot < 5 * d:
                        continue
                    exp = tot / d
                    chi += float(((obs - exp) ** 2 / exp).sum())
                    dof += d - 1
                st["chi2"] = chi
                st["dof"] = dof
            mh[f"{model}_p{p}_q{q}"] = st
        meta["mh_stats_reference"] = mh
        meta["mh_matrix_reference"] = mh_matrix(tmp, woff, wadj)
        meta["mh_stream_matrix_reference"] = mh_stream_matrix(tmp, woff, wadj)
        meta["mh_stream_matrix_reference"]["cells"].update(mh_stream_rmat_cells(tmp))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    if sys.argv[1:] == ["mh-matrix"]:
        sys.exit(main_mh_matrix())
    if sys.argv[1:] == ["mh-stream"]:
        sys.exit(main_mh_matrix(stream_only=True))
    if sys.argv[1:] == ["mh-stream-rmat"]:
        sys.exit(main_mh_stream_rmat())
    sys.exit(main())
