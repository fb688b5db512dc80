#!/usr/bin/env python3
"""Maximum-size check on one MI355X: the configs[4] (com-friendster-sized) graph.

RMAT scale 26 (67.1 M vertices), 1.8 G undirected samples -> m >= 2^32 CSR
entries (exercises the 64-bit CSR offsets / 40-bit record offsets), built on the
device.  One walk per vertex (the 10-walk corpus of this graph does not fit one
GPU next to the graph; on 8 GPUs each holds 1/8 of it).  Checks: step counts,
every sampled transition is an edge, a window of walks re-computed by the
oracle, one 10k-edge insert + delete with affected walks cross-checked.

    python tools/bigscale.py [--scale 26 --samples 1800000000 --model deepwalk]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--samples", type=int, default=1_800_000_000)
    ap.add_argument("--model", default="deepwalk")
    ap.add_argument("--wpv", type=int, default=1)
    a = ap.parse_args()
    import dynamicgraphrepresentationlearning_amd as W
    from oracle import oracle as O

    n = 1 << a.scale
    node2vec = a.model == "node2vec"
    cfg = W.WharfConfig(walks_per_vertex=a.wpv, walk_length=80, deterministic=False, seed=11,
                        model=W.NODE2VEC if node2vec else W.DEEPWALK, paramP=0.5, paramQ=2.0)
    t0 = time.time()
    # seed 4: odd RMAT multiplier, no sample-period repeats below 2^31 samples
    g = W.WharfMH.from_rmat(n, a.samples, 2 * n, seed=4, config=cfg)
    m = g.number_of_edges()
    t_build = time.time() - t0
    print(f"graph n={n} m={m} (m >= 2^32: {m >= 2**32}) built in {t_build:.1f}s", flush=True)
    g.generate_initial_random_walks()
    g.generate_initial_random_walks()
    st = g.stats()
    off, adj = g.flatten_graph()
    deg = np.diff(off.astype(np.int64))
    active = int((deg > 0).sum()) * a.wpv
    ok_steps = st["steps"] == active * 79
    print(f"generate: {st['last_walk_kernel_ms']:.1f} ms, steps {st['steps']} (expected {active * 79}), "
          f"{st['steps'] / st['last_walk_kernel_ms'] / 1e6:.2f} G steps/s", flush=True)
    # sampled transitions are edges
    rng = np.random.default_rng(1)
    wids = rng.choice(n * a.wpv, 2000, replace=False)
    bad = 0
    for w in wids:
        v = g.walk_vertices(int(w))
        for x, y in zip(v[:-1], v[1:]):
            row = adj[off[x]:off[x + 1]]
            j = np.searchsorted(row, y)
            bad += not (j < len(row) and row[j] == y)
    print(f"sampled transitions not in the graph: {bad}", flush=True)
    # oracle re-computes a window of walks on the same (downloaded) CSR
    w0 = int(off.size // 3)
    ref = None
    same = None
    if not node2vec:
        ref = O.Engine(off, adj, wpv=a.wpv, L=80, deterministic=False, seed=11)
        ref.time_generate_range(w0, w0 + 2048)
        mine = np.stack([np.pad(g.walk_vertices(w), (0, 80 - len(g.walk_vertices(w))), constant_values=W.SENTINEL)
                         for w in range(w0, w0 + 2048)])
        same = bool(np.array_equal(mine, ref.walks()[w0:w0 + 2048]))
        print(f"oracle window [{w0}, {w0 + 2048}) identical: {same}", flush=True)
        del ref
    b = W.generate_batch_of_edges(5000, n, 0, False, False)
    t1 = time.time()
    aff = g.insert_edges_batch(b, remove_dups=True)
    s2 = g.stats()
    print(f"insert 10k edges: {(time.time() - t1) * 1e3:.1f} ms wall, graph {s2['last_graph_update_ms']:.1f} ms, "
          f"re-walk {s2['last_walk_update_ms']:.1f} ms, affected {len(aff)}", flush=True)
    m2 = g.number_of_edges()
    aff2 = g.delete_edges_batch(b, remove_dups=True)
    print(f"delete: affected {len(aff2)}, m {m} -> {m2} -> {g.number_of_edges()}", flush=True)
    res = {"n": n, "m": m, "m_ge_2^32": m >= 2 ** 32, "build_s": round(t_build, 1),
           "gen_ms": round(st["last_walk_kernel_ms"], 2), "steps_ok": ok_steps, "bad_transitions": bad,
           "oracle_window_identical": same, "insert_affected": int(len(aff)),
           "insert_graph_ms": round(s2["last_graph_update_ms"], 2), "insert_rewalk_ms": round(s2["last_walk_update_ms"], 2),
           "m_after_insert": m2, "m_after_delete": g.number_of_edges(), "hbm_bytes_graph": st["hbm_bytes_graph"],
           "hbm_bytes_walks": st["hbm_bytes_walks"]}
    print(json.dumps(res), flush=True)
    assert ok_steps and bad == 0 and same in (True, None) and m2 >= m >= g.number_of_edges()
    g.destroy()


if __name__ == "__main__":
    main()
