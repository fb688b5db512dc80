#!/usr/bin/env python3
"""Inverted-index export (walks/inverted_index.h) at configs[1]
size: 3.3 G (wid*L+pos -> next) entries sorted per vertex on the device and
copied out; checks the entry count, that keys ascend within each vertex, and
a sample of entries against the walk matrix.

    python tools/index_probe.py [--scale 22 --samples 117185083]
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
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--samples", type=int, default=117_185_083)
    a = ap.parse_args()
    import dynamicgraphrepresentationlearning_amd as W
    n = 1 << a.scale
    L = 80
    cfg = W.WharfConfig(walks_per_vertex=10, walk_length=L, model=W.DEEPWALK, deterministic=False, seed=0x5EED)
    g = W.WharfMH.from_rmat(n, a.samples, 2 * n, seed=2, config=cfg)
    g.generate_initial_random_walks()
    t0 = time.perf_counter()
    counts, keys, nexts = g.inverted_index()
    dt = time.perf_counter() - t0
    E = len(keys)
    st = g.stats()
    # one entry per stored position: each walk holds 1 + its transitions
    expected = int(st["steps"]) + g.number_of_walks
    off = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
    rng = np.random.default_rng(0)
    bad_order = 0
    for v in rng.choice(np.nonzero(counts)[0], 2000, replace=False):
        k = keys[off[v]:off[v + 1]]
        bad_order += int((np.diff(k.astype(np.int64)) <= 0).sum())
    sample = rng.choice(E, 20000, replace=False)
    wids = keys[sample] // L
    pos = keys[sample] % L
    bad_next = 0
    for wid, p, nx in zip(wids, pos, nexts[sample]):
        walk = g.walk_vertices(int(wid))
        exp = walk[p + 1] if p + 1 < len(walk) else W.SENTINEL
        bad_next += int(exp != nx)
    res = {"n": n, "entries": E, "expected_entries": expected,
           "export_s": round(dt, 2), "entries_per_s": round(E / dt / 1e6, 1), "bad_order": bad_order,
           "bad_next": bad_next}
    print(json.dumps(res), flush=True)
    assert E == expected and bad_order == 0 and bad_next == 0
    g.destroy()


if __name__ == "__main__":
    main()
