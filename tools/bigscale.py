#!/usr/bin/env python3
"""Full-size runs of the large configs on ONE MI355X (288 GB HBM).

configs[4] (com-friendster-sized, default): RMAT scale 26 (67.1 M vertices),
1.8 G undirected samples -> 3.6 G CSR entries, built on the device.  One walk
per vertex with node2vec (the anchors and the edge hash take the room of the
other nine), ten with DeepWalk only at scale 25.

configs[3] (twitter-sized): --scale 25 --samples 1200000000 --wpv 10
--batches 50: 335 M walks (107 GB walk matrix, 26.5 G stored positions)
next to a 2.4 G-entry CSR, initial generation + 50 insert batches.

Checks: step counts, every sampled transition is an edge, a window of walks
re-computed by the oracle (DeepWalk), the walk ids of insert batches, a
delete of the last batch restoring m.  --mixed alternates insert b / delete b
(throughput-latency.cpp:126,135).

    python tools/bigscale.py [--scale 26 --samples 1800000000 --model deepwalk --wpv 1 --batches 1]
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
    ap.add_argument("--batches", type=int, default=1)
    ap.add_argument("--mixed", action="store_true", help="insert batch b, then delete it")
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("--det", action="store_true", help="deterministic mode (DeepWalk)")
    ap.add_argument("--shard", type=int, default=1,
                    help="keep only rank 0's walk shard of an N-way split (the per-GPU work of an N-GPU run; "
                         "the CSR stays whole, as on every rank)")
    ap.add_argument("--shard-index", type=int, default=0, help="which rank's shard of the --shard split to keep")
    a = ap.parse_args()
    import torch
    import dynamicgraphrepresentationlearning_amd as W
    from oracle import oracle as O

    n = 1 << a.scale
    node2vec = a.model == "node2vec"
    cfg = W.WharfConfig(walks_per_vertex=a.wpv, walk_length=80, deterministic=a.det, seed=11,
                        model=W.NODE2VEC if node2vec else W.DEEPWALK, paramP=0.5, paramQ=2.0)
    t0 = time.time()
    # seed 4: odd RMAT multiplier, no sample-period repeats below 2^31 samples
    g = W.WharfMH.from_rmat(n, a.samples, 2 * n, seed=4, config=cfg)
    m = g.number_of_edges()
    t_build = time.time() - t0
    print(f"graph n={n} m={m} built in {t_build:.1f}s", flush=True)
    off, adj = g.flatten_graph()
    deg = np.diff(off.astype(np.int64))
    if a.shard > 1:
        from dynamicgraphrepresentationlearning_amd.distributed import balanced_shards
        lo, hi = balanced_shards(deg, a.shard)[a.shard_index]
        g.set_shard(lo, hi)
        print(f"shard {a.shard_index} of {a.shard}: start vertices [{lo}, {hi}), {g.number_of_walks} walks", flush=True)
    g.generate_initial_random_walks()
    first_ms, first_inits = g.stats()["last_walk_kernel_ms"], g.stats()["last_anchor_inits"]
    g.generate_initial_random_walks()
    st = g.stats()
    lo, hi = g.shard()[:2]
    active = int((deg[lo:hi] > 0).sum()) * a.wpv
    ok_steps = st["steps"] == active * 79
    gen_rate = st["steps"] / st["last_walk_kernel_ms"] / 1e6
    print(f"generate: {st['last_walk_kernel_ms']:.1f} ms, steps {st['steps']} (expected {active * 79}), "
          f"{gen_rate:.2f} G steps/s, accepts {st['accepts']} (first generation {first_ms:.1f} ms, "
          f"anchor inits {first_inits})", flush=True)
    mem = g.memory_footprint(verbose=False)
    free, total = torch.cuda.mem_get_info(0)
    print(f"device bytes: {json.dumps(mem)}; hipMemGetInfo free {free / 2**30:.1f} of {total / 2**30:.1f} GiB",
          flush=True)
    # sampled transitions are edges
    rng = np.random.default_rng(1)
    wids = rng.choice(g.walk_ids(), 2000, replace=False)   # global ids of the owned walks
    bad = 0
    for w in wids:
        v = g.walk_vertices(int(w))
        for x, y in zip(v[:-1], v[1:]):
            row = adj[off[x]:off[x + 1]]
            j = np.searchsorted(row, y)
            bad += not (j < len(row) and row[j] == y)
    print(f"sampled transitions not in the graph: {bad}", flush=True)
    # oracle re-computes a window of walks on the same (downloaded) CSR
    same = None
    if not node2vec and not a.no_oracle and a.shard == 1:
        w0 = int(n // 3)
        ref = O.Engine(off, adj, wpv=a.wpv, L=80, deterministic=a.det, seed=11)
        ref.time_generate_range(w0, w0 + 2048)
        mine = np.stack([np.pad(g.walk_vertices(w), (0, 80 - len(g.walk_vertices(w))), constant_values=W.SENTINEL)
                         for w in range(w0, w0 + 2048)])
        same = bool(np.array_equal(mine, ref.walks()[w0:w0 + 2048]))
        print(f"oracle window [{w0}, {w0 + 2048}) identical: {same}", flush=True)
        del ref
    del off, adj, deg
    out = torch.empty(max(g.number_of_walks, 1), dtype=torch.int32, device="cuda:0")
    lat, gms, wms, affs, steps, inits, passes, ies = [], [], [], [], [], [], [], []
    for b in range(a.batches):
        batch = W.generate_batch_of_edges(5000, n, b, False, False)
        for ins in ((True, False) if a.mixed else (True,)):
            t1 = time.perf_counter()
            aff = (g.insert_edges_batch if ins else g.delete_edges_batch)(batch, remove_dups=True, out=out)
            lat.append((time.perf_counter() - t1) * 1e3)
            s2 = g.stats()
            gms.append(s2["last_graph_update_ms"])
            wms.append(s2["last_walk_update_ms"])
            affs.append(len(aff))
            steps.append(s2["steps"])
            inits.append(s2["last_anchor_inits"])
            passes.append(s2["last_rewalk_passes"])
            ies.append(s2["last_csr_move_ms"])
        print(f"batch {b}: {lat[-1]:.1f} ms (graph {gms[-1]:.1f} incl. in-edge scan {ies[-1]:.2f}, re-walk {wms[-1]:.1f}), "
              f"affected {affs[-1]}, "
              f"steps {steps[-1]}, anchor inits {inits[-1]}, passes {passes[-1]}, m {g.number_of_edges()}", flush=True)
        if b == 0:
            m1 = g.memory_footprint(verbose=False)
            free, _ = torch.cuda.mem_get_info(0)
            print(f"after batch 0: update buffers {m1['update_buffers_bytes'] / 2**30:.1f} GiB, scratch "
                  f"{m1['scratch_bytes'] / 2**30:.1f} GiB, free {free / 2**30:.1f} GiB", flush=True)
    m2 = g.number_of_edges()
    pst = g.stats()
    print(f"slot pool: {pst['pool_slots']} of {pst['pool_capacity']} slots handed out (m {m2}), "
          f"repacks {pst['repacks']}, in-edge scan {pst['last_csr_move_ms']:.2f} ms", flush=True)
    last = W.generate_batch_of_edges(5000, n, a.batches - 1, False, False)
    g.delete_edges_batch(last, remove_dups=True, out=out)
    m3 = g.number_of_edges()
    res = {"config": f"RMAT scale {a.scale}, {a.samples} undirected samples (seed 4), {a.model} {'deterministic' if a.det else 'MH'}, wpv {a.wpv}, "
                     f"L 80, {a.batches} {'insert+delete' if a.mixed else 'insert'} batches of "
                     "generate_batch_of_edges(5000, n, b, false, false)",
           "n": n, "m": m, "walks": g.number_of_walks, "shard_of": a.shard, "shard_index": a.shard_index, "build_s": round(t_build, 1),
           "gen_ms": round(st["last_walk_kernel_ms"], 2), "gen_Gsteps_per_s": round(gen_rate, 2),
           "first_gen_ms": round(first_ms, 2), "first_gen_anchor_inits": first_inits,
           "steps_ok": ok_steps, "bad_transitions": bad, "oracle_window_identical": same,
           "batch_median_ms": round(float(np.median(lat)), 2), "batch_p90_ms": round(float(np.percentile(lat, 90)), 2),
           "graph_update_median_ms": round(float(np.median(gms)), 2),
           "walk_update_median_ms": round(float(np.median(wms)), 2),
           "mean_affected": int(np.mean(affs)),
           "rewalk_Gsteps_per_s": round(float(np.sum(steps) / np.sum(wms) / 1e6), 2),
           "mean_rewalk_steps": int(np.mean(steps)), "mean_anchor_inits": int(np.mean(inits)),
           "rewalk_passes": passes,
           "m_after_batches": m2, "pool_slots": pst["pool_slots"], "pool_capacity": pst["pool_capacity"],
           "repacks": pst["repacks"], "m_after_delete_last": m3, "device_bytes_total": mem["total_bytes"]}
    print(json.dumps(res), flush=True)
    assert ok_steps and bad == 0 and same in (True, None) and m3 <= m2
    g.destroy()


if __name__ == "__main__":
    main()
