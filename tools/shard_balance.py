#!/usr/bin/env python3
"""Per-rank balance of an 8-GPU job, measured on one GPU: every rank's walk
shard (distributed.balanced_shards) run in turn over the same graph, each on a
fresh handle (the same graph and batches every time): first and warm
generation, then `--batches` update batches generate_batch_of_edges(5000, n, b,
false, undirected) (inserted; --mixed: each inserted, then deleted).  Prints
one JSON line per shard and a summary with max / min of the batch medians.

    python tools/shard_balance.py [--scale 25 --samples 1200000000 --wpv 10 --parts 8 --batches 3]
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
    ap.add_argument("--scale", type=int, default=25)
    ap.add_argument("--samples", type=int, default=1_200_000_000)
    ap.add_argument("--model", default="deepwalk")
    ap.add_argument("--wpv", type=int, default=10)
    ap.add_argument("--p", type=float, default=0.5)
    ap.add_argument("--q", type=float, default=2.0)
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--batches", type=int, default=3)
    ap.add_argument("--mixed", action="store_true")
    ap.add_argument("--shards", type=int, nargs="*", default=None, help="shard indices (default: all)")
    ap.add_argument("--blocks", type=int, default=0,
                    help="block shards of 2^BLOCKS vertices dealt round-robin (0: contiguous balanced ranges)")
    a = ap.parse_args()
    import torch
    import dynamicgraphrepresentationlearning_amd as W
    from dynamicgraphrepresentationlearning_amd.distributed import balanced_shards, block_shards, shard_size
    n = 1 << a.scale
    cfg = W.WharfConfig(walks_per_vertex=a.wpv, walk_length=80, deterministic=False, seed=0x5EED,
                        model=W.NODE2VEC if a.model == "node2vec" else W.DEEPWALK, paramP=a.p, paramQ=a.q)
    which = a.shards if a.shards else list(range(a.parts))
    shards = None
    res = []
    for i in which:
        t0 = time.time()
        g = W.WharfMH.from_rmat(n, a.samples, 2 * n, seed=4, config=cfg)
        if shards is None:
            shards = block_shards(n, a.parts, a.blocks) if a.blocks else \
                balanced_shards(np.diff(g.offsets().astype(np.int64)), a.parts)
        g.apply_shard(shards[i])
        g.generate_initial_random_walks()
        first_st = g.stats()
        first = first_st["last_walk_kernel_ms"]
        g.generate_initial_random_walks()
        gen = g.stats()
        ids = torch.empty(max(g.number_of_walks, 1), dtype=torch.int32, device="cuda:0")
        rec = {k: [] for k in ("ms", "graph", "walk", "steps", "affected", "inits", "inedge")}
        for b in range(a.batches):
            batch = W.generate_batch_of_edges(5000, n, b, False, False)
            for ins in ((True, False) if a.mixed else (True,)):
                t1 = time.perf_counter()
                (g.insert_edges_batch if ins else g.delete_edges_batch)(batch, remove_dups=True, out=ids)
                rec["ms"].append((time.perf_counter() - t1) * 1e3)
                st = g.stats()
                rec["graph"].append(st["last_graph_update_ms"])
                rec["walk"].append(st["last_walk_update_ms"])
                rec["steps"].append(st["steps"])
                rec["affected"].append(st["affected"])
                rec["inits"].append(st["last_anchor_inits"])
                rec["inedge"].append(st["last_csr_move_ms"])
        r = {"shard": i, "shard_def": str(shards[i]), "walks": g.number_of_walks,
             "first_generation_ms": round(first, 2), "generation_ms": round(gen["last_walk_kernel_ms"], 2),
             "generation_steps": gen["steps"], "first_generation_anchor_inits": first_st["last_anchor_inits"],
             "batch_median_ms": round(float(np.median(rec["ms"])), 3),
             "graph_update_median_ms": round(float(np.median(rec["graph"])), 3),
             "walk_update_median_ms": round(float(np.median(rec["walk"])), 3),
             "in_edge_scan_median_ms": round(float(np.median(rec["inedge"])), 3),
             "rewalk_steps_mean": int(np.mean(rec["steps"])), "affected_mean": int(np.mean(rec["affected"])),
             "anchor_inits_mean": int(np.mean(rec["inits"])), "batch_ms": [round(x, 2) for x in rec["ms"]],
             "rewalk_Gsteps_per_s": round(float(np.sum(rec["steps"]) / np.sum(rec["walk"]) / 1e6), 2),
             "wall_s": round(time.time() - t0, 1)}
        print(json.dumps(r), flush=True)
        res.append(r)
        g.destroy()
        torch.cuda.empty_cache()
    b = [r["batch_median_ms"] for r in res]
    w = [r["walk_update_median_ms"] for r in res]
    gen = [r["generation_ms"] for r in res]
    print(json.dumps({"summary": True, "config": f"RMAT scale {a.scale}, {a.samples} samples (seed 4), {a.model} MH, "
                                                 f"wpv {a.wpv}, {a.parts} shards "
                                                 f"({'blocks of 2^%d' % a.blocks if a.blocks else 'ranges'}), "
                                                 f"{a.batches} batches"
                                                 f"{' (insert+delete)' if a.mixed else ''}",
                      "batch_median_ms_max": max(b), "batch_median_ms_min": min(b),
                      "batch_max_over_min": round(max(b) / min(b), 3),
                      "walk_update_max_over_min": round(max(w) / min(w), 3),
                      "generation_max_over_min": round(max(gen) / min(gen), 3)}), flush=True)


if __name__ == "__main__":
    main()
