"""One rank of the multi-process HIP-path test (tests/test_gpu_distributed.py).

Launched by `python -m torch.distributed.run --nproc-per-node N` (gloo, every
rank on cuda:0 of the one-GPU box, or one GPU per rank where there are more).
Each rank loads libwharf_gpu.so, builds its OWN handle over the replicated
CSR with the rank's start-vertex shard (wharf_set_shard: the loop of
wharfmh.h:275 split by start vertex), generates, applies the stream of
batches, and after every step exports its walks on the device
(export_walks_device) and reassembles the global corpus with
distributed.allgatherv_corpus — the production path of bench.py.  Rank 0 also
runs one unsharded handle and the CPU oracle and writes a JSON verdict.

    python -m torch.distributed.run --nproc-per-node 2 tests/dist_shard_worker.py <mode> <out.json>
"""
from __future__ import annotations

import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (before the library: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

import dynamicgraphrepresentationlearning_amd as W  # noqa: E402
from dynamicgraphrepresentationlearning_amd.distributed import allgatherv_corpus, balanced_shards, \
    block_shards, corpus_checksum, gather_corpus_chunked, local_corpus_checksum  # noqa: E402
from oracle import oracle as O  # noqa: E402


def stream(mode: str):
    """(n, off, adj, config kwargs, batches): configs[4]-shaped (node2vec p=.5 q=2
    MH, mixed insert/delete of the same batch, throughput-latency.cpp:126,135)
    or configs[3]-shaped (DeepWalk deterministic, insert batches)."""
    n = 1 << 12
    off, adj = O.csr_from_edges(n, O.generate_batch_of_edges(60000, 2 * n, 6, False, False))
    if mode == "node2vec":
        kw = dict(walks_per_vertex=4, walk_length=40, model=W.NODE2VEC, paramP=0.5, paramQ=2.0,
                  sampler_init=W.WEIGHT, deterministic=False, seed=77)
        batches = []
        for b in range(3):
            e = O.generate_batch_of_edges(400, n, 10 + b, False, False)
            batches += [(True, e), (False, e)]
        batches.append((True, O.generate_batch_of_edges(150, n, 40, False, True)))   # directed
    else:
        kw = dict(walks_per_vertex=10, walk_length=80, deterministic=True)
        batches = [(True, O.generate_batch_of_edges(500, n, b, False, False)) for b in range(4)]
    return n, off, adj, kw, batches


def main():
    mode, out_path = sys.argv[1], sys.argv[2]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    n, off, adj, kw, batches = stream(mode)
    wpv, L = kw["walks_per_vertex"], kw["walk_length"]
    # node2vec: vertex blocks dealt round-robin (bench.py's jobs); det: contiguous ranges
    blocks = mode == "node2vec"
    shards = block_shards(n, world, 6) if blocks else balanced_shards(np.diff(off.astype(np.int64)), world)
    g = W.WharfMH.from_csr(off, adj, config=W.WharfConfig(**kw), device=dev)
    g.apply_shard(shards[rank])
    single = ref = None
    if rank == 0:
        single = W.WharfMH.from_csr(off, adj, config=W.WharfConfig(**kw), device=dev)
        ref = O.Engine(off, adj, wpv=wpv, L=L, model=kw.get("model", 0), p=kw.get("paramP", 4.0),
                       q=kw.get("paramQ", 1.0), init=kw.get("sampler_init", 2),
                       deterministic=kw["deterministic"], seed=kw.get("seed", 0x5EED))

    report = {"mode": mode, "world": world, "shards": [str(x) for x in shards], "steps": []}

    def gather_and_check(tag, local_aff=None):
        loc = torch.empty((g.number_of_walks, L), dtype=torch.int32, device=f"cuda:{dev}")
        g.export_walks_device(loc.data_ptr(), layout="walk")
        torch.cuda.synchronize(dev)
        # the whole-corpus all-gatherv takes contiguous ranges; block shards use the chunked form only
        full = None if blocks else allgatherv_corpus(loc.cpu(), shards, n, wpv).numpy().view(np.uint32)
        # the bounded form bench.py uses at configs[4]: chunks of local rows read from the
        # handle one at a time (device rows staged to the host for gloo), checksum of checksums
        dloc = torch.empty((1000, L), dtype=torch.int32, device=f"cuda:{dev}")

        def read_local(first, count, out):
            d = dloc[:count]
            g.export_walk_rows(first, count, d)
            out.copy_(d.cpu())
            # the host form of the same rows
            assert np.array_equal(g.export_walk_rows(first, count), out.numpy().view(np.uint32))

        got = np.zeros((n * wpv, L), dtype=np.uint32)
        acc = [torch.zeros((), dtype=torch.int64)]

        def sink(chunk, segs):
            for r0, c, g0 in segs:
                got[g0:g0 + c] = chunk[r0:r0 + c].numpy().view(np.uint32)
                acc[0] += corpus_checksum(chunk[r0:r0 + c], g0, L)

        gather_corpus_chunked(read_local, shards, n, wpv, L, 1000, sink)
        mine = local_corpus_checksum(read_local, shards[rank], n, wpv, L, 1000)
        dist.all_reduce(mine)
        chunked_ok = (full is None or bool(np.array_equal(got, full))) and int(acc[0]) == int(mine)
        if full is None:
            full = got
        ok_all = torch.tensor([int(chunked_ok)], dtype=torch.int64)
        dist.all_reduce(ok_all, op=dist.ReduceOp.MIN)
        # the affected ids of all ranks (gathered through the same collective as counts)
        aff_all = None
        if local_aff is not None:
            parts = [None] * world
            dist.all_gather_object(parts, sorted(int(x) for x in local_aff))
            aff_all = np.array(sorted(x for p in parts for x in p), dtype=np.uint32)
        steps = torch.tensor([g.stats()["steps"]], dtype=torch.int64)
        dist.all_reduce(steps)
        if rank == 0:
            rec = {"tag": tag,
                   "corpus_eq_single": bool(np.array_equal(full, single.walks())),
                   "corpus_eq_oracle": bool(np.array_equal(full, ref.walks())),
                   "steps_eq": int(steps.item()) == int(ref.steps),
                   "chunked_eq": bool(ok_all.item())}
            if aff_all is not None:
                rec["affected_eq"] = bool(np.array_equal(aff_all, report["_ref_aff"]))
            report["steps"].append(rec)

    g.generate_initial_random_walks()
    if rank == 0:
        single.generate_initial_random_walks()
        ref.generate()
    gather_and_check("generate")
    for i, (ins, b) in enumerate(batches):
        aff = (g.insert_edges_batch if ins else g.delete_edges_batch)(b, remove_dups=True).copy()
        if rank == 0:
            (single.insert_edges_batch if ins else single.delete_edges_batch)(b, remove_dups=True)
            report["_ref_aff"] = ref.update(ins, b)
        gather_and_check(f"{'ins' if ins else 'del'}{i}", aff)
    g.destroy()
    if rank == 0:
        single.destroy()
        report.pop("_ref_aff", None)
        with open(out_path, "w") as f:
            json.dump(report, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
