"""One RCCL rank on the one-GPU box (tests/test_gpu_rccl.py).

RCCL refuses two ranks on one device ("Duplicate GPU detected"), so the only
way to execute the `nccl` leg of bench.py and distributed.py before the
driver's 8-GPU run is a world of one.  This rank runs, on a live RCCL
communicator:
  * init_process_group("nccl", device_id=...) exactly as bench.py does;
  * bench.py's device-tensor collectives (_max_over_ranks, _sum_over_ranks,
    _per_rank) and the barrier;
  * bench.corpus_gather_record -> distributed.gather_corpus_chunked with device
    buffers and rows exported by the HIP library per chunk (both passes and the
    checksum of checksums), plus a sink that rebuilds the corpus, compared with
    the handle's own export;
  * a batch_isend_irecv of a device chunk to the rank itself (whether torch and
    RCCL accept a self-peer is recorded either way; the mesh gather never sends
    to itself).
The report is written before the self-peer attempt, which runs under a watchdog.

    python -m torch.distributed.run --nproc-per-node 1 tests/rccl_world1_worker.py <out.json>
"""
from __future__ import annotations

import json
import os
import sys
import threading
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (before the library: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402


def main():
    out_path = sys.argv[1]
    dev = 0
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    import bench
    import dynamicgraphrepresentationlearning_amd as W
    from dynamicgraphrepresentationlearning_amd.distributed import block_shards, gather_corpus_chunked

    comm = f"cuda:{dev}"
    rep = {"backend": dist.get_backend(), "world": dist.get_world_size(), "rank": dist.get_rank(),
           "rccl_version": ".".join(map(str, torch.cuda.nccl.version())) if hasattr(torch.cuda, "nccl") else None}
    rep["max_over_ranks"] = bench._max_over_ranks(torch, dist, comm, [1.5, -2.0, 7.25])
    rep["sum_over_ranks"] = bench._sum_over_ranks(torch, dist, comm, [3.0, 4.5])
    rep["per_rank"] = bench._per_rank(torch, dist, comm, [11.0, 12.0], 1)
    dist.barrier()
    torch.cuda.synchronize(dev)
    rep["collectives_ok"] = (rep["max_over_ranks"] == [1.5, -2.0, 7.25] and rep["sum_over_ranks"] == [3.0, 4.5]
                             and rep["per_rank"] == [[11.0, 12.0]])

    # the chunked gather, as bench.py runs it for both 8-GPU jobs (block shards, device buffers)
    n, wpv, L = 1 << 15, 3, 40
    cfg = W.WharfConfig(walks_per_vertex=wpv, walk_length=L, model=W.NODE2VEC, paramP=0.5, paramQ=2.0,
                        deterministic=False, seed=21)
    g = W.WharfMH.from_rmat(n, 400_000, 2 * n, seed=3, config=cfg, device=dev)
    shards = block_shards(n, 1, 12)
    g.apply_shard(shards[0])
    g.generate_initial_random_walks()

    def barrier():
        dist.barrier()
        torch.cuda.synchronize(dev)

    args = types.SimpleNamespace(gather_check=1)
    rec = bench.corpus_gather_record(args, torch, dist, g, shards, n, wpv, L, dev, comm, 1, 0, barrier,
                                     budget_bytes=5000 * L * 4)
    rep["corpus_gather_record"] = rec
    want = g.walks()
    got = np.zeros_like(want)

    def read_local(first, count, out):
        g.export_walk_rows(first, count, out)

    def sink(chunk, segs):
        h = chunk.cpu().numpy().view(np.uint32)
        for r0, c, g0 in segs:
            got[g0:g0 + c] = h[r0:r0 + c]

    st = gather_corpus_chunked(read_local, shards, n, wpv, L, 7000, sink, device=comm)
    rep["chunked_gather_chunks"] = st["chunks"]
    rep["chunked_gather_eq_export"] = bool(np.array_equal(got, want))
    # gatherv form (root 0) as the export-to-disk path uses it
    got[:] = 0
    gather_corpus_chunked(read_local, shards, n, wpv, L, 9000, sink, root=0, device=comm)
    rep["gatherv_eq_export"] = bool(np.array_equal(got, want))
    g.destroy()
    with open(out_path, "w") as f:
        json.dump(rep, f)

    # self-peer batch_isend_irecv of a device chunk: recorded either way, under a watchdog
    def watchdog():
        rep["self_p2p"] = {"outcome": "hung > 60 s"}
        with open(out_path, "w") as f:
            json.dump(rep, f)
        os._exit(0)

    t = threading.Timer(60.0, watchdog)
    t.daemon = True
    t.start()
    try:
        src = torch.arange(1 << 20, dtype=torch.int32, device=comm)
        dst = torch.full_like(src, -1)
        reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, src, 0), dist.P2POp(dist.irecv, dst, 0)])
        for r in reqs:
            r.wait()
        torch.cuda.synchronize(dev)
        rep["self_p2p"] = {"outcome": "accepted", "data_eq": bool(torch.equal(src, dst))}
    except Exception as ex:   # noqa: BLE001 (the outcome is the record)
        rep["self_p2p"] = {"outcome": "refused", "error": f"{type(ex).__name__}: {str(ex)[:300]}"}
    t.cancel()
    with open(out_path, "w") as f:
        json.dump(rep, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
