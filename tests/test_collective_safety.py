"""Collective safety of the multi-rank path (gloo, worlds 2 and 4, CPU only).

VERDICT r05 #5: (a) each rank derives the corpus gather's chunk from its own
free memory, and the chunk boundaries and receive sizes must still agree
across ranks; (b) a rank that fails a job phase must not leave its peers
inside a collective.  Here the ranks pass DIFFERENT gather budgets (the
corpus must still arrive bit-exact), and a WHARF_TEST_FAIL hook makes one
rank fail each phase of bench.py's 8-GPU jobs in turn (every rank must return
the same error record, naming the failing rank and phase, and exit 0).

bench.multi_gpu_job runs against tests/fake_wharf.py's host stand-in for the
library (its walks are a pure function of the walk id), so only the job's
control flow and collectives are exercised here; the GPU path of the same
code is tests/test_gpu_rccl.py."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

CASES = [("ok", "configs4", ""), ("build", "configs4", "1:build"), ("generation", "configs4", "1:generation"),
         ("gather", "configs4", "1:gather"), ("gather_read", "configs4", "0:gather_read"),
         ("batch", "configs4", "1:batch"), ("one_gpu", "configs3", "1:one_gpu"), ("ok3", "configs3", ""),
         ("alloc_oom", "configs4", "1:alloc_oom")]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        import bench
        from fake_wharf import FakeHandle, FakeW, TorchProxy, walk_value
        from dynamicgraphrepresentationlearning_amd.distributed import block_shards, gather_corpus_chunked, \
            shard_size
        T = TorchProxy()

        def barrier():
            dist.barrier()

        sys.argv = ["bench.py", "--job-scale-delta", "-20", "--job-batches", "2", "--job-block-bits", "2"]
        args = bench.parse()
        jobs = {}
        for tag, job, spec in CASES:
            os.environ["WHARF_TEST_FAIL"] = spec
            FakeHandle.released = 0
            jobs[tag] = bench.multi_gpu_job(args, job, FakeW, T, 0, world, rank, dist, "cpu", barrier)
            jobs[tag]["_released"] = FakeHandle.released
        os.environ.pop("WHARF_TEST_FAIL", None)

        # (a) unequal budgets: rank 0 can hold 3 rows per rank per chunk, rank 1 fifty
        n, wpv, L = 96, 10, 80
        g = FakeW.WharfMH.from_rmat(n, 0, 2 * n, config=FakeW.WharfConfig(walks_per_vertex=wpv, walk_length=L))
        shards = block_shards(n, world, 3)
        g.apply_shard(shards[rank])
        K = 3 if rank == 0 else 50
        rec = bench.corpus_gather_record(args, T, dist, g, shards, n, wpv, L, 0, "cpu", world, rank, barrier,
                                         K * world * L * 4)
        got = np.full((n * wpv, L), -1, dtype=np.int64)
        sizes = []

        def sink(chunk, segs):
            sizes.append(chunk.shape[0])
            for r0, c, g0 in segs:
                got[g0:g0 + c] = chunk[r0:r0 + c].numpy()

        st = gather_corpus_chunked(lambda f, c, out: g.export_walk_rows(f, c, out), shards, n, wpv, L, K, sink)
        want = walk_value(np.arange(n * wpv)[:, None], np.arange(L)[None, :])
        exact = bool(np.array_equal(got, want)) and max(sizes) <= 3 * world and \
            st["chunks"] == -(-max(shard_size(sh) * wpv for sh in shards) // 3)
        q.put((rank, jobs, rec, exact, st["rows_per_rank"]))
    except Exception as ex:   # noqa: BLE001
        q.put((rank, {"worker_error": repr(ex)}, None, False, None))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module", params=[2, 4], ids=["world2", "world4"])
def results(request):
    world = request.param
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    return {r[0]: r for r in res}, [p.exitcode for p in procs]


def test_ranks_exit_cleanly(results):
    res, codes = results
    assert codes == [0] * len(codes), codes
    for rank, (_, jobs, *_rest) in res.items():
        assert "worker_error" not in jobs, jobs


def test_unequal_gather_budgets_agree_and_deliver_bit_exact(results):
    res, _ = results
    for rank, (_, _, rec, exact, k) in res.items():
        assert exact, rank
        assert k == 3
        assert rec["rows_per_rank_per_chunk"] == 3
        assert rec["rows_per_rank_this_rank_budget"] == (3 if rank == 0 else 50)
        assert rec["checksum_of_checksums_ok"] is True


@pytest.mark.parametrize("tag,job,spec", CASES)
def test_one_rank_failure_is_agreed_by_every_rank(results, tag, job, spec):
    res, _ = results
    recs = [res[r][1][tag] for r in range(len(res))]
    if not spec:
        for r in recs:
            assert "error" not in r, r
            assert r["generation_steps"] > 0
            assert r["updates"] == (4 if job == "configs4" else 2)
        if job == "configs4":
            assert all(r["corpus_allgatherv"]["checksum_of_checksums_ok"] for r in recs)
        else:
            assert "one_gpu_same_graph" in recs[0]
        return
    bad_rank, phase = spec.split(":")
    if phase == "alloc_oom":   # an out-of-memory buffer: the rank frees the library's caches and retries
        for rank, r in enumerate(recs):
            assert "error" not in r, r
            assert r["corpus_allgatherv"]["checksum_of_checksums_ok"]
            assert r["_released"] == (1 if rank == int(bad_rank) else 0), (rank, r["_released"])
        return
    for r in recs:
        assert "error" in r, r
        assert r["failed_rank"] == int(bad_rank), r
        assert r["phase"].startswith({"gather": "corpus gather setup", "gather_read": "corpus gather chunk"}
                                     .get(phase, phase)), r
        assert "injected fault" in r["error"], r
