"""BASELINE.json configs as parity cases (scaled to oracle-checkable sizes).

configs[0] email-Eu-core DeepWalk det  -> tests/test_gpu_parity.py (wiki, RMAT scale 10, golden)
configs[1] com-orkut generation, MH    -> bench.py headline + test_large_rmat_properties
configs[2] LJ streaming, 50 x 10k-edge inserts, re-walk          -> test_config2_streaming_50_batches
configs[3] twitter initial + inserts, 8 source-vertex shards,
           corpus all-gatherv                                     -> test_config3_eight_shards_stream
configs[4] friendster mixed insert/delete, node2vec p=.5 q=2 MH,
           8 shards                                               -> test_config4_node2vec_mixed_8_shards
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def W():
    import dynamicgraphrepresentationlearning_amd as W
    return W


def _graph(scale, samples, seed):
    n = 1 << scale
    off, adj = O.csr_from_edges(n, O.generate_batch_of_edges(samples, 2 * n, seed, False, False))
    return n, off, adj


def test_config2_streaming_50_batches(W):
    # memory-throughput-latency.cpp:126-134: generate_batch_of_edges(bs, n, seed=trial, false, undirected)
    n, off, adj = _graph(13, 80000, 3)
    cfg = W.WharfConfig(walks_per_vertex=10, walk_length=80, deterministic=True)
    g = W.WharfMH.from_csr(off, adj, config=cfg)
    ref = O.Engine(off, adj, wpv=10, L=80)
    g.generate_initial_random_walks()
    ref.generate()
    for b in range(50):
        batch = W.generate_batch_of_edges(500, n, b, False, False)
        aff = g.insert_edges_batch(batch, remove_dups=True).copy()
        np.testing.assert_array_equal(aff, ref.insert_edges_batch(batch), err_msg=f"batch {b}")
        if b % 10 == 9:
            np.testing.assert_array_equal(g.walks(), ref.walks(), err_msg=f"batch {b}")
    np.testing.assert_array_equal(g.walks(), ref.walks())
    o1, a1 = g.flatten_graph()
    o2, a2 = ref.csr()
    np.testing.assert_array_equal(o1, o2)
    np.testing.assert_array_equal(a1, a2)
    g.destroy()


def _sharded_stream(W, n, off, adj, cfg_kw, batches, shards_n):
    import torch
    from dynamicgraphrepresentationlearning_amd.distributed import balanced_shards, shard_walk_ids
    deg = np.diff(off.astype(np.int64))
    shards = balanced_shards(deg, shards_n)
    ref = O.Engine(off, adj, wpv=cfg_kw["walks_per_vertex"], L=cfg_kw["walk_length"],
                   model=cfg_kw.get("model", 0), p=cfg_kw.get("paramP", 4.0), q=cfg_kw.get("paramQ", 1.0),
                   deterministic=cfg_kw.get("deterministic", True), seed=cfg_kw.get("seed", 0x5EED))
    ref.generate()
    hs = [W.WharfMH.from_csr(off, adj, config=W.WharfConfig(shard_lo=lo, shard_hi=hi, **cfg_kw)) for lo, hi in shards]
    for h in hs:
        h.generate_initial_random_walks()
    wpv, L = cfg_kw["walks_per_vertex"], cfg_kw["walk_length"]
    for ins, b in batches:
        raff = ref.update(ins, b)
        got = []
        for h in hs:
            fn = h.insert_edges_batch if ins else h.delete_edges_batch
            got.append(fn(b, remove_dups=True).copy())
        np.testing.assert_array_equal(np.sort(np.concatenate(got)), raff)
    # corpus reassembly in walk-id order (what allgatherv_corpus does across ranks)
    full = np.empty((n * wpv, L), dtype=np.uint32)
    for (lo, hi), h in zip(shards, hs):
        full[shard_walk_ids(n, wpv, lo, hi)] = h.walks()
        # the device export path used by the RCCL gather
        t = torch.empty((h.number_of_walks, L), dtype=torch.int32, device="cuda:0")
        h.export_walks_device(t.data_ptr(), layout="walk")
        torch.cuda.synchronize()
        np.testing.assert_array_equal(t.cpu().numpy().view(np.uint32), h.walks())
        h.destroy()
    np.testing.assert_array_equal(full, ref.walks())


def test_config3_eight_shards_stream(W):
    n, off, adj = _graph(13, 120000, 5)
    batches = [(True, O.generate_batch_of_edges(500, n, b, False, False)) for b in range(6)]
    _sharded_stream(W, n, off, adj, dict(walks_per_vertex=10, walk_length=80, deterministic=True), batches, 8)


def test_config4_node2vec_mixed_8_shards(W):
    n, off, adj = _graph(12, 60000, 6)
    batches = []
    for b in range(4):     # throughput-latency.cpp:126,135: insert batch b, then delete the same batch
        e = O.generate_batch_of_edges(400, n, 10 + b, False, False)
        batches += [(True, e), (False, e)]
    _sharded_stream(W, n, off, adj, dict(walks_per_vertex=4, walk_length=40, model=1, paramP=0.5, paramQ=2.0,
                                         deterministic=False, seed=77), batches, 8)


def test_node2vec_long_mixed_stream_vs_oracle(W):
    """25 batches of mixed inserts/deletes (undirected and directed) on one
    handle: the anchor cache's epoch tags stay exact across many resets."""
    n, off, adj = _graph(11, 25000, 9)
    rng = np.random.default_rng(3)
    batches = []
    for b in range(25):
        e = O.generate_batch_of_edges(int(rng.integers(20, 400)), n, 100 + b, False, bool(b % 3 == 2))
        batches.append((bool(rng.integers(0, 2)) or b < 3, e, O.REMOVE_DUPS | O.APPLY_WALK_UPDATES))
    from test_gpu_parity import _compare_stream
    _compare_stream(W, off, adj, batches, wpv=3, L=30, model=1, paramP=0.5, paramQ=2.0, deterministic=False, seed=41)
