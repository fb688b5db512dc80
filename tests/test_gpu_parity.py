"""GPU parity: the HIP path (through the C ABI) against the reference's golden
vectors and the CPU oracle.  Run on an MI355X with ``pytest -m gpu``.

Bit-exact for every integer output (walk corpus, affected walk ids, CSR,
inverted index, RMAT batches, MH walks under the Philox semantics);
statistical (stated tolerances) for MH transition classes against the
reference, whose MH mode is not reproducible.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import mh_stats
from oracle import oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def W():
    import dynamicgraphrepresentationlearning_amd as W
    return W


@pytest.fixture(scope="module")
def meta():
    return json.load(open(os.path.join(G, "golden.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _has_edge(off, adj, a, c):
    """vectorised (a -> c) in CSR"""
    n = len(off) - 1
    src = np.repeat(np.arange(n, dtype=np.int64), np.diff(off.astype(np.int64)))
    ekeys = src * n + adj.astype(np.int64)          # ascending: rows sorted
    q = a.astype(np.int64) * n + c.astype(np.int64)
    j = np.minimum(np.searchsorted(ekeys, q), max(len(ekeys) - 1, 0))
    return ekeys[j] == q


def det_cfg(W, wpv, L, model=0):
    return W.WharfConfig(walks_per_vertex=wpv, walk_length=L, model=model, deterministic=True)


# ---------------------------------------------------------------------------
# deterministic mode vs the reference's own outputs
# ---------------------------------------------------------------------------
def test_six_vertex_golden(W, meta):
    z = np.load(os.path.join(G, "six.npz"))
    for model in (W.DEEPWALK, W.NODE2VEC):
        g = W.WharfMH.from_csr(z["off"], z["adj"], config=det_cfg(W, 2, 5, model))
        g.generate_initial_random_walks()
        np.testing.assert_array_equal(g.walks(), z["walks"])
        c, k, nx = g.inverted_index()
        np.testing.assert_array_equal(c, z["index_counts"])
        np.testing.assert_array_equal(k, z["index_keys"])
        np.testing.assert_array_equal(nx, z["index_nexts"])
        assert g.walk(0) == meta["six_walkstr"]["0"]
        assert g.walk(11) == meta["six_walkstr"]["11"]
        assert g.vertex_at_walk(11, 4) == int(z["walks"][11, 4])
        assert g.stats()["steps"] == 12 * 4
        g.destroy()


def _paired_reference(counts, keys, nexts):
    """CompressedWalks values from the golden (key, next) lists: per vertex,
    Szudzik(key, next) ascending (the oracle's codec pins the formula)."""
    a, b = keys.astype(np.uint64), nexts.astype(np.uint64)
    z = np.where(b >= a, b * (b + np.uint64(1)) + a, a * a + b)
    for i in range(0, len(z), max(len(z) // 17, 1)):
        assert int(z[i]) == O.szudzik64_pair(int(a[i]), int(b[i]))
    off = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
    return np.concatenate([np.sort(z[off[v]:off[v + 1]]) for v in range(len(counts))])


def test_compressed_walks_pairing_export(W):
    """wharf_export_index_paired against the golden inverted indexes."""
    z = np.load(os.path.join(G, "six.npz"))
    g = W.WharfMH.from_csr(z["off"], z["adj"], config=det_cfg(W, 2, 5))
    g.generate_initial_random_walks()
    c, p = g.compressed_walks()
    np.testing.assert_array_equal(c, z["index_counts"])
    np.testing.assert_array_equal(p, _paired_reference(z["index_counts"], z["index_keys"], z["index_nexts"]))
    g.destroy()
    r = np.load(os.path.join(G, "rmat10.npz"))
    g = W.WharfMH.from_rmat(1024, 12800, 2048, seed=1, config=det_cfg(W, 2, 20))
    g.generate_initial_random_walks()
    c, p = g.compressed_walks()
    np.testing.assert_array_equal(c, r["index_counts_0"])
    np.testing.assert_array_equal(p, _paired_reference(r["index_counts_0"], r["index_keys_0"], r["index_nexts_0"]))
    g.destroy()


def test_rmat_batches_golden(W):
    z = np.load(os.path.join(G, "rmat_batches.npz"))
    for k in z.files:
        _, M, V, s, d = k.split("_")
        got = W.generate_batch_of_edges(int(M), int(V), int(s), False, bool(int(d)))
        np.testing.assert_array_equal(got, z[k], err_msg=k)


def test_rmat10_streaming_golden(W):
    z = np.load(os.path.join(G, "rmat10.npz"))
    for model in (W.DEEPWALK, W.NODE2VEC):
        g = W.WharfMH.from_rmat(1024, 12800, 2048, seed=1, config=det_cfg(W, 2, 20, model))
        off, adj = g.flatten_graph()
        np.testing.assert_array_equal(off, z["off_0"])
        np.testing.assert_array_equal(adj, z["adj_0"])
        assert g.number_of_edges() == len(z["adj_0"])
        g.generate_initial_random_walks()
        np.testing.assert_array_equal(g.walks(), z["walks_gen"])
        c, k, nx = g.inverted_index()
        np.testing.assert_array_equal(c, z["index_counts_0"])
        np.testing.assert_array_equal(k, z["index_keys_0"])
        np.testing.assert_array_equal(nx, z["index_nexts_0"])
        steps = [("1_ins", True, "ins1", "1"), ("2_del", False, "del2", "2"), ("3_ins", True, "ins3", "3"),
                 ("4_del", False, "del4", "4")]
        for tag, ins, wname, gtag in steps:
            fn = g.insert_edges_batch if ins else g.delete_edges_batch
            aff = fn(z[f"batch_{tag}"], sorted=False, remove_dups=True)
            np.testing.assert_array_equal(aff, z[f"affected_{tag}"], err_msg=tag)
            o2, a2 = g.flatten_graph()
            np.testing.assert_array_equal(o2, z[f"off_{gtag}"], err_msg=tag)
            np.testing.assert_array_equal(a2, z[f"adj_{gtag}"], err_msg=tag)
            np.testing.assert_array_equal(g.offsets(), o2, err_msg=tag)
            np.testing.assert_array_equal(g.walks(), z[f"walks_{wname}"], err_msg=tag)
            if f"index_counts_{gtag}" in z.files:
                c, k, nx = g.inverted_index()
                np.testing.assert_array_equal(c, z[f"index_counts_{gtag}"])
                np.testing.assert_array_equal(k, z[f"index_keys_{gtag}"])
                np.testing.assert_array_equal(nx, z[f"index_nexts_{gtag}"])
        g.destroy()


def test_rmat10_directed_golden(W):
    z = np.load(os.path.join(G, "rmat10_directed.npz"))
    g = W.WharfMH.from_rmat(1024, 12800, 2048, seed=1, config=det_cfg(W, 2, 20))
    g.generate_initial_random_walks()
    np.testing.assert_array_equal(g.walks(), z["walks_gen"])
    b = W.generate_batch_of_edges(50, 1024, 0, False, True)
    np.testing.assert_array_equal(b, z["batch_ins"])
    np.testing.assert_array_equal(g.insert_edges_batch(b, remove_dups=True), z["affected_ins"])
    np.testing.assert_array_equal(g.walks(), z["walks_ins"])
    np.testing.assert_array_equal(g.delete_edges_batch(b, remove_dups=True), z["affected_del"])
    np.testing.assert_array_equal(g.walks(), z["walks_del"])


def test_wiki_full_corpus_golden(W, meta):
    z = np.load(os.path.join(G, "wiki_csr.npz"))
    wz = np.load(os.path.join(G, "wiki_golden.npz"))
    gm = meta["wiki"]
    g = W.WharfMH.from_csr(z["off"], z["adj"], config=det_cfg(W, 10, 80))
    assert g.number_of_vertices() == 2405 and g.number_of_edges() == 23192
    g.generate_initial_random_walks()
    w = g.walks()
    np.testing.assert_array_equal(w[:64], wz["first64_0_gen"])
    assert sha(w) == gm["0_gen"]["sha256"]
    b = wz["batch_1_ins"]
    aff = g.insert_edges_batch(b, remove_dups=True)
    assert len(aff) == gm["affected_1_ins"]["count"] and sha(aff) == gm["affected_1_ins"]["sha256"]
    assert sha(g.walks()) == gm["1_ins"]["sha256"]
    aff = g.delete_edges_batch(b, remove_dups=True)
    assert len(aff) == gm["affected_2_del"]["count"] and sha(aff) == gm["affected_2_del"]["sha256"]
    assert sha(g.walks()) == gm["2_del"]["sha256"]
    assert g.walk(12345) == gm["walkstr_12345"]


# ---------------------------------------------------------------------------
# deterministic mode vs the oracle: edge cases
# ---------------------------------------------------------------------------
def _compare_stream(W, off, adj, batches, wpv=3, L=12, **kw):
    cfg = W.WharfConfig(walks_per_vertex=wpv, walk_length=L, **kw)
    g = W.WharfMH.from_csr(off, adj, config=cfg)
    ref = O.Engine(off, adj, wpv=wpv, L=L, model=cfg.model, p=cfg.paramP, q=cfg.paramQ, init=cfg.sampler_init,
                   deterministic=cfg.deterministic, seed=cfg.seed)
    g.generate_initial_random_walks()
    ref.generate()
    np.testing.assert_array_equal(g.walks(), ref.walks())
    assert g.stats()["steps"] == ref.steps
    assert g.stats()["accepts"] == ref.accepts
    for ins, b, flags in batches:
        fn = g.insert_edges_batch if ins else g.delete_edges_batch
        aff = fn(b, remove_dups=bool(flags & O.REMOVE_DUPS), apply_walk_updates=bool(flags & O.APPLY_WALK_UPDATES))
        aff_r = ref.update(ins, b, flags)
        np.testing.assert_array_equal(aff, aff_r)
        np.testing.assert_array_equal(g.walks(), ref.walks())
        o2, a2 = g.flatten_graph()
        o3, a3 = ref.csr()
        np.testing.assert_array_equal(o2, o3)
        np.testing.assert_array_equal(a2, a3)
        if flags & O.APPLY_WALK_UPDATES:
            assert g.stats()["steps"] == ref.steps
            assert g.stats()["accepts"] == ref.accepts
    g.destroy()


@pytest.mark.parametrize("preinit_all", ["0", "1", "1-by-cur", "1-by-prev", "1-hybrid", "1-hybrid-all"])
@pytest.mark.parametrize("init", [1, 2])   # BURNIN, WEIGHT
def test_node2vec_anchors_up_front_or_lazily(W, monkeypatch, preinit_all, init):
    """Every anchor computed at the first generation (round 4's rule: >= 1 walk step
    per slot) or lazily by the walkers (WHARF_PREINIT_ALL=0): the same corpus,
    counters, affected ids and CSR as the oracle either way, with few walks per
    slot (wpv 1, L 20 on ~5 k slots: ~4 steps per slot) and a stream of inserts
    and deletes, so the re-walks run into states no walker had entered.  Up
    front, the states of hub curs with small prevs are computed in cur order
    (k_anchor_init_by_cur; 1-by-cur: thresholds lowered so that most states go
    that way) or all in prev order (1-by-prev: WHARF_INIT_BY_CUR=0).  With the reverse-slot
    index (1-hybrid*, WHARF_REV=1) each state goes to the cheaper order by the line model
    (k_anchor_init_all + k_anchor_init_cur); the bias moves the small test graph's states to
    cur order when their cur's row spans 2+ lines (1-hybrid, reverse slots verified) or all of
    them (1-hybrid-all, the production instantiation without the check)."""
    monkeypatch.setenv("WHARF_PREINIT_ALL", preinit_all[0])
    hybrid = preinit_all.startswith("1-hybrid")
    if hybrid:
        monkeypatch.setenv("WHARF_REV", "1")
        monkeypatch.setenv("WHARF_INIT_CUR_BIAS", "-100" if preinit_all == "1-hybrid-all" else "-1.5")
        # the default (unverified) instantiation of k_anchor_init_cur too: the index is exact here
        monkeypatch.setenv("WHARF_REV_VERIFY", "0" if preinit_all == "1-hybrid-all" else "1")
    else:
        monkeypatch.delenv("WHARF_REV", raising=False)
        monkeypatch.delenv("WHARF_INIT_CUR_BIAS", raising=False)
    monkeypatch.setenv("WHARF_NO_PREINIT", "")
    monkeypatch.setenv("WHARF_INIT_BY_CUR", "0" if preinit_all == "1-by-prev" else "1")
    monkeypatch.setenv("WHARF_INIT_BY_CUR_Y", "4" if preinit_all == "1-by-cur" else "")
    monkeypatch.setenv("WHARF_INIT_BY_CUR_X", "40" if preinit_all == "1-by-cur" else "")
    base = O.generate_batch_of_edges(4000, 1 << 11, 9, False, False)
    off, adj = O.csr_from_edges(1 << 10, base)
    batches = [(True, O.generate_batch_of_edges(300, 1 << 10, 21, False, False), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES),
               (False, O.generate_batch_of_edges(200, 1 << 10, 22, False, False), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES),
               (True, O.generate_batch_of_edges(300, 1 << 10, 23, False, False), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES)]
    _compare_stream(W, off, adj, batches, wpv=1, L=20, deterministic=False, seed=17, model=1, paramP=0.5,
                    paramQ=2.0, sampler_init=init)
    # which path ran: up front, exactly one init per slot (every target has a neighbour: undirected) and
    # none left for the walkers; lazily, one per state entered, plus duplicates of states two walkers
    # enter at once (benign: the same value)
    g = W.WharfMH.from_csr(off, adj, config=W.WharfConfig(walks_per_vertex=1, walk_length=20, deterministic=False,
                                                          seed=17, model=1, paramP=0.5, paramQ=2.0,
                                                          sampler_init=init))
    g.generate_initial_random_walks()
    inits = g.stats()["last_anchor_inits"]
    csr_bytes = g.memory_footprint(verbose=False)["csr_bytes"]
    g.destroy()
    assert (inits == len(adj)) if preinit_all != "0" else (0 < inits != len(adj)), (inits, len(adj))
    if hybrid:   # the two-order path needs the reverse-slot index: it was there (4 B per slot)
        monkeypatch.setenv("WHARF_REV", "0")
        g0 = W.WharfMH.from_csr(off, adj, config=W.WharfConfig(walks_per_vertex=1, walk_length=20, deterministic=False,
                                                               seed=17, model=1, paramP=0.5, paramQ=2.0,
                                                               sampler_init=init))
        assert csr_bytes >= g0.memory_footprint(verbose=False)["csr_bytes"] + 4 * len(adj)
        g0.destroy()


@pytest.mark.parametrize("init", [1, 2])   # BURNIN, WEIGHT
def test_up_front_init_orders_agree_on_an_rmat_graph_with_hubs(W, monkeypatch, init):
    """The two-order up-front inits at a size where the line model itself sends hub curs' states to
    cur order (no bias): RMAT scale 15 with the reverse-slot index forced on.  Anchors are a pure
    function of the snapshot, so prev order only (WHARF_INIT_ORDER=0), the two orders with the
    reverse slots verified, and the two orders unverified give the same corpus and counters, then the
    same corpus again after an insert and a delete batch."""
    monkeypatch.setenv("WHARF_REV", "1")
    monkeypatch.setenv("WHARF_PREINIT_ALL", "1")
    monkeypatch.delenv("WHARF_INIT_CUR_BIAS", raising=False)
    n = 1 << 15
    cfg = W.WharfConfig(walks_per_vertex=2, walk_length=24, model=1, paramP=0.5, paramQ=2.0, deterministic=False,
                        seed=23, sampler_init=init)
    ins = O.generate_batch_of_edges(3000, n, 41, False, False)
    out = {}
    for variant, order, verify in (("prev", "0", "1"), ("two-verified", "1", "1"), ("two", "1", "0")):
        monkeypatch.setenv("WHARF_INIT_ORDER", order)
        monkeypatch.setenv("WHARF_REV_VERIFY", verify)
        g = W.WharfMH.from_rmat(n, 400_000, 2 * n, seed=5, config=cfg)
        g.generate_initial_random_walks()
        st = g.stats()
        assert st["last_anchor_inits"] == g.number_of_edges()   # one init per state, up front
        w0 = g.walks()
        g.insert_edges_batch(ins, sorted=False, remove_dups=True)
        w1 = g.walks()
        g.delete_edges_batch(ins, sorted=False, remove_dups=True)
        out[variant] = (w0, st["steps"], st["accepts"], w1, g.walks())
        g.destroy()
    for variant in ("two-verified", "two"):
        for a, b in zip(out["prev"], out[variant]):
            np.testing.assert_array_equal(a, b)


def test_edge_cases_isolated_dead_ends_and_flags(W):
    # vertex 5 isolated, 6 a sink (directed edge 4->6), self loop 3->3
    off = np.array([0, 2, 4, 7, 9, 11, 11, 11], dtype=np.uint64)
    adj = np.array([1, 2, 0, 2, 0, 1, 3, 2, 3, 2, 6], dtype=np.uint32)
    R, A = O.REMOVE_DUPS, O.APPLY_WALK_UPDATES
    batches = [
        (True, np.array([[5, 0], [0, 5], [5, 0]], np.uint32), R | A),        # isolated vertex gets edges; dup
        (False, np.array([[4, 2], [4, 6]], np.uint32), R | A),               # 4 loses every edge -> dead end
        (True, np.array([[6, 6], [1, 6]], np.uint32), A),                    # self loop kept (no REMOVE_DUPS)
        (True, np.array([[2, 5]], np.uint32), R),                            # apply_walk_updates = false
        (False, np.array([[0, 1], [1, 0], [6, 6]], np.uint32), R | A),
        (True, np.zeros((0, 2), np.uint32), R | A),                          # empty batch
        (False, np.array([[3, 6]], np.uint32), R | A),                       # absent edge: row unchanged, still a source
    ]
    _compare_stream(W, off, adj, batches, wpv=3, L=12)
    _compare_stream(W, off, adj, batches, wpv=2, L=9, model=1, paramP=0.5, paramQ=2.0, deterministic=False, seed=3)
    _compare_stream(W, off, adj, batches, wpv=2, L=9, model=0, deterministic=False, seed=9)


@pytest.mark.parametrize("wpv,L", [(3, 2), (1, 255), (255, 7)])
@pytest.mark.parametrize("mode", ["det", "deepwalk", "node2vec"])
def test_extreme_walk_shapes(W, wpv, L, mode):
    """The u8 limits of types::Position / walks_per_vertex (L = 2 and 255, wpv = 255)
    through generation and updates, against the oracle."""
    base = O.generate_batch_of_edges(3000, 512, 8, False, False)
    off, adj = O.csr_from_edges(300, base)
    batches = [(True, O.generate_batch_of_edges(200, 300, 21, False, False), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES),
               (False, O.generate_batch_of_edges(150, 300, 22, False, False), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES)]
    kw = dict(deterministic=True) if mode == "det" else dict(
        deterministic=False, seed=5, model=1 if mode == "node2vec" else 0, paramP=0.5, paramQ=2.0)
    _compare_stream(W, off, adj, batches, wpv=wpv, L=L, **kw)


def test_single_vertex_graph(W):
    g = W.WharfMH(1, 0, config=det_cfg(W, 3, 4))
    g.generate_initial_random_walks()
    assert (g.walks()[:, 0] == 0).all() and (g.walks()[:, 1:] == W.SENTINEL).all()
    aff = g.insert_edges_batch(np.array([[0, 0]], np.uint32))     # a self loop: every walk re-walks on it
    assert aff.tolist() == [0, 1, 2] and (g.walks() == 0).all()
    g.destroy()


def test_empty_graph_and_errors(W):
    g = W.WharfMH(10, 0, config=det_cfg(W, 2, 5))
    assert g.number_of_edges() == 0
    g.generate_initial_random_walks()
    w = g.walks()
    assert (w[:, 0] == np.tile(np.arange(10), 2)).all() and (w[:, 1:] == W.SENTINEL).all()
    assert g.walk(13) == "3 "
    with pytest.raises(RuntimeError):
        g.insert_edges_batch(np.array([[1, 10]], np.uint32))      # id >= n
    with pytest.raises(RuntimeError):
        g.walk(20)                                                # wid >= n * wpv
    with pytest.raises(RuntimeError):
        W.WharfMH(4, 1, np.zeros(4, np.uint64), np.array([7], np.uint32))   # target >= n
    with pytest.raises(RuntimeError):
        W.WharfMH(4, 0, config=W.WharfConfig(walk_length=300))
    aff = g.insert_edges_batch(np.array([[1, 2], [2, 1]], np.uint32), remove_dups=True)
    assert sorted(aff.tolist()) == [1, 2, 11, 12]
    g.destroy_index()
    assert (g.walks() == W.SENTINEL).all()


def test_rmat_scale14_stream_vs_oracle(W):
    base = O.generate_batch_of_edges(200000, 1 << 15, 4, False, False)
    off, adj = O.csr_from_edges(1 << 14, base)
    batches = []
    for s in range(3):
        b = O.generate_batch_of_edges(5000, 1 << 14, 100 + s, False, False)
        batches.append((True, b, O.REMOVE_DUPS | O.APPLY_WALK_UPDATES))
        batches.append((False, b, O.REMOVE_DUPS | O.APPLY_WALK_UPDATES))
    batches.append((True, O.generate_batch_of_edges(3000, 1 << 14, 77, False, True), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES))
    _compare_stream(W, off, adj, batches, wpv=10, L=80)


@pytest.mark.parametrize("mode", ["det", "deepwalk", "node2vec"])
def test_batch_walk_update_deferred_equals_applied(W, mode):
    """wharf_batch_walk_update (wharfmh.h:733): an update with
    apply_walk_updates=False followed by batch_walk_update(the batch's sources)
    gives the walks and affected ids of the applied update, which equal the
    oracle's; a standalone call over a vertex set equals an update whose batch
    has those sources and changes no edge (deterministic: same draws)."""
    base = O.generate_batch_of_edges(40000, 1 << 12, 31, False, False)
    off, adj = O.csr_from_edges(1 << 12, base)
    kw = dict(deterministic=True) if mode == "det" else dict(
        deterministic=False, seed=11, model=1 if mode == "node2vec" else 0, paramP=0.5, paramQ=2.0)
    cfg = W.WharfConfig(walks_per_vertex=4, walk_length=40, **kw)
    ga = W.WharfMH.from_csr(off, adj, config=cfg)
    gd = W.WharfMH.from_csr(off, adj, config=cfg)
    ref = O.Engine(off, adj, wpv=4, L=40, model=cfg.model, p=cfg.paramP, q=cfg.paramQ, init=cfg.sampler_init,
                   deterministic=cfg.deterministic, seed=cfg.seed)
    for g in (ga, gd):
        g.generate_initial_random_walks()
    ref.generate()
    for s, ins in ((41, True), (42, False), (43, True)):
        b = O.generate_batch_of_edges(600, 1 << 12, s, False, False)
        fa = ga.insert_edges_batch if ins else ga.delete_edges_batch
        fd = gd.insert_edges_batch if ins else gd.delete_edges_batch
        aa = fa(b, remove_dups=True)
        fd(b, remove_dups=True, apply_walk_updates=False)
        ad = gd.batch_walk_update(b[:, 0][::-1])          # any order, duplicates allowed
        ar = ref.update(ins, b, O.REMOVE_DUPS | O.APPLY_WALK_UPDATES)
        np.testing.assert_array_equal(aa, ar)
        np.testing.assert_array_equal(ad, aa)
        np.testing.assert_array_equal(gd.walks(), ga.walks())
        np.testing.assert_array_equal(ga.walks(), ref.walks())
        assert gd.stats()["steps"] == ga.stats()["steps"] == ref.steps
    if mode == "det":
        # standalone: sources S, graph unchanged == an insert of existing edges out of S
        o2, a2 = ga.flatten_graph()
        S = np.array([v for v in range(0, 1 << 12, 37) if o2[v + 1] > o2[v]], np.uint32)
        ex = np.stack([S, a2[o2[S].astype(np.int64)]], axis=1).astype(np.uint32)
        ad = gd.batch_walk_update(S)
        ar = ref.update(True, ex, O.REMOVE_DUPS | O.APPLY_WALK_UPDATES)
        np.testing.assert_array_equal(ad, ar)
        np.testing.assert_array_equal(gd.walks(), ref.walks())
    assert len(gd.batch_walk_update(np.zeros(0, np.uint32))) == 0
    with pytest.raises(RuntimeError):
        gd.batch_walk_update(np.array([1 << 12], np.uint32))
    ga.destroy()
    gd.destroy()


def test_affected_ids_on_device_match_host_list(W):
    """WHARF_AFFECTED_DEVICE: ids written to HBM equal the host list and the oracle's."""
    import torch
    base = O.generate_batch_of_edges(60000, 1 << 13, 9, False, False)
    off, adj = O.csr_from_edges(1 << 13, base)
    cfg = W.WharfConfig(walks_per_vertex=3, walk_length=30, model=W.DEEPWALK, deterministic=False, seed=7)
    gh = W.WharfMH.from_csr(off, adj, config=cfg)
    gd = W.WharfMH.from_csr(off, adj, config=cfg)
    ref = O.Engine(off, adj, wpv=3, L=30, model=O.DEEPWALK, deterministic=False, seed=7)
    gh.generate_initial_random_walks()
    gd.generate_initial_random_walks()
    ref.generate()
    dout = torch.full((gd.number_of_walks,), -1, dtype=torch.int32, device="cuda:0")
    for s, ins in ((1, True), (2, False)):
        b = O.generate_batch_of_edges(1000, 1 << 13, s, False, False)
        fl = O.REMOVE_DUPS | O.APPLY_WALK_UPDATES
        ah = (gh.insert_edges_batch if ins else gh.delete_edges_batch)(b, remove_dups=True)
        ad = (gd.insert_edges_batch if ins else gd.delete_edges_batch)(b, remove_dups=True, out=dout)
        ar = ref.update(ins, b, fl)
        assert ad.is_cuda and len(ad) == len(ah) > 0
        assert np.array_equal(ad.cpu().numpy().view(np.uint32), ah)
        np.testing.assert_array_equal(ah, ar)
    assert np.array_equal(gd.walks(), ref.walks())
    mem = gd.memory_footprint(verbose=False)
    assert mem["walks_bytes"] >= gd.number_of_walks * 30 * 4 and mem["csr_bytes"] >= gd.number_of_edges() * 4
    gh.destroy()
    gd.destroy()


# (WHARF_N2V_REWALK, WHARF_NO_ROW_SLACK, WHARF_POOL_NO_HEADROOM, neighbour filter, WHARF_NO_MEMO,
#  WHARF_NO_CHUNKED_SCAN, node2vec re-walk start-state table: on / off / 2 buckets, WHARF_NO_PREINIT,
#  WHARF_NT_ROWS: chunked scans with non-temporal or plain row loads)
# park/*: the node2vec re-walk by passes (k_rewalk_park + k_park_init), parking until no walker is
# left (WHARF_PARK_TAIL=0) or finishing a short list with in-wave inits (the default tail)
PATHS = {"sorted/slack": ("sorted", "0", "0", "on", "1", "0", "on", "0", "1"),
         "park/slack": ("park", "0", "0", "on", "1", "0", "on", "1", "1"),
         "sorted/move-lazy": ("sorted", "1", "0", "on", "1", "0", "on", "1", "0"),
         # round 3's faulted combination: move-lazy with the list sorted by rewalk point over all
         # blocks (WHARF_N2V_LIST_ORDER=global; waves of entries from many blocks)
         "sorted/global-move": ("sorted", "1", "0", "on", "1", "0", "on", "1", "0"),
         "block/slack": ("block", "0", "0", "on", "0", "0", "on", "0", "1"),
         "block/move-lazy": ("block", "1", "0", "noslack", "1", "0", "tiny", "1", "0"),
         "park/repack-tail": ("park", "1", "1", "off", "0", "1", "tiny", "0", "0"),
         "flat/move": ("flat", "1", "0", "noslack", "0", "0", "off", "0", "0"),
         "sorted/repack": ("sorted", "1", "1", "off", "0", "1", "tiny", "0", "1"),
         "flat/slack-repack": ("flat", "0", "1", "on", "1", "1", "on", "0", "0"),
         "sorted/lazy-inits": ("sorted", "0", "0", "on", "0", "0", "on", "1", "1"),
         "sorted/plain-rows": ("sorted", "0", "0", "on", "0", "0", "on", "1", "0")}


@pytest.mark.parametrize("rows", ["slack", "repack", "compact"])
@pytest.mark.parametrize("rec", ["wide", "compact", "compact-escape"])
@pytest.mark.parametrize("mode", ["det", "deepwalk"])
def test_edge_record_layouts(W, monkeypatch, rows, rec, mode):
    """DeepWalk and deterministic handles keep 8-B edge records when the ids and slot offsets fit
    (RecFmt: v | off << vb | deg << (vb + ob), a degree of 2^db - 1 or more read from deg[v]); the
    16-B layout (WHARF_COMPACT_REC=0) and the compact one with a 4-bit degree field (every row of
    degree >= 15 takes the escape) give the oracle's corpus, affected ids, counters and CSR through a
    stream of RMAT batches, across pool repacks (records rebuilt for the new pool) and in-place
    compactions; the records take 8 B per pool slot instead of 16."""
    if rec == "wide":
        monkeypatch.setenv("WHARF_COMPACT_REC", "0")
    if rec == "compact-escape":
        monkeypatch.setenv("WHARF_COMPACT_DEG_BITS", "4")
    if rows == "repack":
        monkeypatch.setenv("WHARF_POOL_NO_HEADROOM", "1")
    if rows == "compact":
        monkeypatch.setenv("WHARF_REPACK_MEM_CAP", "1")
        monkeypatch.setenv("WHARF_NO_ROW_SLACK", "1")
        monkeypatch.setenv("WHARF_POOL_HEADROOM", "30000")
    n = 1 << 12
    off, adj = O.csr_from_edges(n, O.generate_batch_of_edges(30000, 2 * n, 47, False, False))
    kw = dict(deterministic=True) if mode == "det" else dict(deterministic=False, seed=13, model=0)
    batches = []
    for b in range(3):
        e = O.generate_batch_of_edges(600, n, 50 + b, False, False)
        batches += [(True, e, O.REMOVE_DUPS | O.APPLY_WALK_UPDATES), (False, e, O.REMOVE_DUPS | O.APPLY_WALK_UPDATES)]
    batches.append((True, O.generate_batch_of_edges(900, n, 60, False, False), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES))
    batches.append((True, O.generate_batch_of_edges(200, n, 61, False, True), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES))
    g = W.WharfMH.from_csr(off, adj, config=W.WharfConfig(walks_per_vertex=3, walk_length=24, **kw))
    cap = g.stats()["pool_capacity"]
    rec_bytes = g.memory_footprint(verbose=False)["records_bytes"] - 16 * n
    assert rec_bytes == (16 if rec == "wide" else 8) * cap
    g.destroy()
    _compare_stream(W, off, adj, batches, wpv=3, L=24, **kw)


@pytest.mark.parametrize("path", list(PATHS))
@pytest.mark.parametrize("mode", ["det", "deepwalk", "node2vec"])
def test_rewalk_and_update_paths(W, monkeypatch, path, mode):
    """Every re-walk kernel and every CSR-update path reproduces the oracle's
    corpus, counters, affected ids and CSR.  Re-walk: the interleaved sweep
    (DeepWalk, deterministic); for node2vec the planned, sorted re-walk list
    swept in lock step (k_rewalk_sorted) or by lanes at their own pace
    (WHARF_N2V_REWALK=flat, k_rewalk_list).  CSR update (slack rows): rows
    merged in place within their slack, rows without slack that move to the
    pool's end on every insert (WHARF_NO_ROW_SLACK=1), and a pool without
    headroom that is repacked whenever a row moves (WHARF_POOL_NO_HEADROOM=1,
    node2vec anchors carried along).  node2vec anchor inits with the per-row
    neighbour filters (re-filled per source row, or with no pool headroom
    re-built whole whenever a row outgrows its words) and without them.
    Deterministic re-walks by suffix table (k_rewalk_chunked copy) and by
    walking every suffix (WHARF_NO_MEMO=1, k_rewalk_sweep).  Rewalk points
    alone (apply_walk_updates = false): the chunked scan, or with
    WHARF_NO_CHUNKED_SCAN=1 the sweep kernels in scan-only mode.  node2vec
    re-walk starts find their state's anchor entry in the per-batch start-state
    table, by the binary search in prev's row (WHARF_NO_START_TABLE=1), or
    mostly by the search after a 2-bucket table fills up.  The anchors a batch
    invalidates are computed ahead of the node2vec re-walk (k_anchor_preinit,
    into the edge entries and the start-state table) or lazily by the walkers
    (WHARF_NO_PREINIT=1).  The chunked scans run with non-temporal and with
    plain walk-matrix row loads (WHARF_NT_ROWS; the host picks per batch)."""
    n2v_list, no_slack, no_headroom, filt, no_memo, no_chunked, stab, no_pre, nt_rows = PATHS[path]
    monkeypatch.setenv("WHARF_NT_ROWS", nt_rows)
    monkeypatch.setenv("WHARF_PARK_TAIL", "0" if path == "park/slack" else "8192")
    # rewalk points alone: k_rewalk_scan_lean (default); k_rewalk_scan_big (round 2), or with the
    # 16-KiB filter k_rewalk_chunked<false>.  Every filter bit set on two paths (every position a
    # positive: the exact checks and the lean scan's false-positive fallback decide)
    monkeypatch.setenv("WHARF_SCAN_SMALL_BLOOM", "1" if path == "sorted/plain-rows" else "0")
    monkeypatch.setenv("WHARF_SCAN_KERNEL", "big" if path in ("flat/move", "block/move-lazy") else "lean")
    monkeypatch.setenv("WHARF_BLOOM_SATURATE", "1" if path in ("sorted/lazy-inits", "block/slack") else "0")
    # deterministic copy: positives settled by the source index (default) or by the bitmap word first
    monkeypatch.setenv("WHARF_COPY_BITMAP", "1" if path in ("flat/move", "sorted/repack") else "0")
    # node2vec sorted re-walk: a wave's entries in column order (default) or in list order
    monkeypatch.setenv("WHARF_N2V_LANE_SORT", "0" if path in ("sorted/plain-rows", "sorted/repack") else "1")
    # node2vec WEIGHT inits of the re-walk: return-first (default: a step settled by any non-return
    # anchor reads only its proposals' targets) or always the full init
    monkeypatch.setenv("WHARF_RET_FIRST", "0" if path in ("sorted/plain-rows", "flat/slack-repack") else "1")
    # node2vec anchor entries of the sources' rows carried through the merge, the ones a changed edge can
    # affect reset (default, undirected graphs; the last, directed batch turns it off), or all reset
    monkeypatch.setenv("WHARF_ANCHOR_CARRY", "0" if path in ("flat/move", "block/move-lazy") else "1")
    # node2vec plan (rewalk points + the binned re-walk list): on the lean scan (default) or k_rewalk_plan
    monkeypatch.setenv("WHARF_PLAN_KERNEL", "chunked" if path in ("flat/move", "sorted/plain-rows", "park/repack-tail")
                       else "lean")
    # the lean plan as the per-wave scan + a binning pass over its points (default) or fused in one kernel
    monkeypatch.setenv("WHARF_PLAN_SPLIT", "0" if path in ("sorted/slack", "block/slack", "sorted/global-move") else "1")
    # deterministic suffix copy: the 32-KiB filter folded from the 64-KiB one (default) or the 16-KiB one
    monkeypatch.setenv("WHARF_COPY_SMALL_BLOOM", "1" if path == "sorted/plain-rows" else "0")
    monkeypatch.setenv("WHARF_NO_PREINIT", no_pre)
    monkeypatch.setenv("WHARF_NO_START_TABLE", "1" if stab == "off" else "0")
    monkeypatch.setenv("WHARF_START_TABLE_BUCKETS", "2" if stab == "tiny" else "0")
    monkeypatch.setenv("WHARF_NO_MEMO", no_memo)
    monkeypatch.setenv("WHARF_NO_CHUNKED_SCAN", no_chunked)
    monkeypatch.setenv("WHARF_NO_NEIGHBOUR_FILTER", "1" if filt == "off" else "0")
    monkeypatch.setenv("WHARF_FILTER_NO_SLACK", "1" if filt == "noslack" else "0")
    monkeypatch.setenv("WHARF_N2V_REWALK", n2v_list)
    monkeypatch.setenv("WHARF_N2V_LIST_ORDER", "global" if path == "sorted/global-move" else "block")
    monkeypatch.setenv("WHARF_NO_ROW_SLACK", no_slack)
    monkeypatch.setenv("WHARF_POOL_NO_HEADROOM", no_headroom)
    # node2vec plan: the re-walk list binned per 256-walk block (default) or per 1024-walk workgroup
    monkeypatch.setenv("WHARF_N2V_PLAN_GROUP", "1" if path in ("sorted/lazy-inits", "park/slack", "sorted/move-lazy")
                       else "0")
    # in-edge records of the sources: the reverse-slot index (default on undirected graphs; the last,
    # directed batch drops it) or the streaming scan of the pool
    monkeypatch.setenv("WHARF_REV", "0" if path in ("flat/move", "sorted/plain-rows", "block/slack") else "1")
    base = O.generate_batch_of_edges(50000, 1 << 13, 6, False, False)
    off, adj = O.csr_from_edges(1 << 12, base)
    batches = [(True, O.generate_batch_of_edges(800, 1 << 12, 11, False, False), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES),
               (False, O.generate_batch_of_edges(600, 1 << 12, 12, False, False), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES),
               (True, O.generate_batch_of_edges(500, 1 << 12, 14, False, False), O.REMOVE_DUPS),   # rewalk points only
               (True, O.generate_batch_of_edges(40, 1 << 12, 13, False, True), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES)]
    kw = dict(deterministic=True) if mode == "det" else dict(
        deterministic=False, seed=99, model=1 if mode == "node2vec" else 0, paramP=0.5, paramQ=2.0)
    _compare_stream(W, off, adj, batches, wpv=3, L=40, **kw)


@pytest.mark.parametrize("mode", ["det", "node2vec"])
def test_release_caches_drops_the_reverse_index(W, monkeypatch, mode):
    """wharf_release_caches (a caller's allocation out of device memory, e.g. bench.py's gather
    buffer): the reverse-slot index is freed (csr_bytes falls by >= 4 B per edge), later updates scan
    the pool for in-edges, and the corpus, affected ids and CSR stay the oracle's; a second call
    frees nothing."""
    monkeypatch.setenv("WHARF_REV", "1")
    n = 1 << 11
    off, adj = O.csr_from_edges(n, O.generate_batch_of_edges(20000, 2 * n, 43, False, False))
    kw = dict(deterministic=True) if mode == "det" else dict(
        deterministic=False, seed=5, model=1, paramP=0.5, paramQ=2.0)
    cfg = W.WharfConfig(walks_per_vertex=2, walk_length=24, **kw)
    g = W.WharfMH.from_csr(off, adj, config=cfg)
    ref = O.Engine(off, adj, wpv=2, L=24, model=cfg.model, p=cfg.paramP, q=cfg.paramQ, init=cfg.sampler_init,
                   deterministic=cfg.deterministic, seed=cfg.seed)
    g.generate_initial_random_walks()
    ref.generate()
    e = O.generate_batch_of_edges(300, n, 90, False, False)
    assert np.array_equal(g.insert_edges_batch(e, remove_dups=True), ref.insert_edges_batch(e))
    assert g.stats()["last_in_edge_mode"] == 1
    held = g.memory_footprint(verbose=False)["csr_bytes"]
    freed = g.release_caches()
    assert freed >= 4 * g.number_of_edges()
    assert g.memory_footprint(verbose=False)["csr_bytes"] <= held - 4 * g.number_of_edges()
    assert g.release_caches() == 0
    for ins in (False, True):
        e = O.generate_batch_of_edges(300, n, 91, False, False)
        ga = (g.insert_edges_batch if ins else g.delete_edges_batch)(e, remove_dups=True)
        assert np.array_equal(ga, ref.insert_edges_batch(e) if ins else ref.delete_edges_batch(e))
        assert np.array_equal(g.walks(), ref.walks())
        assert g.stats()["last_in_edge_mode"] == 0 and g.stats()["rev_fallbacks"] == 0
    g.generate_initial_random_walks()   # not rebuilt lazily after a release
    ref.generate()
    assert np.array_equal(g.walks(), ref.walks())
    assert g.memory_footprint(verbose=False)["csr_bytes"] <= held - 4 * g.number_of_edges()
    o2, a2 = g.flatten_graph()
    o3, a3 = ref.csr()
    assert np.array_equal(o2, o3) and np.array_equal(a2, a3)
    g.destroy()


@pytest.mark.parametrize("rows", ["slack", "slack-lazy", "move", "repack", "compact"])
@pytest.mark.parametrize("mode", ["det", "deepwalk", "node2vec"])
def test_reverse_slot_index(W, monkeypatch, rows, mode):
    """The in-edge records of a batch's sources patched through the reverse-slot
    index (k_patch_rev: rev[e] = the slot of the reverse edge, carried through
    the merge, searched for edges between sources and new edges, rebuilt after a
    repack or compaction) instead of the streaming scan: over a stream of
    undirected insert/delete batches (RMAT hubs: many edges between sources) the
    corpus, counters, affected ids and CSR stay the oracle's.  The index is
    allocated (4 B per pool slot in csr_bytes) while the graph is undirected and
    dropped by the first directed batch, which the scan then serves."""
    rev_on = "2" if rows == "slack-lazy" else "1"   # 2: built at the first generation, not at creation
    monkeypatch.setenv("WHARF_REV", rev_on)
    if rows == "move":
        monkeypatch.setenv("WHARF_NO_ROW_SLACK", "1")
    if rows == "repack":
        monkeypatch.setenv("WHARF_POOL_NO_HEADROOM", "1")
    if rows == "compact":   # no room for a second pool: in-place compactions
        monkeypatch.setenv("WHARF_REPACK_MEM_CAP", "1")
        monkeypatch.setenv("WHARF_NO_ROW_SLACK", "1")
        monkeypatch.setenv("WHARF_POOL_HEADROOM", "45000")
    n = 1 << 12
    base = O.generate_batch_of_edges(40000, 2 * n, 41, False, False)
    off, adj = O.csr_from_edges(n, base)
    kw = dict(deterministic=True) if mode == "det" else dict(
        deterministic=False, seed=31, model=1 if mode == "node2vec" else 0, paramP=0.5, paramQ=2.0)
    cfg = W.WharfConfig(walks_per_vertex=3, walk_length=30, **kw)
    g = W.WharfMH.from_csr(off, adj, config=cfg)
    ref = O.Engine(off, adj, wpv=3, L=30, model=cfg.model, p=cfg.paramP, q=cfg.paramQ, init=cfg.sampler_init,
                   deterministic=cfg.deterministic, seed=cfg.seed)
    monkeypatch.setenv("WHARF_REV", "0")
    g0 = W.WharfMH.from_csr(off, adj, config=cfg)
    no_rev = g0.memory_footprint(verbose=False)["csr_bytes"]
    g0.destroy()
    monkeypatch.setenv("WHARF_REV", rev_on)
    g.generate_initial_random_walks()
    assert g.memory_footprint(verbose=False)["csr_bytes"] >= no_rev + 4 * g.number_of_edges()
    ref.generate()
    assert np.array_equal(g.walks(), ref.walks())
    stream = []
    for b in range(4):   # throughput-latency.cpp:126,135: insert batch b, delete it again
        e = O.generate_batch_of_edges(700, n, 60 + b, False, False)
        stream += [(True, e), (False, e)]
    stream.append((True, O.generate_batch_of_edges(900, n, 70, False, False)))
    used = 0
    for ins, e in stream:
        rp0 = g.stats()["repacks"]
        ga = (g.insert_edges_batch if ins else g.delete_edges_batch)(e, remove_dups=True)
        ra = ref.insert_edges_batch(e) if ins else ref.delete_edges_batch(e)
        assert np.array_equal(ga, ra)
        assert np.array_equal(g.walks(), ref.walks())
        st = g.stats()
        assert st["steps"] == ref.steps
        # the index served this batch's in-edge records unless the batch repacked or compacted the pool
        # (every row moved: scan, then rebuild); it never missed (a miss drops it and scans)
        assert st["rev_fallbacks"] == 0
        assert st["last_in_edge_mode"] == (0 if st["repacks"] != rp0 else 1), (rows, st["repacks"], rp0)
        used += st["last_in_edge_mode"]
    if rows in ("slack", "slack-lazy"):   # rows merged in place: the index serves the batches
        assert used >= len(stream) // 2
    o2, a2 = g.flatten_graph()
    o3, a3 = ref.csr()
    assert np.array_equal(o2, o3) and np.array_equal(a2, a3)
    # a directed batch: the graph is no longer undirected, the index is dropped and the scan takes over
    held = g.memory_footprint(verbose=False)["csr_bytes"]
    d = O.generate_batch_of_edges(300, n, 80, False, True)
    assert np.array_equal(g.insert_edges_batch(d, remove_dups=True), ref.insert_edges_batch(d))
    assert np.array_equal(g.walks(), ref.walks())
    assert g.stats()["last_in_edge_mode"] == 0
    assert g.memory_footprint(verbose=False)["csr_bytes"] <= held - 4 * g.number_of_edges()
    e = O.generate_batch_of_edges(500, n, 81, False, False)
    assert np.array_equal(g.insert_edges_batch(e, remove_dups=True), ref.insert_edges_batch(e))
    assert np.array_equal(g.walks(), ref.walks())
    assert g.stats()["last_in_edge_mode"] == 0 and g.stats()["rev_fallbacks"] == 0
    g.destroy()


@pytest.mark.parametrize("rows", ["slack", "move", "repack"])   # rows merged in place / moved / pool repacked
@pytest.mark.parametrize("init", [1, 2])                        # BURNIN, WEIGHT: inits that read prev's row
def test_node2vec_anchor_reset_with_prev_row(W, monkeypatch, rows, init):
    """The anchor of state (cur=c, prev=s) is cached in slot s->c of s's row.
    Directed batches make s a source while its targets are not: s's rebuilt
    row starts with empty entries, so (c, s) is re-initialised against s's new
    row with the same Philox proposals (c's row epoch is unchanged) — the
    shard-invariant rule of DESIGN.md §4 (the reference keeps c's sampler,
    initialised against s's row at the first visit).  Exercised on all three
    row-update paths, bit-exact against the oracle, which restates the same rule."""
    monkeypatch.setenv("WHARF_NO_ROW_SLACK", "0" if rows == "slack" else "1")
    monkeypatch.setenv("WHARF_POOL_NO_HEADROOM", "1" if rows == "repack" else "0")
    base = O.generate_batch_of_edges(30000, 1 << 12, 21, False, False)
    off, adj = O.csr_from_edges(1 << 11, base)
    R, A = O.REMOVE_DUPS, O.APPLY_WALK_UPDATES
    batches = [(True, O.generate_batch_of_edges(400, 1 << 11, 31, False, True), R | A),
               (False, O.generate_batch_of_edges(400, 1 << 11, 31, False, True), R | A),
               (True, O.generate_batch_of_edges(300, 1 << 11, 32, False, True), R | A),
               (False, O.generate_batch_of_edges(900, 1 << 11, 33, False, False), R | A)]
    _compare_stream(W, off, adj, batches, wpv=4, L=30, model=1, paramP=0.5, paramQ=2.0, sampler_init=init,
                    deterministic=False, seed=4321)


@pytest.mark.parametrize("rows", ["slack", "repack"])
def test_hub_row_cut_down_then_regrown(W, monkeypatch, rows):
    """a hub row cut down by deletions keeps the neighbour filter its
    old degree sized (deletions never shrink it), so after a repack recaps the row
    the filter can hold more words than the row's chunks cover; the refill clears
    every word of it.  A hub loses most of its edges, the pool is repacked
    (WHARF_POOL_NO_HEADROOM=1) or the row merged in its slack, then the hub gains
    edges again: node2vec MH corpus, counters, affected ids and CSR stay the
    oracle's (the filter is exact for negatives either way; stale bits would only
    cost extra edge-hash probes, which the counts below do not see)."""
    monkeypatch.setenv("WHARF_POOL_NO_HEADROOM", "1" if rows == "repack" else "0")
    n = 1 << 11
    base = O.generate_batch_of_edges(30000, 2 * n, 23, False, False)
    off, adj = O.csr_from_edges(n, base)
    deg = np.diff(off.astype(np.int64))
    hub = int(np.argmax(deg))
    nbrs = adj[off[hub]:off[hub + 1]].astype(np.uint32)
    cut = nbrs[: (len(nbrs) * 7) // 8]                        # most of the hub's row, both directions
    cut_pairs = np.concatenate([np.stack([np.full_like(cut, hub), cut], 1), np.stack([cut, np.full_like(cut, hub)], 1)])
    back = cut[: len(cut) // 3]
    back_pairs = np.concatenate([np.stack([np.full_like(back, hub), back], 1), np.stack([back, np.full_like(back, hub)], 1)])
    R, A = O.REMOVE_DUPS, O.APPLY_WALK_UPDATES
    batches = [(False, cut_pairs.astype(np.uint32), R | A),
               (True, O.generate_batch_of_edges(300, n, 41, False, False), R | A),   # rows move, the pool repacks
               (True, back_pairs.astype(np.uint32), R | A),
               (True, O.generate_batch_of_edges(300, n, 42, False, False), R | A)]
    assert len(nbrs) > 100, len(nbrs)
    _compare_stream(W, off, adj, batches, wpv=3, L=30, model=1, paramP=0.5, paramQ=2.0, sampler_init=2,
                    deterministic=False, seed=99)


@pytest.mark.parametrize("mode", ["det", "node2vec"])
def test_pool_compaction_without_room_for_a_second_pool(W, monkeypatch, mode):
    """When the pool runs out of headroom and the device cannot hold a second
    pool (WHARF_REPACK_MEM_CAP: as if only 1 byte were free), the repack falls
    back to the in-place compaction: rows keep their capacities and close up the
    dead slots that moved rows left (node2vec anchors carried along).  Rows
    without slack move on every growing insert (WHARF_NO_ROW_SLACK=1) and the
    headroom (22000 slots) holds one batch's moved rows but not two (hub rows:
    11-19 k slots per batch), so most batches compact first; corpus,
    counters, affected ids and CSR stay the oracle's throughout."""
    monkeypatch.setenv("WHARF_REPACK_MEM_CAP", "1")
    monkeypatch.setenv("WHARF_NO_ROW_SLACK", "1")
    monkeypatch.setenv("WHARF_POOL_HEADROOM", "22000")
    base = O.generate_batch_of_edges(30000, 1 << 12, 17, False, False)
    off, adj = O.csr_from_edges(1 << 11, base)
    kw = dict(deterministic=True) if mode == "det" else dict(deterministic=False, seed=77, model=1, paramP=0.5,
                                                              paramQ=2.0)
    cfg = W.WharfConfig(walks_per_vertex=3, walk_length=30, **kw)
    g = W.WharfMH.from_csr(off, adj, config=cfg)
    ref = O.Engine(off, adj, wpv=3, L=30, model=cfg.model, p=cfg.paramP, q=cfg.paramQ, init=cfg.sampler_init,
                   deterministic=cfg.deterministic, seed=cfg.seed)
    g.generate_initial_random_walks()
    ref.generate()
    dead_seen = 0
    for i in range(8):
        ins = i % 3 != 2
        b = O.generate_batch_of_edges(300, 1 << 11, 300 + i, False, i % 2 == 1)
        aff = (g.insert_edges_batch if ins else g.delete_edges_batch)(b, remove_dups=True)
        np.testing.assert_array_equal(aff, ref.update(ins, b, O.REMOVE_DUPS | O.APPLY_WALK_UPDATES))
        np.testing.assert_array_equal(g.walks(), ref.walks())
        o2, a2 = g.flatten_graph()
        o3, a3 = ref.csr()
        np.testing.assert_array_equal(o2, o3)
        np.testing.assert_array_equal(a2, a3)
        st = g.stats()
        assert st["steps"] == ref.steps and st["accepts"] == ref.accepts
        dead_seen = max(dead_seen, st["dead_slots"])
        assert st["pool_slots"] <= st["pool_capacity"]
    assert g.stats()["repacks"] >= 1 and dead_seen > 0
    g.destroy()


def test_pool_exhausted_leaves_the_handle_unchanged(W, monkeypatch):
    """No headroom, no row slack and no memory for a second pool: a growing insert
    cannot be placed even after the compaction.  It fails with WHARF_E_NOMEM
    before anything is applied — graph, walks, the update epoch and the sources'
    sampler epochs (the MH draws of later batches) stay as they were — and the
    handle goes on: a delete batch afterwards equals the oracle's, which never
    saw the failed insert."""
    monkeypatch.setenv("WHARF_REPACK_MEM_CAP", "1")
    monkeypatch.setenv("WHARF_NO_ROW_SLACK", "1")
    monkeypatch.setenv("WHARF_POOL_NO_HEADROOM", "1")
    base = O.generate_batch_of_edges(30000, 1 << 12, 19, False, False)
    off, adj = O.csr_from_edges(1 << 11, base)
    cfg = W.WharfConfig(walks_per_vertex=3, walk_length=30, deterministic=False, seed=5, model=1, paramP=0.5,
                        paramQ=2.0)
    g = W.WharfMH.from_csr(off, adj, config=cfg)
    ref = O.Engine(off, adj, wpv=3, L=30, model=1, p=0.5, q=2.0, init=cfg.sampler_init, deterministic=False, seed=5)
    g.generate_initial_random_walks()
    ref.generate()
    w0 = g.walks()
    ins = O.generate_batch_of_edges(500, 1 << 11, 41, False, False)
    with pytest.raises(RuntimeError, match=r"\(-3\).*slot pool exhausted"):
        g.insert_edges_batch(ins, remove_dups=True)
    np.testing.assert_array_equal(g.walks(), w0)
    o2, a2 = g.flatten_graph()
    np.testing.assert_array_equal(o2, off)
    np.testing.assert_array_equal(a2, adj)
    d = O.generate_batch_of_edges(800, 1 << 11, 42, False, False)
    aff = g.delete_edges_batch(d, remove_dups=True)
    np.testing.assert_array_equal(aff, ref.update(False, d, O.REMOVE_DUPS | O.APPLY_WALK_UPDATES))
    np.testing.assert_array_equal(g.walks(), ref.walks())
    assert g.stats()["accepts"] == ref.accepts
    g.destroy()


def test_walk_readout_snapshot_follows_every_change(W, monkeypatch):
    """walk() / vertex_at_walk() read a pinned host snapshot of the walk matrix
    (chunks of 64 Ki walks, taken on first use); every change to the walks —
    generation, an update with its re-walk, batch_walk_update, destroy_index,
    set_shard — invalidates it.  After each, every walk read through the
    snapshot equals the exported corpus and the per-call device path
    (WHARF_WALK_NO_SNAPSHOT=1), text included."""
    base = O.generate_batch_of_edges(60000, 1 << 17, 4, False, False)
    off, adj = O.csr_from_edges(1 << 16, base)          # 2 snapshot chunks per round: several chunks in play
    cfg = W.WharfConfig(walks_per_vertex=2, walk_length=12, model=W.DEEPWALK, deterministic=False, seed=3)
    g = W.WharfMH.from_csr(off, adj, config=cfg)
    rng = np.random.default_rng(5)

    def check():
        w = g.walks()
        ids = rng.choice(g.number_of_walks, 300, replace=False)
        for i in ids:
            row = w[i][w[i] != W.SENTINEL]
            assert np.array_equal(g.walk_vertices(int(i)), row)
            assert g.walk(int(i)) == O.walk_string(w[i])
            assert g.vertex_at_walk(int(i), 0) == int(w[i][0])
        monkeypatch.setenv("WHARF_WALK_NO_SNAPSHOT", "1")
        for i in ids[:50]:
            assert g.walk(int(i)) == O.walk_string(w[i])
        monkeypatch.setenv("WHARF_WALK_NO_SNAPSHOT", "0")

    g.generate_initial_random_walks()
    check()
    b = O.generate_batch_of_edges(3000, 1 << 16, 9, False, False)
    g.insert_edges_batch(b, remove_dups=True)
    check()
    g.batch_walk_update(b[:100, 0])
    check()
    g.delete_edges_batch(b, remove_dups=True)
    check()
    g.destroy_index()
    assert g.walk(5) == O.walk_string(g.walks()[5]) == ""   # no walks left: the snapshot was dropped too
    g.set_shard(1000, 30000)
    g.generate_initial_random_walks()
    w = g.walks()
    ids = g.walk_ids()
    for j in (0, 17, len(ids) - 1):
        assert g.walk(int(ids[j])) == O.walk_string(w[j])
    g.destroy()


def test_rewalk_list_entry_out_of_range_is_reported(W, monkeypatch):
    """A node2vec re-walk list entry outside the walks (planted between the plan
    and the consumer, WHARF_TEST_CORRUPT_LIST=1) is skipped, not dereferenced,
    and the update fails with WHARF_E_STATE (round 3's global-sort fault:
    k_rewalk_sorted read walks[p * W + li] for whatever the list held).  Every
    list consumer: the lock-step sweep, the flat list, the passes."""
    base = O.generate_batch_of_edges(20000, 1 << 12, 6, False, False)
    off, adj = O.csr_from_edges(1 << 11, base)
    b = O.generate_batch_of_edges(400, 1 << 11, 3, False, False)
    for kernel in ("sorted", "flat", "park"):
        monkeypatch.setenv("WHARF_N2V_REWALK", kernel)
        cfg = W.WharfConfig(walks_per_vertex=4, walk_length=20, model=W.NODE2VEC, paramP=0.5, paramQ=2.0,
                            deterministic=False, seed=5)
        g = W.WharfMH.from_csr(off, adj, config=cfg)
        g.generate_initial_random_walks()
        monkeypatch.setenv("WHARF_TEST_CORRUPT_LIST", "1")
        with pytest.raises(RuntimeError, match="outside the walks"):
            g.insert_edges_batch(b, remove_dups=True)
        monkeypatch.setenv("WHARF_TEST_CORRUPT_LIST", "0")
        # the walks are half re-walked: reads and updates fail loudly until a new generation
        with pytest.raises(RuntimeError, match="incomplete"):
            g.walk(0)
        with pytest.raises(RuntimeError, match="incomplete"):
            g.walks()
        with pytest.raises(RuntimeError, match="incomplete"):
            g.delete_edges_batch(b, remove_dups=True)
        g.generate_initial_random_walks()
        assert g.walk(0).startswith("0 ")
        g.delete_edges_batch(b, remove_dups=True)
        g.destroy()


def test_walk_rows_export_and_sparse_readout(W):
    """wharf_export_walk_rows[_device] (one bounded chunk of the corpus, the
    chunked corpus gather's source) equals the whole export on any row range;
    walk() of a few walks per 64 Ki-walk chunk reads them one by one (ADVICE r3:
    no chunk pulled for a sparse affected-walk readout), a dense readout takes the
    chunk, the affected walks of an update are staged together on the first read
    of one of them, and all agree with the export after every change."""
    import torch
    base = O.generate_batch_of_edges(60000, 1 << 18, 4, False, False)
    off, adj = O.csr_from_edges(1 << 17, base)
    cfg = W.WharfConfig(walks_per_vertex=2, walk_length=10, deterministic=True)
    g = W.WharfMH.from_csr(off, adj, config=cfg)
    g.generate_initial_random_walks()
    full = g.walks()
    Wn = g.number_of_walks
    for first, count in ((0, 1), (0, Wn), (65535, 2), (100_000, 61_000), (Wn - 3, 3), (Wn, 0)):
        assert np.array_equal(g.export_walk_rows(first, count), full[first:first + count])
        d = torch.empty((max(count, 1), 10), dtype=torch.int32, device="cuda:0")
        g.export_walk_rows(first, count, d)
        assert np.array_equal(d[:count].cpu().numpy().view(np.uint32), full[first:first + count])
    with pytest.raises(RuntimeError):
        g.export_walk_rows(Wn - 1, 2)
    for rnd in range(2):
        # sparse: a few walks of each chunk, and every position of one walk
        for c in range(0, Wn, 1 << 16):
            for i in (c, c + 7, min(c + 40_000, Wn - 1)):
                assert g.walk(i) == O.walk_string(full[i])
        assert [g.vertex_at_walk(70_001, p) for p in range(10)] == [int(x) for x in full[70_001]]
        # dense: one whole chunk walk by walk (the chunk is taken after 32 single reads)
        for i in range(1 << 16, 1 << 17):
            assert g.walk_vertices(i).tolist() == full[i][full[i] != W.SENTINEL].tolist()
        b = O.generate_batch_of_edges(2000, 1 << 17, 20 + rnd, False, False)
        aff = g.insert_edges_batch(b, remove_dups=True)
        full = g.walks()
        # the reference's incremental readout: walk(i) of the affected walks (staged together)
        for i in aff[::max(1, len(aff) // 3000)]:
            assert g.walk(int(i)) == O.walk_string(full[i])
    # an update whose walks are staged, then a read of an unaffected walk, then of affected ones
    b = O.generate_batch_of_edges(30, 1 << 17, 77, False, False)
    aff = g.insert_edges_batch(b, remove_dups=True)
    full = g.walks()
    other = int(np.setdiff1d(np.arange(Wn), aff)[5])
    assert g.walk(other) == O.walk_string(full[other])
    for i in aff:
        assert g.walk_vertices(int(i)).tolist() == full[i][full[i] != W.SENTINEL].tolist()
    g.destroy()


# ---------------------------------------------------------------------------
# MH mode
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("pq", [(0.5, 2.0), (4.0, 1.0), (2.0, 0.5)])   # BASELINE, reference default, q < 1
@pytest.mark.parametrize("init", [0, 1, 2])
def test_mh_node2vec_bit_exact_vs_oracle(W, init, pq):
    base = O.generate_batch_of_edges(40000, 1 << 12, 5, False, False)
    off, adj = O.csr_from_edges(1 << 11, base)
    batches = [(True, O.generate_batch_of_edges(2000, 1 << 11, 1, False, False), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES),
               (False, O.generate_batch_of_edges(1500, 1 << 11, 2, False, False), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES),
               (True, O.generate_batch_of_edges(300, 1 << 11, 3, False, True), O.REMOVE_DUPS | O.APPLY_WALK_UPDATES)]
    _compare_stream(W, off, adj, batches, wpv=4, L=40, model=1, paramP=pq[0], paramQ=pq[1], sampler_init=init,
                    deterministic=False, seed=1234 + init)


def test_mh_deepwalk_bit_exact_and_uniform(W):
    z = np.load(os.path.join(G, "wiki_csr.npz"))
    off, adj = z["off"], z["adj"]
    cfg = W.WharfConfig(walks_per_vertex=10, walk_length=80, model=W.DEEPWALK, deterministic=False, seed=42)
    g = W.WharfMH.from_csr(off, adj, config=cfg)
    g.generate_initial_random_walks()
    ref = O.Engine(off, adj, wpv=10, L=80, model=O.DEEPWALK, deterministic=False, seed=42)
    ref.generate()
    w = g.walks()
    np.testing.assert_array_equal(w, ref.walks())
    st = g.stats()
    assert st["accepts"] == st["steps"] == ref.steps      # DeepWalk weights are 1: every proposal accepted
    # uniform next-vertex per current vertex: chi-square over all vertices, like the reference's
    src = w[:, :-1].ravel()
    dst = w[:, 1:].ravel()
    keep = dst != W.SENTINEL
    src, dst = src[keep].astype(np.int64), dst[keep].astype(np.int64)
    pos = np.searchsorted(adj, dst)  # index within row not needed; count (src,dst)
    key = src * 4096 + dst
    uk, cnt = np.unique(key, return_counts=True)
    obs = dict(zip(uk.tolist(), cnt.tolist()))
    chi = dof = 0.0
    for v in range(len(off) - 1):
        d = int(off[v + 1] - off[v])
        if d < 2:
            continue
        o = np.array([obs.get(v * 4096 + int(x), 0) for x in adj[off[v]:off[v + 1]]], dtype=np.float64)
        if o.sum() < 5 * d:
            continue
        e = o.sum() / d
        chi += ((o - e) ** 2 / e).sum()
        dof += d - 1
    # chi2/dof ~ 1 +- sqrt(2/dof); reference run: 20992 / 20829
    assert abs(chi / dof - 1.0) < 6 * np.sqrt(2.0 / dof)
    del pos


_MATRIX = json.load(open(os.path.join(G, "golden.json")))["mh_matrix_reference"]


@pytest.mark.parametrize("cell", mh_stats.cells(_MATRIX), ids=lambda c: c[0])
def test_mh_matrix_vs_reference(W, cell):
    """Every (model, p, q, sampler init) cell of the reference's MH statistics
    (8 reference seeds per cell, `make_golden.py mh-matrix`): the HIP path over
    the same 8 seeds gives return / triangle / outward fractions within
    mh_stats.Z_TOL standard errors of the reference means, the standard error
    coming from the reference's own seed-to-seed sd
    (metropolis_hastings_sampler.h:69-122, node2vec.h:74-119)."""
    key, model, p, q, init = cell
    z = np.load(os.path.join(G, "wiki_csr.npz"))
    off, adj = z["off"], z["adj"]
    inits = {"random": 0, "burnin": 1, "weight": 2}
    ours = []
    for s in _MATRIX["seeds"]:
        cfg = W.WharfConfig(walks_per_vertex=_MATRIX["wpv"], walk_length=_MATRIX["L"],
                            model=W.NODE2VEC if model == "node2vec" else W.DEEPWALK, paramP=p, paramQ=q,
                            sampler_init=inits[init], deterministic=False, seed=s)
        g = W.WharfMH.from_csr(off, adj, config=cfg)
        g.generate_initial_random_walks()
        w = g.walks()
        if s == _MATRIX["seeds"][0]:      # and the corpus is the oracle's, bit for bit
            ref = O.Engine(off, adj, wpv=_MATRIX["wpv"], L=_MATRIX["L"], model=cfg.model, p=p, q=q,
                           init=inits[init], deterministic=False, seed=s)
            ref.generate()
            np.testing.assert_array_equal(w, ref.walks())
            assert g.stats()["accepts"] == ref.accepts
        ours.append(mh_stats.class_fractions(w, off, adj))
        g.destroy()
    bad = mh_stats.check_cell(_MATRIX[key], np.array(ours), key)
    assert not bad, bad


_STREAM = json.load(open(os.path.join(G, "golden.json")))["mh_stream_matrix_reference"]


@pytest.mark.parametrize("cell", mh_stats.stream_cells(_STREAM), ids=lambda c: c[0])
def test_mh_stream_vs_reference(W, cell):
    """MH re-walks through an insert and a delete batch (the reference's MH
    update path, wharfmh.h:439-923, sampler resets of batch sources): class
    fractions of the final corpus on the final graph against the reference's 8
    seeds (`mh_stream_matrix_reference`), for undirected RMAT batches on wiki and
    for the directed insert/delete pairs of one batch of the reference's driver
    (throughput-latency.cpp:121,126,135) on wiki without isolated vertices; the
    first seed also bit-exact against the oracle."""
    key, p, q, init = cell
    c = _STREAM["cells"][key]
    z = np.load(os.path.join(G, "wiki_csr.npz"))
    off, adj = mh_stats.stream_graph(c, z["off"], z["adj"])
    n = len(off) - 1
    inits = {"random": 0, "burnin": 1, "weight": 2}
    ours = []
    for i, s in enumerate(_STREAM["seeds"]):
        cfg = W.WharfConfig(walks_per_vertex=_STREAM["wpv"], walk_length=_STREAM["L"], model=W.NODE2VEC,
                            paramP=p, paramQ=q, sampler_init=inits[init], deterministic=False, seed=s)
        g = W.WharfMH.from_csr(off, adj, config=cfg)
        g.generate_initial_random_walks()
        batches = mh_stats.stream_batches(c, i, n, O.generate_batch_of_edges)
        for ins, b in batches:
            (g.insert_edges_batch if ins else g.delete_edges_batch)(b, remove_dups=True)
        o2, a2 = g.flatten_graph()
        w = g.walks()
        if i == 0:
            ref = O.Engine(off, adj, wpv=_STREAM["wpv"], L=_STREAM["L"], model=O.NODE2VEC, p=p, q=q,
                           init=inits[init], deterministic=False, seed=s)
            ref.generate()
            for ins, b in batches:
                ref.update(ins, b)
            np.testing.assert_array_equal(w, ref.walks())
        ours.append(mh_stats.class_fractions(w, o2, a2))
        g.destroy()
    bad = mh_stats.check_cell(c, np.array(ours), key)
    assert not bad, bad


# ---------------------------------------------------------------------------
# full-size properties (no oracle needed)
# ---------------------------------------------------------------------------
def test_large_rmat_properties(W):
    """Scale-20 RMAT, DeepWalk MH: every transition is an edge, walks start at
    wid % n, isolated starts stay length 1, steps = active walks * (L-1);
    a sample of walks is re-computed by the oracle bit for bit."""
    n = 1 << 20
    cfg = W.WharfConfig(walks_per_vertex=4, walk_length=80, model=W.DEEPWALK, deterministic=False, seed=7)
    g = W.WharfMH.from_rmat(n, 8_000_000, 2 * n, seed=2, config=cfg)
    off, adj = g.flatten_graph()
    deg = np.diff(off.astype(np.int64))
    g.generate_initial_random_walks()
    st = g.stats()
    active = int((deg > 0).sum()) * 4
    assert st["steps"] == active * 79 and st["accepts"] == st["steps"]
    w = g.walks(layout="position")
    Wn = w.shape[1]
    wid = np.arange(Wn, dtype=np.int64)
    assert (w[0] == wid % n).all()
    iso = deg[wid % n] == 0
    assert (w[1][iso] == W.SENTINEL).all() and (w[1][~iso] != W.SENTINEL).all()
    rng = np.random.default_rng(0)
    for p in rng.choice(79, 8, replace=False):
        cols = rng.choice(np.nonzero(~iso)[0], 20000, replace=False)
        u, v = w[p, cols].astype(np.int64), w[p + 1, cols].astype(np.int64)
        assert _has_edge(off, adj, u, v).all()
    ref = O.Engine(off, adj, wpv=4, L=80, model=O.DEEPWALK, deterministic=False, seed=7)
    ref.time_generate_range(123456, 123456 + 4096)
    rw = ref.walks()[123456:123456 + 4096]
    np.testing.assert_array_equal(w[:, 123456:123456 + 4096].T, rw)
    g.destroy()


def test_szudzik_device(W):
    x = np.array([0, 1, 65535, 123, 4000000000, 3999999999, 2**31 + 5], dtype=np.uint64)
    y = np.array([0, 7, 65535, 25, 3999999999, 4000000000, 17], dtype=np.uint64)
    z = W.szudzik64_pair(x, y)
    for a, b, c in zip(x, y, z):
        assert int(c) == O.szudzik64_pair(int(a), int(b))
    ux, uy = W.szudzik64_unpair(z)
    np.testing.assert_array_equal(ux, x)
    np.testing.assert_array_equal(uy, y)


@pytest.mark.parametrize("kind", ["ranges", "blocks"])
@pytest.mark.parametrize("mode", ["det", "mh_deepwalk", "mh_node2vec"])
def test_shards_reproduce_the_full_corpus(W, mode, kind):
    """Walks sharded by start-vertex range or by vertex blocks dealt round-robin
    (the multi-GPU layouts) are bit-identical to the single-handle corpus,
    through generation and an insert/delete pair: walks, walk ids, affected ids,
    walk() text, the inverted index of each shard's walks; block shards on a
    graph whose last block is short."""
    from dynamicgraphrepresentationlearning_amd.distributed import balanced_shards, block_shards, shard_walk_ids_of
    n = 1 << 12 if kind == "ranges" else 4000
    base = np.asarray(O.generate_batch_of_edges(60000, 2 * n, 8, False, False)).reshape(-1, 2)
    base = base[(base < n).all(axis=1)]   # (4000 vertices: the pairs among them)
    off, adj = O.csr_from_edges(n, base)
    deg = np.diff(off.astype(np.int64))
    kw = dict(walks_per_vertex=3, walk_length=30, seed=5, deterministic=(mode == "det"),
              model=W.NODE2VEC if mode == "mh_node2vec" else W.DEEPWALK, paramP=0.5, paramQ=2.0)
    full = W.WharfMH.from_csr(off, adj, config=W.WharfConfig(**kw))
    full.generate_initial_random_walks()
    b = O.generate_batch_of_edges(1500, n, 4, False, False)
    fw0 = full.walks()
    fa1 = full.insert_edges_batch(b, remove_dups=True).copy()
    fw1 = full.walks()
    fa2 = full.delete_edges_batch(b, remove_dups=True).copy()
    fw2 = full.walks()
    shards = balanced_shards(deg, 3) if kind == "ranges" else block_shards(n, 3, 6)
    seen = []
    for sh in shards:
        g = W.WharfMH.from_csr(off, adj, config=W.WharfConfig(**kw))
        g.apply_shard(sh)
        ids = shard_walk_ids_of(sh, n, 3)
        seen.append(ids)
        np.testing.assert_array_equal(g.walk_ids(), ids)
        g.generate_initial_random_walks()
        np.testing.assert_array_equal(g.walks(), fw0[ids])
        a1 = g.insert_edges_batch(b, remove_dups=True)
        np.testing.assert_array_equal(np.sort(a1), np.intersect1d(fa1, ids))
        np.testing.assert_array_equal(g.walks(), fw1[ids])
        a2 = g.delete_edges_batch(b, remove_dups=True)
        np.testing.assert_array_equal(np.sort(a2), np.intersect1d(fa2, ids))
        np.testing.assert_array_equal(g.walks(), fw2[ids])
        for i in (0, len(ids) // 2, len(ids) - 1):
            assert g.walk(int(ids[i])) == O.walk_string(fw2[ids[i]])
        with pytest.raises(RuntimeError):
            g.walk(int(np.setdiff1d(np.arange(3 * n), ids)[0]))   # not owned by this shard
        c, k, nx = g.inverted_index()
        keys = (ids[:, None] * 30 + np.arange(30)[None, :])[fw2[ids] != W.SENTINEL]
        assert int(c.sum()) == len(keys) and np.array_equal(np.sort(k), np.sort(keys.astype(np.uint64)))
        g.destroy()
    assert np.array_equal(np.sort(np.concatenate(seen)), np.arange(3 * n))
    full.destroy()


def test_set_shard_keeps_the_callers_config(W):
    """set_shard re-partitions one handle; a config shared with a later handle on a
    smaller graph (bench.py's stream graph) keeps its own shard fields."""
    cfg = W.WharfConfig(walks_per_vertex=2, walk_length=10)
    g = W.WharfMH.from_rmat(1 << 12, 30000, 1 << 13, seed=3, config=cfg)
    g.set_shard(100, 1 << 12)
    assert (cfg.shard_lo, cfg.shard_hi) == (0, 0)
    assert g.shard()[:2] == (100, 1 << 12)
    h = W.WharfMH.from_rmat(1 << 10, 5000, 1 << 11, seed=3, config=cfg)
    assert h.shard()[:2] == (0, 1 << 10)
    h.destroy()
    g.destroy()
