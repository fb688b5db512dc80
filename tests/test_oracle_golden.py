"""Pin the CPU oracle (oracle/wharf_oracle.c) to the reference's own outputs.

Every expected value here was produced by the reference implementation
(oracle/_ref/ref_harness built from /root/reference, tests/golden/make_golden.py).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")


def _kat():
    rows = [l.split() for l in open(os.path.join(G, "kat.txt"))]
    return rows


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def meta():
    return json.load(open(os.path.join(G, "golden.json")))


def test_random_lrand_drand_irand_kat():
    # utility::Random (utils/utility.h:152-223): arithmetic-shift seeding
    seen = 0
    for r in _kat():
        if r[0] == "random":
            seed = int(r[1])
            rng = O.Random(seed)
            assert [int(rng.s[0]), int(rng.s[1])] == [int(r[3]), int(r[4])]
            assert [rng.lrand() for _ in range(8)] == [int(x) for x in r[6:14]]
            seen += 1
        elif r[0] == "drand":
            rng = O.Random(int(r[1]))
            got = [rng.drand() for _ in range(4)]
            assert got == [float(x) for x in r[2:6]]
        elif r[0] == "irand":
            rng = O.Random(int(r[1]))
            mx = [1, 2, 3, 7, 80, 1000, 65537, 2147483647]
            assert [rng.irand(m) for m in mx] == [int(x) for x in r[2:10]]
    assert seen == 7


def test_survey_appendix_a_random_vectors():
    r = O.Random(0)
    assert [r.lrand() for _ in range(3)] == [10407335079877134008, 3962074050977524353, 12330921719341810270]
    r = O.Random(9)
    assert (int(r.s[0]), int(r.s[1])) == (903954156499315436, 4598867501830367842)


def test_hash_kat():
    for r in _kat():
        if r[0] == "hash64":
            assert O.hash64(int(r[1])) == int(r[2])
        elif r[0] == "hash32":
            assert O.hash32(int(r[1])) == int(r[2])


def test_szudzik_kat():
    # walks/pairings.h; tests/pairings.cpp:27-40,73-91
    kat = {tuple(r[:3]): r[3:] for r in _kat() if r[0].startswith("szudzik")}
    assert O.szudzik32_pair(65535, 65535) == int(kat[("szudzik32", "65535", "65535")][0]) == 4294967295
    assert O.szudzik32_pair(10, 3) == int(kat[("szudzik32", "10", "3")][0])
    assert O.szudzik32_pair(3, 10) == int(kat[("szudzik32", "3", "10")][0])
    assert O.szudzik32_unpair(4294967295) == (65535, 65535)
    t = O.szudzik32_pair(O.szudzik32_pair(123, 25), 200)
    assert t == 229643916 == int(kat[("szudzik32_triplet", "123", "25")][1])
    assert O.szudzik64_pair(4000000000, 3999999999) == int(kat[("szudzik64", "4000000000", "3999999999")][0])
    assert O.szudzik64_pair(3999999999, 4000000000) == int(kat[("szudzik64", "3999999999", "4000000000")][0])
    assert O.szudzik64_unpair(O.szudzik64_pair(123456789, 987654321)) == (123456789, 987654321)


def test_philox_random123_kat():
    # Random123 known-answer vectors for philox4x32_10
    assert O.philox4x32_10([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert O.philox4x32_10([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert O.philox4x32_10([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_rmat_batches_match_reference():
    z = np.load(os.path.join(G, "rmat_batches.npz"))
    assert z["b_8_64_0_1"].tolist() == [[0, 20], [1, 3], [3, 7], [4, 21], [8, 24], [22, 17], [24, 9]]
    for k in z.files:
        _, M, V, s, d = k.split("_")
        got = O.generate_batch_of_edges(int(M), int(V), int(s), False, bool(int(d)))
        np.testing.assert_array_equal(got, z[k], err_msg=k)


def test_six_vertex_corpus(meta):
    z = np.load(os.path.join(G, "six.npz"))
    e = O.Engine(z["off"], z["adj"], wpv=2, L=5)
    e.generate()
    w = e.walks()
    np.testing.assert_array_equal(w, z["walks"])
    # node2vec in deterministic mode produces the same corpus (wharfmh.h:304-309)
    np.testing.assert_array_equal(z["walks_node2vec"], z["walks"])
    c, k, nx = e.index()
    np.testing.assert_array_equal(c, z["index_counts"])
    np.testing.assert_array_equal(k, z["index_keys"])
    np.testing.assert_array_equal(nx, z["index_nexts"])
    assert O.walk_string(w[0]) == meta["six_walkstr"]["0"]
    assert O.walk_string(w[11]) == meta["six_walkstr"]["11"]


def _csr_from_batch_sources(z):
    return z["off_0"], z["adj_0"]


def test_rmat10_streaming_insert_delete():
    z = np.load(os.path.join(G, "rmat10.npz"))
    # base graph = generate_batch_of_edges(12800, 2048, 1, undirected) on n = 1024
    base = O.generate_batch_of_edges(12800, 2048, 1, False, False)
    off, adj = O.csr_from_edges(1024, base)
    np.testing.assert_array_equal(off, z["off_0"])
    np.testing.assert_array_equal(adj, z["adj_0"])
    e = O.Engine(off, adj, wpv=2, L=20)
    e.generate()
    np.testing.assert_array_equal(e.walks(), z["walks_gen"])
    c, k, nx = e.index()
    np.testing.assert_array_equal(c, z["index_counts_0"])
    np.testing.assert_array_equal(k, z["index_keys_0"])
    np.testing.assert_array_equal(nx, z["index_nexts_0"])
    steps = [("1_ins", True, "ins1", "1"), ("2_del", False, "del2", "2"), ("3_ins", True, "ins3", "3"),
             ("4_del", False, "del4", "4")]
    for tag, ins, wname, gtag in steps:
        aff = e.update(ins, z[f"batch_{tag}"])
        np.testing.assert_array_equal(aff, z[f"affected_{tag}"], err_msg=tag)
        o2, a2 = e.csr()
        np.testing.assert_array_equal(o2, z[f"off_{gtag}"], err_msg=tag)
        np.testing.assert_array_equal(a2, z[f"adj_{gtag}"], err_msg=tag)
        np.testing.assert_array_equal(e.walks(), z[f"walks_{wname}"], err_msg=tag)
        if f"index_counts_{gtag}" in z.files:
            c, k, nx = e.index()
            np.testing.assert_array_equal(c, z[f"index_counts_{gtag}"])
            np.testing.assert_array_equal(k, z[f"index_keys_{gtag}"])
            np.testing.assert_array_equal(nx, z[f"index_nexts_{gtag}"])
    # node2vec deterministic mode: identical corpus to DeepWalk
    np.testing.assert_array_equal(z["n2v_walks_gen"], z["walks_gen"])
    np.testing.assert_array_equal(z["n2v_walks_ins1"], z["walks_ins1"])
    np.testing.assert_array_equal(z["n2v_walks_del2"], z["walks_del2"])


def test_rmat10_directed_batches():
    z = np.load(os.path.join(G, "rmat10_directed.npz"))
    base = O.generate_batch_of_edges(12800, 2048, 1, False, False)
    off, adj = O.csr_from_edges(1024, base)
    e = O.Engine(off, adj, wpv=2, L=20)
    e.generate()
    np.testing.assert_array_equal(e.walks(), z["walks_gen"])
    b = O.generate_batch_of_edges(50, 1024, 0, False, True)
    np.testing.assert_array_equal(b, z["batch_ins"])
    np.testing.assert_array_equal(e.insert_edges_batch(b), z["affected_ins"])
    np.testing.assert_array_equal(e.walks(), z["walks_ins"])
    np.testing.assert_array_equal(e.delete_edges_batch(b), z["affected_del"])
    np.testing.assert_array_equal(e.walks(), z["walks_del"])


def test_wiki_full_corpus_and_updates(meta):
    z = np.load(os.path.join(G, "wiki_csr.npz"))
    wz = np.load(os.path.join(G, "wiki_golden.npz"))
    g = meta["wiki"]
    assert len(z["off"]) - 1 == 2405 and len(z["adj"]) == 23192
    e = O.Engine(z["off"], z["adj"], wpv=10, L=80)
    e.generate()
    w = e.walks()
    np.testing.assert_array_equal(w[:64], wz["first64_0_gen"])
    assert sha(w) == g["0_gen"]["sha256"]
    assert O.walk_string(w[12345]) != ""
    b = O.generate_batch_of_edges(5000, 2405, 0, False, False)
    np.testing.assert_array_equal(b, wz["batch_1_ins"])
    aff = e.insert_edges_batch(b)
    assert len(aff) == g["affected_1_ins"]["count"] and sha(aff) == g["affected_1_ins"]["sha256"]
    assert sha(e.walks()) == g["1_ins"]["sha256"]
    aff = e.delete_edges_batch(b)
    assert len(aff) == g["affected_2_del"]["count"] and sha(aff) == g["affected_2_del"]["sha256"]
    assert sha(e.walks()) == g["2_del"]["sha256"]
    assert O.walk_string(e.walks()[12345]) == g["walkstr_12345"]
