"""Pin the CPU oracle (oracle/) to the reference: golden fixtures made by the reference's
own code (tests/golden/make_golden.py), plus an independent scipy formulation of the
exact-distance hop sets. CPU only."""
import math
import os

import numpy as np
import pytest
import scipy.sparse as sp
from hypothesis import given, settings
from hypothesis import strategies as st

import blp_oracle as O
import coracle
from helpers import (B_FILES, GOLDEN, METHODS, SIM_CASES, U_FILES, assert_same_scores, bipartite_edges, dense_edges,
                     golden, load, read_edges)


@pytest.mark.parametrize("case", SIM_CASES)
def test_python_oracle_matches_reference_similarity(case):
    adj = O.load_edge_list(os.path.join(GOLDEN, case, "graph.txt"))
    ex = golden(case, "examples.json")
    for m, f, got in zip(METHODS, U_FILES, O.users(ex, adj, METHODS)):
        assert_same_scores(got, golden(case, f), m)
    for m, f, got in zip(METHODS, B_FILES, O.business(ex, adj, METHODS)):
        assert_same_scores(got, golden(case, f), m)


def _flat(ex):
    us, vs = [], []
    for u, inner in ex.items():
        for v in inner:
            us.append(u)
            vs.append(v)
    return us, vs


@pytest.mark.parametrize("case", SIM_CASES)
def test_c_oracle_matches_reference_similarity(case):
    a, b = read_edges(os.path.join(GOLDEN, case, "graph.txt"))
    ids, da, db = dense_edges(a, b)
    g = coracle.OracleGraph(len(ids), da, db)
    ex = golden(case, "examples.json")
    us, vs = _flat(ex)
    ui = np.array([int(u) for u in us])
    vi = np.array([int(v) for v in vs])
    ok = np.isin(ui, ids) & np.isin(vi, ids)
    x = np.searchsorted(ids, ui[ok])
    y = np.searchsorted(ids, vi[ok])
    ucn, ujac, uaa, _ = g.score_pairs(x, y, 7)
    bcn, bjac, _, _ = g.score_pairs(y, x, 3)
    ref = {k: golden(case, f) for k, f in zip(["ucn", "ujac", "uaa", "bcn", "bjac"],
                                              U_FILES + B_FILES[:2])}
    k = 0
    for i in range(len(us)):
        if not ok[i]:
            continue
        u, v = us[i], vs[i]
        assert ucn[k] == ref["ucn"][u][v]
        assert ujac[k] == ref["ujac"][u][v]
        assert math.isclose(uaa[k], ref["uaa"][u][v], rel_tol=1e-12)  # set-order sum vs exact
        assert bcn[k] == ref["bcn"][u][v]
        assert bjac[k] == ref["bjac"][u][v]
        k += 1


def test_b_adamic_reference_bug_is_reproduced():
    # similarity.py:102 never matches 'adamic_adar': only missing-node zeros are written
    for case in SIM_CASES:
        ex = golden(case, "examples.json")
        adj = O.load_edge_list(os.path.join(GOLDEN, case, "graph.txt"))
        exp = golden(case, "b_adamic.json")
        for u in exp:
            for v in exp[u]:
                assert exp[u][v] == 0 and not (int(u) in adj and int(v) in adj)
        got = O.business(ex, adj, ["adamic_adar"])[0]
        assert got == exp


@pytest.mark.parametrize("split", ["train", "test"])
def test_svd_reconstruction_matches_reference(split):
    d = os.path.join(GOLDEN, "bip", split)
    U = np.load(os.path.join(d, "svd_U.npy"))
    s = np.load(os.path.join(d, "svd_s.npy"))
    Vt = np.load(os.path.join(d, "svd_Vt.npy"))
    users = list(load(os.path.join(d, "user.json")).keys())
    bus = list(load(os.path.join(d, "business.json")).keys())
    row = {u: i for i, u in enumerate(users)}
    col = {b: i for i, b in enumerate(bus)}
    exp = load(os.path.join(d, "svd.json"))
    ex = load(os.path.join(d, "examples.json"))
    us, vs = _flat(ex)
    got = O.svd_pair_scores(U * s, Vt, [row[u] for u in us], [col[v] for v in vs])
    want = np.array([exp[u][v] for u, v in zip(us, vs)])
    np.testing.assert_array_equal(got, want)


def test_eval_matches_reference():
    d = os.path.join(GOLDEN, "bip", "test")
    ex = load(os.path.join(d, "examples.json"))
    ev = load(os.path.join(GOLDEN, "bip", "eval.json"))
    for method, res in ev.items():
        if "raises" in res:
            continue
        pred = load(os.path.join(d, method + ".json"))
        ys, ps = [], []
        for u in pred:
            for b in pred[u]:
                ys.append(ex[u][b])
                ps.append(pred[u][b])
        assert math.isclose(O.roc_auc(ys, ps), res["auc"], rel_tol=1e-12)
        assert "ROC Auc = {:.4f}".format(O.roc_auc(ys, ps)) == res["auc_line"]
        assert "Precision @20 = {:.4f}".format(O.precision_at(ex, pred, 20)) == res["precision_line"]


def test_hop3_candidates_match_reference():
    d = os.path.join(GOLDEN, "hop3")
    adj = O.load_edge_list(os.path.join(d, "graph.txt"))
    ex = load(os.path.join(d, "examples.json"))
    new = {tuple(map(int, l.split())) for l in open(os.path.join(d, "new_edges.txt"))}
    assert len(ex) > 10
    for u, inner in ex.items():
        cand = O.hop3_candidates(adj, int(u))
        assert {int(b) for b in inner} == cand  # negative_sample_rate=1.0 keeps every candidate
        for b, lab in inner.items():
            assert lab == (1 if (int(u), int(b)) in new else 0)
    # C oracle agrees
    a, b = read_edges(os.path.join(d, "graph.txt"))
    ids, da, db = dense_edges(a, b)
    g = coracle.OracleGraph(len(ids), da, db)
    users = [int(u) for u in ex]
    counts, members = g.hop3(np.searchsorted(ids, users))
    k = 0
    for u, c in zip(users, counts):
        assert set(ids[members[k:k + c]].tolist()) == {int(x) for x in ex[str(u)]}
        k += c


@pytest.mark.parametrize("case", ["bip/train", "general"])
def test_random_walks_match_reference(case):
    d = os.path.join(GOLDEN, case)
    a, b = read_edges(os.path.join(d, "graph.txt"))
    ex = load(os.path.join(d, "examples.json"))
    exp = load(os.path.join(d, "random_walks.json"))
    got = O.random_walk_scores(list(zip(a.tolist(), b.tolist())), ex)
    for u in exp:
        for v in exp[u]:
            assert math.isclose(got[u][v], exp[u][v], rel_tol=1e-9, abs_tol=1e-300)
    if case == "general":
        assert any(exp[u][v] > 0 for u in exp for v in exp[u])


def _scipy_scores(n, da, db, x, y):
    """Independent formulation: D2 = (A^2 > 0) minus distance <= 1; cn = (D2 @ A)[x, y]."""
    A = sp.coo_matrix((np.ones(2 * len(da)), (np.r_[da, db], np.r_[db, da])), shape=(n, n)).tocsr()
    A.data[:] = 1.0
    A.setdiag(0)
    A.eliminate_zeros()
    A.data[:] = 1.0
    A2 = (A @ A).tocsr()
    A2.data[:] = 1.0
    D2 = A2 - A2.multiply(A)
    D2.setdiag(0)
    D2.eliminate_zeros()
    cn = np.asarray((D2 @ A)[x, y]).ravel()
    h2 = np.asarray(D2.sum(axis=1)).ravel()
    hop1 = np.asarray(A.sum(axis=1)).ravel()
    return cn, h2, hop1


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_c_oracle_matches_scipy_formulation(seed):
    rng = np.random.default_rng(seed)
    if seed == 2:  # general graph with self-loops and user-user edges
        a = rng.integers(0, 300, 2000)
        b = rng.integers(0, 300, 2000)
    else:
        a, b = bipartite_edges(rng, 400, 60, 2500)
    ids, da, db = dense_edges(a, b)
    n = len(ids)
    g = coracle.OracleGraph(n, da, db)
    x = rng.integers(0, n, 3000).astype(np.int32)
    y = rng.integers(0, n, 3000).astype(np.int32)
    cn, jac, aa, h2 = g.score_pairs(x, y, 7, nthreads=4)
    scn, sh2, shop1 = _scipy_scores(n, da, db, x, y)
    np.testing.assert_array_equal(cn, scn.astype(np.uint32))
    np.testing.assert_array_equal(h2, sh2[x].astype(np.uint32))
    uni = sh2[x] + shop1[y] - scn
    np.testing.assert_array_equal(jac, scn / uni)


@pytest.mark.parametrize("threads", [2, 7])
def test_c_oracle_partitioned_build_equals_serial(threads, monkeypatch):
    """og_create's many-thread path (edges partitioned by row range, each range counting-sorted
    on its own: what builds the 1B-edge config-5 oracle) gives the serial path's CSR, self-loops,
    duplicates and reversed duplicates included, and the same scores."""
    rng = np.random.default_rng(threads)
    a = rng.integers(0, 3000, 60000)
    b = 3000 + np.minimum((rng.pareto(1.0, 60000) * 20).astype(np.int64), 999)
    a[:50] = b[:50]  # self-loops
    a = np.concatenate([a, b[:500]])  # reversed duplicates
    b = np.concatenate([b, a[:500]])
    monkeypatch.setenv("OG_THREADS", "1")
    g1 = coracle.OracleGraph(4000, a, b)
    monkeypatch.setenv("OG_THREADS", str(threads))
    g2 = coracle.OracleGraph(4000, a, b)
    (r1, c1), (r2, c2) = g1.csr(), g2.csr()
    np.testing.assert_array_equal(r1, r2)
    np.testing.assert_array_equal(c1, c2)
    x = rng.integers(0, 4000, 2000).astype(np.int32)
    y = rng.integers(0, 4000, 2000).astype(np.int32)
    for p, q in zip(g1.score_pairs(x, y, 5), g2.score_pairs(x, y, 5)):  # (isolated ids: no Jaccard)
        np.testing.assert_array_equal(p, q)


@settings(max_examples=40, deadline=None)
@given(st.lists(st.tuples(st.integers(0, 25), st.integers(0, 25)), min_size=1, max_size=80),
       st.integers(0, 10 ** 6))
def test_c_oracle_matches_python_oracle_random(edges, seed):
    rng = np.random.default_rng(seed)
    a = np.array([e[0] for e in edges], np.int64)
    b = np.array([e[1] for e in edges], np.int64)
    ids, da, db = dense_edges(a, b)
    g = coracle.OracleGraph(len(ids), da, db)
    adj = {}
    for p, q in zip(a.tolist(), b.tolist()):
        adj.setdefault(p, set()).add(q)
        adj.setdefault(q, set()).add(p)
    x = rng.integers(0, len(ids), 20).astype(np.int32)
    y = rng.integers(0, len(ids), 20).astype(np.int32)
    try:
        cn, jac, aa, _ = g.score_pairs(x, y, 7)
    except ZeroDivisionError:
        cn = None
    for i in range(len(x)):
        h2 = O.nodes_at_hop(adj, int(ids[x[i]]), 2)
        n1 = O.nodes_at_hop(adj, int(ids[y[i]]), 1)
        if not (h2 | n1):
            assert cn is None
            return
        if cn is None:
            continue
        assert cn[i] == O.common_neighbors(h2, n1)
        assert jac[i] == O.jaccard(h2, n1)
        assert math.isclose(aa[i], O.adamic_adar(h2, n1, adj), rel_tol=1e-12, abs_tol=1e-300)
        assert aa[i] == O.adamic_adar_exact(h2, n1, adj)  # 128-bit sum == math.fsum, bit for bit


@pytest.mark.parametrize("split", ["bip/train", "bip/test"])
def test_topk_oracle_composes_reference_scorers(split):
    """The full-candidate top-k oracle (config 3) scores each distance-3 candidate with the
    reference's own formulas: every (user, business) pair of the golden examples that is a
    distance-3 candidate gets the reference's CN / Jaccard exactly and its Adamic-Adar to 1e-9."""
    adj = O.load_edge_list(os.path.join(GOLDEN, split, "graph.txt"))
    ex = golden(split, "examples.json")
    ref = {m: golden(split, f) for m, f in zip(METHODS, U_FILES)}
    checked = 0
    for u in list(ex)[:12]:
        if int(u) not in adj:
            continue
        tops = {m: dict(O.topk_full_candidates(adj, int(u), 10**9, m)[0]) for m in METHODS}
        for b in ex[u]:
            if int(b) in tops["jaccard"]:
                assert tops["common_neighbors"][int(b)] == ref["common_neighbors"][u][b]
                assert tops["jaccard"][int(b)] == ref["jaccard"][u][b]
                assert math.isclose(tops["adamic_adar"][int(b)], ref["adamic_adar"][u][b], rel_tol=1e-9)
                checked += 1
        ranked = O.topk_full_candidates(adj, int(u), 10**9, "jaccard")[0]
        assert ranked == sorted(ranked, key=lambda t: (-t[1], t[0]))
    assert checked > 20


def test_svd_entry_parity_rule():
    """The per-entry SVD comparator: two ARPACK runs from different starts pass; a perturbed
    entry, a non-zero structural zero and a wrong near-zero entry fail."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla

    rng = np.random.default_rng(0)
    M = sp.random(400, 300, density=0.03, random_state=1, format="csr")
    M.data[:] = 1.0
    M = sp.vstack([M, sp.csr_matrix((5, 300))]).tocsr()
    u1, s1, vt1 = spla.svds(M, k=10, v0=rng.standard_normal(min(M.shape)))
    u2, s2, vt2 = spla.svds(M, k=10, v0=rng.standard_normal(min(M.shape)))
    rows = np.r_[rng.integers(0, 400, 3000), np.arange(400, 405)]
    cols = rng.integers(0, 300, len(rows))
    a = np.einsum("ij,ji->i", (u1 * s1)[rows], vt1[:, cols])
    b = np.einsum("ij,ji->i", (u2 * s2)[rows], vt2[:, cols])
    zero = np.diff(M.indptr)[rows] == 0
    a[zero] = 0.0
    assert O.svd_entry_parity(a, b, zero)["ok"]
    bad = a.copy()
    i = int(np.argmax(np.abs(b)))
    bad[i] *= 1 + 1e-4
    r = O.svd_entry_parity(bad, b, zero)
    assert not r["ok"] and r["worst_entry"]["index"] == i
    bad = a.copy()
    bad[np.flatnonzero(zero)[0]] = 1e-300
    assert not O.svd_entry_parity(bad, b, zero)["ok"]


def test_exact_adamic_sum_on_many_terms():
    """The C oracle's 128-bit Adamic-Adar sum equals math.fsum of the reference's terms on a pair
    with 20K common neighbours of mixed degree (where naive float addition drifts by many ulps)."""
    rng = np.random.default_rng(5)
    n_users = 20000
    users = np.arange(n_users)
    extra_b = 2 + rng.integers(0, 3000, 60000)
    a = np.concatenate([users, users, rng.integers(0, n_users, 60000)])
    b = np.concatenate([np.zeros(n_users, np.int64), np.ones(n_users, np.int64), extra_b]) + n_users
    ids, da, db = dense_edges(a, b)
    g = coracle.OracleGraph(len(ids), da, db)
    x = np.searchsorted(ids, [0, 7]).astype(np.int32)
    y = np.searchsorted(ids, [n_users + 1, n_users + 1]).astype(np.int32)
    cn, _, aa, _ = g.score_pairs(x, y, 7)
    adj = {}
    for p, q in zip(a.tolist(), b.tolist()):
        adj.setdefault(p, set()).add(q)
        adj.setdefault(q, set()).add(p)
    for i, u in enumerate([0, 7]):
        h2 = O.nodes_at_hop(adj, u, 2)
        n1 = O.nodes_at_hop(adj, n_users + 1, 1)
        assert cn[i] == len(h2 & n1) > 19000
        assert aa[i] == O.adamic_adar_exact(h2, n1, adj)
        assert math.isclose(aa[i], O.adamic_adar(h2, n1, adj), rel_tol=1e-12)
