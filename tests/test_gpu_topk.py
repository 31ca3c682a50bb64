"""GPU full-candidate top-k (BASELINE.json configs[2]) vs the oracle.

The oracle (oracle/blp_oracle.topk_full_candidates) scores every exact-distance-3 candidate
with the reference's set formulas (similarity.py:108-126) and sorts by (score desc, id asc).
Bit-exact bars: CN and Jaccard lists (ids and scores), |H3| counts, and Adamic-Adar as the
correctly rounded sum of the reference's own terms (exact two-word integer sums of
w * 2^58, blp_internal.h; equal to blp_score_pairs' values and to math.fsum of the terms),
within a few ulps of the reference's set-order float sums (checked below).
The reference itself has no top-k: the composition is "parity unpinned" beyond its scorers.
"""
import math

import numpy as np
import pytest

import blp
import blp_oracle as bo
from helpers import bipartite_edges

pytestmark = pytest.mark.gpu

METHODS = ["common_neighbors", "jaccard", "adamic_adar"]
ALL = blp.CN | blp.JACCARD | blp.ADAMIC


def adj_of(a, b):
    adj = {}
    for x, y in zip(a.tolist(), b.tolist()):
        adj.setdefault(x, set()).add(y)
        adj.setdefault(y, set()).add(x)
    return adj


def check_against_oracle(G, T, adj, src, k, mask=ALL, methods=METHODS):
    res = T(src, k=k, mask=mask)
    for m in methods:
        cols, scores, ncand = res[m]
        for i, x in enumerate(src):
            exp, n_exp = bo.topk_full_candidates(adj, int(G.node_ids[x]), k, m)
            assert ncand[i] == n_exp, (m, i)
            got_ids = [int(G.node_ids[c]) for c in cols[i] if c >= 0]
            assert got_ids == [b for b, _ in exp], (m, i, got_ids[:5], exp[:5])
            assert np.all(cols[i][len(exp):] == -1)
            got_s = scores[i][: len(exp)].tolist()
            assert got_s == [s for _, s in exp], (m, i)
    return res


@pytest.fixture(scope="module")
def small(gpu):
    rng = np.random.default_rng(3)
    a, b = bipartite_edges(rng, 3000, 300, 20000)
    G = blp.DeviceGraph(a, b, device=gpu)
    return G, adj_of(a, b), rng


@pytest.mark.parametrize("wavesel", ["0", "1"])
@pytest.mark.parametrize("expand", ["1", "0"])
def test_topk_all_methods_match_oracle(small, monkeypatch, expand, wavesel):
    """Both row layouts: expanded wedge rows (default) and the rp[w] -> N(w) walk; block-round
    and per-wave CN / Jaccard selection (BLP_TK_WAVESEL)."""
    G, adj, rng = small
    monkeypatch.setenv("BLP_TOPK_EXPAND", expand)
    monkeypatch.setenv("BLP_TK_WAVESEL", wavesel)
    T = blp.TopK(G, "user")
    assert (T.info()["wedge_entries"] > 0) == (expand == "1")
    src = rng.choice(G.n_col0, 40, replace=False)
    check_against_oracle(G, T, adj, src, 20)


def test_topk_u32_tier_and_multi_chunk(small, monkeypatch):
    """Tiny tier limits force u32/u16 counters; a tiny counter space forces many chunks (and
    the direct Adamic-Adar path)."""
    G, adj, rng = small
    src = rng.choice(G.n_col0, 16, replace=False)
    monkeypatch.setenv("BLP_TOPK_T8", "20")
    monkeypatch.setenv("BLP_TOPK_T16", "60")
    T = blp.TopK(G, "user")
    info = T.info()
    assert info["chunks"] == 1 and info["tier32"] > 0 and info["tier16"] > 0
    check_against_oracle(G, T, adj, src, 20)
    monkeypatch.setenv("BLP_TOPK_ACC_WORDS", "40")
    T2 = blp.TopK(G, "user")
    assert T2.info()["chunks"] >= 3
    check_against_oracle(G, T2, adj, src, 20)
    assert T2.stats(2)[1] == len(src)  # every source took the direct Adamic-Adar path


@pytest.mark.parametrize("wavesel", ["0", "1"])
@pytest.mark.parametrize("acc_words", [None, "600"])
def test_topk_selection_pruning_many_targets(gpu, monkeypatch, acc_words, wavesel):
    """More targets than one selection round (1,024): the CN and Jaccard walks stop once the
    degree bound falls below the k-th key. Many equal degrees and equal counts (ties broken by
    id), k = 1, 5, 20 and 64 (the per-wave selection's largest list) and 65 (its fallback to
    block rounds); with a small counter space the bound is applied per chunk and the per-wave
    selection starts from the earlier chunks' list."""
    monkeypatch.setenv("BLP_TK_WAVESEL", wavesel)
    rng = np.random.default_rng(21)
    a, b = bipartite_edges(rng, 20000, 5000, 120000, zipf=0.5)
    G = blp.DeviceGraph(a, b, device=gpu)
    adj = adj_of(a, b)
    if acc_words:
        monkeypatch.setenv("BLP_TOPK_ACC_WORDS", acc_words)
    T = blp.TopK(G, "user")
    assert (T.info()["chunks"] > 1) == (acc_words is not None)
    src = rng.choice(np.flatnonzero(G.hop1_size[: G.n_col0] > 1), 12, replace=False)
    for k in (1, 5, 20, 64, 65):
        check_against_oracle(G, T, adj, src, k, mask=blp.CN | blp.JACCARD, methods=METHODS[:2])


@pytest.mark.parametrize("knobs", [
    {},                                               # dense counts for the hot prefix (default)
    {"BLP_TOPK_NO_DENSE": "1"},                       # every target walked
    {"BLP_TOPK_DENSE_MAX": "1"},                      # one dense target per source, the rest walked
    {"BLP_TOPK_DENSE_MAX": "3"},                      # corrections between dense targets
    {"BLP_TOPK_DENSE_F": "40"},                       # only the most popular targets dense
    {"BLP_TOPK_DENSE_MAX": "64", "BLP_TOPK_T8": "20", "BLP_TOPK_T16": "60"},  # all tiers
    {"BLP_TOPK_DENSE_MAX": "64", "BLP_TOPK_NO_FUSE": "1"},
    {"BLP_TOPK_FUSE_H": "20"},                        # AA through the candidate hash, dense words added
    {"BLP_TOPK_FUSE_H": "20", "BLP_TOPK_HCAP": "0"},  # ... through the direct chunks
    {"BLP_TOPK_NO_FUSE": "1", "BLP_TOPK_HCAP": "0", "BLP_TOPK_DENSE_MAX": "3"},
    {"BLP_TOPK_FUSE_H": "20", "BLP_TOPK_DENSE_AA_MB": "0"},  # no dense AA words: those passes walk all
])
def test_topk_dense_counts_match_oracle(small, monkeypatch, knobs):
    """Hot targets' counts added from their precomputed member counts (minus members already
    counted through an earlier hot target, minus x) give the walk's lists exactly."""
    G, adj, rng = small
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    T = blp.TopK(G, "user")
    src = rng.choice(np.flatnonzero(G.hop1_size[: G.n_col0] > 2), 30, replace=False)
    check_against_oracle(G, T, adj, src, 20)
    dense = T.stats(7)[1]
    assert (dense == 0) == ("BLP_TOPK_NO_DENSE" in knobs)
    if knobs.get("BLP_TOPK_HCAP") == "0":
        assert T.stats(2)[1] > 0  # direct AA path taken
    elif "BLP_TOPK_FUSE_H" in knobs:
        assert T.stats(1)[1] > 0  # candidate hash path taken
    if "BLP_TOPK_DENSE_MAX" in knobs and knobs["BLP_TOPK_DENSE_MAX"] == "1":
        assert dense <= len(src)


def test_topk_unfused_matches_oracle(small, monkeypatch):
    G, adj, rng = small
    monkeypatch.setenv("BLP_TOPK_NO_FUSE", "1")
    T = blp.TopK(G, "user")
    src = rng.choice(G.n_col0, 24, replace=False)
    check_against_oracle(G, T, adj, src, 20)


def test_topk_aa_paths_agree(small, monkeypatch):
    """Adamic-Adar top-k through the fused sums (default on this graph), the candidate hash
    and the direct chunked accumulation: identical lists."""
    G, adj, rng = small
    src = rng.choice(G.n_col0, 32, replace=False)
    T = blp.TopK(G, "user")
    r0 = T(src, k=15, mask=blp.ADAMIC)["adamic_adar"]
    assert T.stats(5)[1] == len(src)  # fused
    monkeypatch.setenv("BLP_TOPK_NO_FUSE", "1")
    T1 = blp.TopK(G, "user")
    r1 = T1(src, k=15, mask=blp.ADAMIC)["adamic_adar"]
    assert T1.stats(1)[1] > 0 and T1.stats(5)[1] == 0  # candidate hash
    monkeypatch.setenv("BLP_TOPK_HCAP", "0")
    r2 = T1(src, k=15, mask=blp.ADAMIC)["adamic_adar"]
    assert T1.stats(2)[1] == len(src)  # direct
    for x, y, z in zip(r0, r1, r2):
        assert np.array_equal(x, y) and np.array_equal(x, z)


def test_topk_scores_equal_pair_scorer(small):
    """Top-k scores are the pair kernel's values bit-for-bit; AA equals math.fsum of the
    reference's terms exactly and the reference's own set-order float sum to 1e-12."""
    G, adj, rng = small
    src = rng.choice(G.n_col0, 24, replace=False)
    res = blp.TopK(G, "user")(src, k=25, mask=ALL)
    for m, key in (("common_neighbors", "cn"), ("jaccard", "jaccard"), ("adamic_adar", "adamic")):
        cols, scores, _ = res[m]
        ok = cols >= 0
        x = np.repeat(src, cols.shape[1]).reshape(cols.shape)[ok]
        pair = G.score_pairs(x, cols[ok], 7)[key]
        assert np.array_equal(pair.astype(np.float64), scores[ok]), m
    cols, scores, _ = res["adamic_adar"]
    for i, x in enumerate(src[:6]):
        h2 = bo.nodes_at_hop(adj, int(G.node_ids[x]), 2)
        for c, s in zip(cols[i], scores[i]):
            if c >= 0:
                nb = bo.nodes_at_hop(adj, int(G.node_ids[c]), 1)
                assert s == bo.adamic_adar_exact(h2, nb, adj)
                assert math.isclose(s, bo.adamic_adar(h2, nb, adj), rel_tol=1e-12)


def test_topk_business_side(small):
    G, adj, rng = small
    T = blp.TopK(G, "business")
    src = G.n_col0 + rng.choice(G.n - G.n_col0, 12, replace=False)
    check_against_oracle(G, T, adj, src, 10)


@pytest.mark.parametrize("knobs", [{}, {"BLP_TOPK_NO_DENSE": "1"}, {"BLP_TOPK_DENSE_MAX": "2"}])
def test_topk_sources_with_long_rows(small, monkeypatch, knobs):
    """Business-side sources with more than one batch of N(x) (TK_SEG = 256 entries): the most
    reviewed businesses. Every batch must be walked (the flattened push once stopped after the
    first batch)."""
    G, adj, rng = small
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    nb = G.n - G.n_col0
    deg = G.hop1_size[G.n_col0:]
    top = np.argsort(-deg, kind="stable")[:6]
    assert deg[top[0]] > 256
    src = G.n_col0 + np.concatenate([top, rng.choice(nb, 6, replace=False)])
    T = blp.TopK(G, "business")
    check_against_oracle(G, T, adj, src, 10)


def test_topk_edge_cases(gpu):
    # user 0 shares business 10 with user 1, who also reviewed 11 and 12; user 2 is alone on 13
    a = np.array([0, 1, 1, 1, 2, 3, 3], np.int64)
    b = np.array([10, 10, 11, 12, 13, 11, 12], np.int64)
    G = blp.DeviceGraph(a, b, device=gpu)
    adj = adj_of(a, b)
    T = blp.TopK(G, "user")
    src = G.dense([0, 1, 2, 3])
    res = check_against_oracle(G, T, adj, src, 5)
    cols, _, ncand = res["jaccard"]
    assert ncand.tolist() == [2, 0, 0, 1]  # user 1: 11/12 are its own businesses
    assert (cols[2] == -1).all()
    check_against_oracle(G, T, adj, src, 1)  # k = 1 (ties broken by id)


def test_topk_rejects_non_bipartite(gpu):
    a = np.array([0, 1, 2], np.int64)
    b = np.array([1, 2, 0], np.int64)  # triangle: column-0 ids also appear in column 1
    G = blp.DeviceGraph(a, b, device=gpu)
    with pytest.raises(blp.BLPError):
        blp.TopK(G, "user")


def test_topk_repeat_is_deterministic(small):
    G, adj, rng = small
    src = rng.choice(G.n_col0, 64, replace=False)
    T = blp.TopK(G, "user")
    T.set_sources(src)
    outs = []
    for _ in range(2):
        T.run(20, ALL)
        outs.append([T.fetch(m) for m in METHODS])
    for r1, r2 in zip(*outs):
        for x, y in zip(r1, r2):
            assert np.array_equal(x, y)


def test_topk_largest_first_order_matches_list_order(small, monkeypatch):
    """Sources are claimed largest two-hop walk first (blp_topk_set_sources), results land by
    list index: the lists equal those of the plain list order (BLP_TK_ORDER=0) and the oracle's."""
    G, adj, rng = small
    src = rng.choice(G.n_col0, 48, replace=False)
    got = {}
    for order in ("0", "1", "2"):
        monkeypatch.setenv("BLP_TK_ORDER", order)
        T = blp.TopK(G, "user")
        T.set_sources(src)
        T.run(15, ALL)
        got[order] = [T.fetch(m) for m in METHODS]
    for o in ("1", "2"):
        for r0, r1 in zip(got["0"], got[o]):
            for x, y in zip(r0, r1):
                assert np.array_equal(x, y)
    check_against_oracle(G, blp.TopK(G, "user"), adj, src, 15)
