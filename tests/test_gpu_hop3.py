"""GPU hop-3 candidate generation (dataset_maker.py:137-144) vs the reference fixture and
the C oracle. The candidate SET is exact (rate = 1); the 1% negative sample is checked
statistically (the reference's Python RNG order over SNAP's BFS is not reproducible)."""
import os

import numpy as np
import pytest

import blp
import coracle
from helpers import GOLDEN, bipartite_edges, dense_edges, load, read_edges

pytestmark = pytest.mark.gpu


def test_hop3_matches_reference_fixture(gpu):
    d = os.path.join(GOLDEN, "hop3")
    G = blp.load_edge_list(os.path.join(d, "graph.txt"))
    ex = load(os.path.join(d, "examples.json"))
    new = np.array([list(map(int, l.split())) for l in open(os.path.join(d, "new_edges.txt"))])
    users = [int(u) for u in ex]
    src = G.dense(users)
    pu, okp = G.lookup(new[:, 0])
    pb, okb = G.lookup(new[:, 1])
    rank = {int(s): i for i, s in enumerate(src)}
    buckets = [[] for _ in src]
    for a, b, ok in zip(pu, pb, okp & okb):
        if ok and int(a) in rank:
            buckets[rank[int(a)]].append(int(b))
    pos_off = np.r_[0, np.cumsum([len(x) for x in buckets])].astype(np.int32)
    pos_y = np.array([b for x in buckets for b in x] or [0], np.int32)
    x, y, lab = G.hop3_sample(src, pos_off, pos_y, rate=1.0, seed=0)
    got = {}
    for xi, yi, li in zip(G.node_ids[x], G.node_ids[y], lab):
        got.setdefault(str(xi), {})[str(yi)] = int(li)
    assert set(got) == {u for u in ex if ex[u]}
    for u in got:
        assert got[u] == {b: l for b, l in ex[u].items()}


@pytest.mark.parametrize("seed,mode", [(0, "wedge"), (1, "wedge"), (0, "wedge_rows"), (0, "wedge_bitmaps"),
                                       (1, "wedge_bitmaps"), (0, "lds"), (1, "lds"), (0, "hbm")])
def test_hop3_sets_vs_oracle(gpu, seed, mode, monkeypatch):
    """wedge: marks from the graph's wedge rows (default on review graphs), rows longer than
    their set's bitmap OR-ed as wedge-row bitmaps; wedge_rows: no bitmaps; wedge_bitmaps: every
    row through its bitmap; lds: H2 bitmap then N(H2) row walks in LDS; hbm: the same in
    per-workgroup HBM bitmaps (configs 4/5)."""
    if mode == "wedge_rows":
        monkeypatch.setenv("BLP_HOP3_NO_WBM", "1")
    if mode == "wedge_bitmaps":
        monkeypatch.setenv("BLP_WBM_MIN_X", "0")
    if not mode.startswith("wedge"):
        monkeypatch.setenv("BLP_HOP3_NO_WEDGE", "1")
    if mode == "hbm":
        monkeypatch.setenv("BLP_HOP3_FORCE_GLOBAL", "1")
    rng = np.random.default_rng(seed)
    a, b = bipartite_edges(rng, 40000, 3000, 250000)
    G = blp.DeviceGraph(a, b)
    ids, da, db = dense_edges(a, b)
    og = coracle.OracleGraph(len(ids), da, db)
    nu = G.n - len(np.unique(b))
    src = np.sort(rng.choice(nu, 64, replace=False)).astype(np.int32)
    x, y, lab = G.hop3_sample(src, rate=1.0)
    assert not lab.any()
    counts, members = og.hop3(np.searchsorted(ids, G.node_ids[src]))
    k = 0
    for i, s in enumerate(src):
        sel = x == s
        got = np.sort(G.node_ids[y[sel]])
        exp = ids[members[k:k + counts[i]]]
        k += counts[i]
        np.testing.assert_array_equal(got, exp)
        assert np.all(np.diff(y[sel]) > 0)  # ascending dense ids within a source


def test_hop3_sampling_rate_and_determinism(gpu):
    rng = np.random.default_rng(3)
    a, b = bipartite_edges(rng, 40000, 3000, 250000)
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    src = np.sort(rng.choice(nu, 200, replace=False)).astype(np.int32)
    full = G.hop3_sample(src, rate=1.0)
    s1 = G.hop3_sample(src, rate=0.05, seed=9)
    s2 = G.hop3_sample(src, rate=0.05, seed=9)
    for p, q in zip(s1, s2):
        np.testing.assert_array_equal(p, q)
    frac = len(s1[0]) / len(full[0])
    assert 0.04 < frac < 0.06, frac
    kept = set(zip(s1[0].tolist(), s1[1].tolist()))
    assert kept <= set(zip(full[0].tolist(), full[1].tolist()))


def test_general_graph_hop3_vs_oracle(gpu):
    # non-bipartite: distance-3 must exclude distance <= 2 nodes that N(H2) also reaches
    rng = np.random.default_rng(4)
    a = rng.integers(0, 2000, 6000)
    b = rng.integers(0, 2000, 6000)
    G = blp.DeviceGraph(a, b)
    ids, da, db = dense_edges(a, b)
    og = coracle.OracleGraph(len(ids), da, db)
    src = np.arange(0, G.n, 37, dtype=np.int32)
    x, y, _ = G.hop3_sample(src, rate=1.0)
    counts, members = og.hop3(np.searchsorted(ids, G.node_ids[src]))
    k = 0
    for i, s in enumerate(src):
        got = np.sort(G.node_ids[y[x == s]])
        np.testing.assert_array_equal(got, ids[members[k:k + counts[i]]])
        k += counts[i]


def test_dataset_maker_drop_in_matches_reference(gpu, tmp_path):
    """dataset_maker.make_examples (dataset_maker.py:80-159) on the reference fixture's graph
    with negative_sample_rate=1.0 and every eligible user: the written examples.json equals
    the reference's (exact hop-3 candidate sets and labels)."""
    import json
    import shutil

    import dataset_maker

    d = os.path.join(GOLDEN, "hop3")
    for f in ("graph.txt", "new_edges.txt"):
        shutil.copy(os.path.join(d, f), tmp_path / f)
    a, b = read_edges(os.path.join(d, "graph.txt"))
    (tmp_path / "review.json").write_text(json.dumps({str(u): {} for u in np.unique(a)}))
    got = dataset_maker.make_examples(str(tmp_path) + "/", n_users=10**9, negative_sample_rate=1.0)
    ref = load(os.path.join(d, "examples.json"))
    assert {u: v for u, v in ref.items() if v} == got
    assert json.loads((tmp_path / "examples.json").read_text()) == got


@pytest.mark.parametrize("long_rows", [False, True])
def test_hop3_wedge_and_row_walk_agree(gpu, long_rows, monkeypatch):
    """The wedge-row path and the row-walk path emit identical (x, y, label) lists, positives
    and sampled negatives included. With users of > 64 reviews some businesses have no wedge
    row and the launch falls back to the row walk (same output either way)."""
    rng = np.random.default_rng(11)
    a, b = bipartite_edges(rng, 30000, 2000, 200000)
    if long_rows:  # a few heavy users: their businesses get no wedge row
        heavy = rng.choice(30000, 20, replace=False)
        a = np.concatenate([a, np.repeat(heavy, 90)])
        b = np.concatenate([b, 30000 + rng.integers(0, 2000, 20 * 90)])
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    src = np.sort(rng.choice(nu, 120, replace=False)).astype(np.int32)
    pos_off = np.arange(0, 2 * len(src) + 1, 2, dtype=np.int32)
    pos_y = rng.integers(nu, G.n, 2 * len(src)).astype(np.int32)
    got = G.hop3_sample(src, pos_off, pos_y, rate=0.05, seed=4)
    sub = G.hop3_sample(src[::3], pos_off[:len(src[::3]) + 1], pos_y, rate=0.05, seed=4)  # bitmaps reused or rebuilt
    monkeypatch.setenv("BLP_HOP3_NO_WEDGE", "1")
    ref_sub = G.hop3_sample(src[::3], pos_off[:len(src[::3]) + 1], pos_y, rate=0.05, seed=4)
    for p, q in zip(sub, ref_sub):
        np.testing.assert_array_equal(p, q)
    ref = G.hop3_sample(src, pos_off, pos_y, rate=0.05, seed=4)
    for p, q in zip(got, ref):
        np.testing.assert_array_equal(p, q)
