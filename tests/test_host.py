"""Host-side logic on CPU (no GPU): libblp's host helpers, the id map, SNAP degree rules,
the score-file assembly, the svd.py matrix build, and the C-ABI symbol table."""
import ctypes
import math
import os
import re
import shutil

import numpy as np
import pytest

import blp
import blp_oracle as O
import coracle
import similarity
import svd as S
from helpers import (B_FILES, GOLDEN, METHODS, SIM_CASES, U_FILES, assert_same_scores, dense_edges, golden, load,
                     read_edges)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "blp.h")).read()
    names = set(re.findall(r"^\s*(?:int|const char\*)\s+(blp_\w+)\s*\(", hdr, re.M))
    assert len(names) >= 20
    L = blp.lib()
    missing = [n for n in sorted(names) if not hasattr(L, n)]
    assert not missing, missing


def test_edge_list_parser_matches_snap_text_rules(tmp_path):
    p = tmp_path / "g.txt"
    p.write_text("# header\n1 2\n3\t4 extra\n\n5\n  6   7\n#8 9\n-1 +10\n")
    a, b = blp.parse_edge_list(str(p))
    assert a.tolist() == [1, 3, 6, -1] and b.tolist() == [2, 4, 7, 10]
    for case in SIM_CASES:
        a, b = blp.parse_edge_list(os.path.join(GOLDEN, case, "graph.txt"))
        ra, rb = read_edges(os.path.join(GOLDEN, case, "graph.txt"))
        assert a.tolist() == ra.tolist() and b.tolist() == rb.tolist()
    # > 1 MiB (threaded slices): the one-pass "digits ws digits" lines mixed with every other
    # shape the SNAP rules accept or skip (CRLF, tabs, extra columns, signs, comments, blanks,
    # 18- and 19-digit ids)
    rng = np.random.default_rng(9)
    shapes = ["%d %d\n", "%d\t%d\r\n", "%d  %d extra\n", "-%d +%d\n", "  %d %d\n", "%d\t%d \t\n", "# %d %d\n", "%d\n\n",
              "%d000000000 %d\n", "%d 1%018d\n"]
    lines = []
    for k in rng.integers(0, len(shapes), 200000):
        x, y = rng.integers(0, 10**9, 2)
        lines.append(shapes[k] % ((x,) if shapes[k] == "%d\n\n" else (x, y)))
    q = tmp_path / "big.txt"
    q.write_text("".join(lines) + "12 34")  # last line without a newline
    a, b = blp.parse_edge_list(str(q))
    ra, rb = read_edges(str(q))
    assert len(ra) > 100000 and a.tolist() == ra.tolist() and b.tolist() == rb.tolist()


@pytest.mark.parametrize("case", SIM_CASES + ["hop3"])
def test_host_graph_matches_snap_semantics(case):
    path = os.path.join(GOLDEN, case, "graph.txt")
    adj = O.load_edge_list(path)
    G = blp.HostGraph(*blp.parse_edge_list(path))
    assert sorted(G.node_ids.tolist()) == sorted(adj)
    for v, nbrs in adj.items():
        d = G.dense([v])[0]
        row = G.node_ids[G.col_idx[G.row_ptr[d]:G.row_ptr[d + 1]]]
        assert set(row.tolist()) == nbrs - {v}               # CSR: hop-1 set (self-loop not stored)
        assert G.degree[d] == O.degree(adj, v)                # SNAP GetDeg counts a self-loop once
        exp_w = math.log(O.degree(adj, v)) ** -1 if O.degree(adj, v) > 1 else 0.0
        assert G.aa_weight[d] == exp_w                        # bit-identical AA term
    ids, present = G.lookup(np.array([10**9, -5]))
    assert not present.any() and (ids == -1).all()


@pytest.mark.parametrize("case", SIM_CASES)
def test_score_file_assembly_matches_reference(case):
    """similarity.py's dict/JSON contract, fed with oracle scores (GPU-free)."""
    path = os.path.join(GOLDEN, case, "graph.txt")
    ex = golden(case, "examples.json")
    G = blp.HostGraph(*blp.parse_edge_list(path))
    _, _, ui, vi = similarity.flatten_examples(ex)
    du, pu = G.lookup(ui)
    dv, pv = G.lookup(vi)
    present = pu & pv
    a, b = read_edges(path)
    ids, da, db = dense_edges(a, b)
    og = coracle.OracleGraph(len(ids), da, db)
    xo = np.searchsorted(ids, G.node_ids[du[present]])
    yo = np.searchsorted(ids, G.node_ids[dv[present]])
    for side, files, table in ((0, U_FILES, similarity._U_BITS), (1, B_FILES, similarity._B_BITS)):
        x, y = (xo, yo) if side == 0 else (yo, xo)
        cn, jac, aa, _ = og.score_pairs(x, y, 7) if len(x) else (np.zeros(0, np.uint32),) * 4
        scores = {"cn": cn, "jaccard": jac, "adamic": aa}
        for m, f in zip(METHODS, files):
            got = similarity.assemble(ex, similarity._values(table.get(m, 0), present, scores))
            assert_same_scores(got, golden(case, f), m)


def test_unknown_method_writes_only_missing_zeros():
    ex = golden("edge", "examples.json")
    present = np.array([True] * 26)
    present[4] = False
    vals = similarity._values(0, present, {})
    assert vals.count(0) == 1 and vals.count(None) == 25


@pytest.mark.parametrize("split", ["train", "test"])
def test_svd_matrix_build(split, tmp_path, monkeypatch):
    shutil.copytree(os.path.join(GOLDEN, "bip", split), tmp_path / "data" / split)
    monkeypatch.chdir(tmp_path)
    users, bus, ex, ur, bc, M = S.user_business_matrix(split)
    assert users == list(load(os.path.join(GOLDEN, "bip", split, "user.json")))
    edges = {(l.split()[0], l.split()[1]) for l in open(os.path.join(GOLDEN, "bip", split, "graph.txt"))}
    assert M.nnz == len(edges) and set(M.data.tolist()) == {1.0}
    for u, b in list(edges)[:50]:
        assert M[ur[u], bc[b]] == 1.0


def test_svd_dead_code_raises_like_reference(tmp_path, monkeypatch):
    shutil.copytree(os.path.join(GOLDEN, "bip", "train"), tmp_path / "data" / "train")
    monkeypatch.chdir(tmp_path)
    with pytest.raises(IndexError):
        S.svd("train")


def test_engine_fails_loudly_without_library(monkeypatch):
    from blp import _lib

    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libblp.so")
    with pytest.raises(_lib.BLPUnavailable):
        _lib.lib()


@pytest.mark.parametrize("case", ["bip/train", "general"])
def test_walk_transition_matrix_matches_networkx(case):
    """random_walks.py:14,26-29 built with networkx (the reference's own construction)."""
    import networkx as nx
    import random_walks as RW

    path = os.path.join(GOLDEN, case, "graph.txt")
    G = nx.read_edgelist(path, nodetype=int)
    A = nx.to_scipy_sparse_array(G, format="csr").astype(float)
    rs = np.asarray(A.sum(axis=1)).ravel()
    T = (np.diag(1.0 / rs) @ A.toarray())
    order, (rp, ci, val, n) = RW.transition_pull_csr(path)
    assert order.tolist() == list(G.nodes())
    W = np.zeros((n, n))
    for j in range(n):
        W[j, ci[rp[j]:rp[j + 1]]] = val[rp[j]:rp[j + 1]]
    np.testing.assert_allclose(W.T, T, rtol=1e-15, atol=0)


@pytest.mark.parametrize("case,name", [("bip/test", "u_adamic.json"), ("bip/test", "u_cn.json"),
                                       ("edge", "u_jaccard.json")])
def test_sidecar_round_trips_the_score_file(case, name, tmp_path):
    """util.write_sidecar / load_scores: the binary twin of a reference
    score file reads back as the identical dict (keys, order, int/float types, values)."""
    import util

    ref = golden(case, name)
    f = str(tmp_path / name)
    util.write_sidecar(ref, f)
    got = util.load_scores(f)
    assert list(got) == list(ref)
    for u in ref:
        assert list(got[u].items()) == list(ref[u].items())
        assert [type(v) for v in got[u].values()] == [type(v) for v in ref[u].values()]


@pytest.mark.parametrize("span", [50, 10**6, 10**12])
def test_unique_ids_match_numpy(span):
    """blp.graph._unique (presence table for compact id spans) == np.unique."""
    from blp.graph import _unique

    rng = np.random.default_rng(span % 97)
    for n in (0, 1, 1000, 200000):
        x = rng.integers(-5, span, n).astype(np.int64) + 3
        assert np.array_equal(_unique(x), np.unique(x))
        assert _unique(x).dtype == np.int64


def test_main_missing_examples_raises_like_reference(tmp_path):
    """similarity.main on a missing examples.json raises what the reference's util.load_json
    (open()) raises -- FileNotFoundError, an IOError -- before any device work."""
    with pytest.raises(FileNotFoundError):
        similarity.main(str(tmp_path / "nope.json"), str(tmp_path / "graph.txt"), METHODS,
                        [None] * 3, METHODS, [None] * 3)


def _native_edges(path, device_entry=False):
    L = blp.lib()
    from blp import graph as bg  # noqa: F401  (registers the blp_edges_* signatures)

    h = ctypes.c_void_p()
    if device_entry:
        blp._lib.check(L.blp_edges_load_device(str(path).encode(), 0, 1, 0, ctypes.byref(h)))
        on = ctypes.c_int(7)
        blp._lib.check(L.blp_edges_device(h, ctypes.byref(on)))
        assert on.value == -1  # parsed on the host
    else:
        blp._lib.check(L.blp_edges_load(str(path).encode(), 0, 1, ctypes.byref(h)))
    try:
        m, n, n0, lo, span = (ctypes.c_int64() for _ in range(5))
        blp._lib.check(L.blp_edges_info(h, *(ctypes.byref(v) for v in (m, n, n0, lo, span))))
        a = np.empty(m.value, np.int64)
        b = np.empty(m.value, np.int64)
        out = {"m": m.value, "n": n.value, "n_col0": n0.value, "lo": lo.value, "span": span.value, "a": a, "b": b}
        P = blp._lib.ptr
        if span.value:
            out.update(da=np.empty(m.value, np.int32), db=np.empty(m.value, np.int32),
                       node_ids=np.empty(n.value, np.int64), id_map=np.empty(span.value, np.int32))
            blp._lib.check(L.blp_edges_fetch(h, P(a), P(b), P(out["da"]), P(out["db"]), P(out["node_ids"]),
                                             P(out["id_map"])))
        else:
            blp._lib.check(L.blp_edges_fetch(h, P(a), P(b), None, None, None, None))
        return out
    finally:
        L.blp_edges_destroy(h)


@pytest.mark.parametrize("kind", ["golden", "compact", "negative", "sparse"])
def test_native_edge_load_equals_host_id_map(tmp_path, kind):
    """blp_edges_load (one threaded parse + the dense id map, similarity.py:16) gives the same
    endpoints as blp_edges_parse and the same id map as HostGraph._ids: column-0 ids ascending,
    then column-1-only ids ascending; dense lookups agree with HostGraph.lookup, absent ids -1."""
    rng = np.random.default_rng(3)
    if kind == "golden":
        path = os.path.join(GOLDEN, "bip", "train", "graph.txt")
    else:
        if kind == "compact":
            a = rng.integers(0, 5000, 300000)
            b = rng.integers(5000, 5600, 300000)
        elif kind == "negative":
            a = rng.integers(-3000, 3000, 300000)
            b = rng.integers(-3000, 3000, 300000)
        else:
            a = rng.integers(0, 10**12, 1000) * 7
            b = rng.integers(0, 10**12, 1000) * 11
        a[:5] = b[:5]  # self-loops
        path = tmp_path / "graph.txt"
        with open(path, "w") as f:
            f.write("# comment\n")
            f.write("".join("%d\t%d\n" % (x, y) for x, y in zip(a, b)))
    got = _native_edges(path)
    ra, rb = blp.parse_edge_list(str(path))
    np.testing.assert_array_equal(got["a"], ra)
    np.testing.assert_array_equal(got["b"], rb)
    H = blp.HostGraph(ra, rb)
    if kind == "sparse":
        assert got["span"] == 0
        return
    assert got["span"] > 0 and got["n"] == H.n and got["n_col0"] == H.n_col0
    np.testing.assert_array_equal(got["node_ids"], H.node_ids)
    np.testing.assert_array_equal(got["da"], H.dense(ra))
    np.testing.assert_array_equal(got["db"], H.dense(rb))
    probe = np.concatenate([ra[:1000], rb[:1000], [got["lo"] - 1, got["lo"] + got["span"], 10**15, -10**15]])
    probe = np.ascontiguousarray(probe, np.int64)
    dense = np.empty(len(probe), np.int32)
    blp._lib.check(blp.lib().blp_ids_lookup(blp._lib.ptr(got["id_map"]), got["lo"], got["span"],
                                            blp._lib.ptr(probe), len(probe), blp._lib.ptr(dense)))
    exp, _ = H.lookup(probe)
    np.testing.assert_array_equal(dense, exp)


def test_device_edge_load_small_files_stay_on_host(tmp_path):
    """blp_edges_load_device leaves files under 1 MiB (and text outside graph.txt's line shape)
    to the host loader -- no device is touched, so this runs without one -- with the host
    loader's results."""
    rng = np.random.default_rng(4)
    a = rng.integers(0, 5000, 20000)
    b = rng.integers(5000, 5600, 20000)
    path = tmp_path / "graph.txt"
    path.write_text("".join("%d %d\n" % (x, y) for x, y in zip(a, b)))
    got, exp = _native_edges(path, device_entry=True), _native_edges(path)
    assert got.keys() == exp.keys()
    for k in got:
        np.testing.assert_array_equal(got[k], exp[k])


@pytest.mark.parametrize("thp", ["1", "0"])
def test_host_alloc_arrays(thp, monkeypatch):
    """blp_host_alloc / blp_host_free (huge-page host memory for result arrays; BLP_NO_THP=1:
    malloc) behind blp._lib.host_empty: shapes, dtypes, writable, independent, released with the
    last view; sizes below and above the 4 MiB huge-page threshold, and zero."""
    import subprocess
    import sys

    code = r'''
import gc, numpy as np
from blp import _lib
for shape, dt in [(0, np.uint8), (10, np.uint32), ((1 << 20, 24), np.uint8), (3_000_001, np.float64)]:
    a = _lib.host_empty(shape, dt)
    b = _lib.host_empty(shape, dt)
    assert a.shape == ((shape,) if np.isscalar(shape) else shape) and a.dtype == dt and a.flags["C_CONTIGUOUS"]
    a[...] = 1
    b[...] = 2
    assert (a == 1).all() and (b == 2).all()
    v = a.reshape(-1)[: max(a.size // 2, 0)]
    del a
    gc.collect()
    assert (v == 1).all()  # a view keeps the block alive
    del v, b
print("ok")
'''
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(os.path.dirname(__file__), "..",
                                                                   "bipartite-link-prediction_amd")]))
    if thp == "0":
        env["BLP_NO_THP"] = "1"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
