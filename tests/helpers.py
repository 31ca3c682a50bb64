"""Shared test helpers: fixtures, random graphs, oracle-backed expectations, comparators."""
import json
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

METHODS = ["common_neighbors", "jaccard", "adamic_adar"]
U_FILES = ["u_cn.json", "u_jaccard.json", "u_adamic.json"]
B_FILES = ["b_cn.json", "b_jaccard.json", "b_adamic.json"]
SIM_CASES = ["edge", "general", "bip/train", "bip/test"]


def load(path):
    with open(path) as f:
        return json.load(f)


def golden(case, name):
    return load(os.path.join(GOLDEN, case, name))


def read_edges(path):
    """graph.txt -> int64 arrays with SNAP LoadEdgeList text rules (test-side reader)."""
    a, b = [], []
    with open(path) as f:
        for line in f:
            if line.startswith("#"):
                continue
            c = line.split()
            if len(c) < 2:
                continue
            a.append(int(c[0]))
            b.append(int(c[1]))
    return np.array(a, np.int64), np.array(b, np.int64)


def assert_same_scores(got, exp, method, rtol=1e-5):
    """Reference file contract: same keys in the same order; CN int bit-exact; Jaccard
    float bit-exact (correctly rounded quotient of exact integers); Adamic-Adar float
    within rtol (summation order differs from the reference's set order), and an int 0
    exactly where the reference wrote the untouched int 0."""
    assert list(got.keys()) == list(exp.keys()), "user keys differ"
    for u in exp:
        assert list(got[u].keys()) == list(exp[u].keys()), "business keys differ for %s" % u
        for v, e in exp[u].items():
            g = got[u][v]
            assert type(g) is type(e), (method, u, v, g, e)
            if method == "adamic_adar" and isinstance(e, float):
                assert math.isclose(g, e, rel_tol=rtol, abs_tol=0.0), (u, v, g, e)
            else:
                assert g == e, (method, u, v, g, e)


def bipartite_edges(rng, n_users, n_bus, n_draws, zipf=0.8, shuffle_ids=False):
    """Synthetic review graph: uniform users, Zipf business popularity."""
    p = np.arange(1, n_bus + 1, dtype=np.float64) ** -zipf
    p /= p.sum()
    u = rng.integers(0, n_users, n_draws).astype(np.int64)
    b = rng.choice(n_bus, size=n_draws, p=p).astype(np.int64) + n_users
    if shuffle_ids:
        perm = rng.permutation(n_users + n_bus).astype(np.int64)
        u, b = perm[u], perm[b]
    return u, b


def dense_edges(a, b):
    """Independent dense relabel (sorted unique ids) for the C oracle."""
    ids = np.unique(np.concatenate([a, b]))
    return ids, np.searchsorted(ids, a).astype(np.int32), np.searchsorted(ids, b).astype(np.int32)
