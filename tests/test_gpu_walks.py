"""random_walks.py drop-in: golden outputs of the reference (bipartite: all 0.0; general
graph: nonzero) and scipy parity for run_random_walk, including rows split across items."""
import os
import shutil

import numpy as np
import pytest
import scipy.sparse as sp

import random_walks as RW
from helpers import GOLDEN, load

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", ["bip/train", "general"])
def test_run_random_walks_matches_reference(gpu, case, tmp_path, monkeypatch):
    os.makedirs(tmp_path / "data" / "train")
    for f in ("graph.txt", "examples.json"):
        shutil.copy(os.path.join(GOLDEN, case, f), tmp_path / "data" / "train" / f)
    monkeypatch.chdir(tmp_path)
    RW.run_random_walks("test", True)  # the reference forces 'train' / unweighted
    got = load(str(tmp_path / "data" / "train" / "random_walks.json"))
    exp = load(os.path.join(GOLDEN, case, "random_walks.json"))
    assert list(got) == list(exp)
    for u in exp:
        assert list(got[u]) == list(exp[u])
        for b in exp[u]:
            assert isinstance(got[u][b], float)
            assert got[u][b] == pytest.approx(exp[u][b], rel=1e-9, abs=1e-300)


def _scipy_walk(T, u, iterations, jump_p):
    p = np.zeros(T.shape[0])
    p[u] = 1.0
    p = sp.csr_matrix(p)
    for _ in range(iterations):
        p = p.dot(T)
        p *= 1 - jump_p
    return np.asarray(p.todense()).ravel()


@pytest.mark.parametrize("seed", [0, 1])
def test_run_random_walk_vs_scipy(gpu, seed):
    rng = np.random.default_rng(seed)
    n = 3000
    a = rng.integers(0, n, 20000)
    b = rng.integers(0, n, 20000)
    hub = np.arange(1, 1500)  # node 0 has degree ~1500 > 256: its pull row is split
    a = np.r_[a, np.zeros(len(hub), np.int64)]
    b = np.r_[b, hub]
    A = sp.coo_matrix((np.ones(2 * len(a)), (np.r_[a, b], np.r_[b, a])), shape=(n, n)).tocsr()
    A.data[:] = 1.0
    rs = np.asarray(A.sum(axis=1)).ravel()
    rs[rs == 0] = 1.0
    T = sp.diags(1.0 / rs) @ A
    for u in (0, 5, 77):
        got = RW.run_random_walk(T, u, 10, 0.2)
        assert got.shape == (1, n)
        want = _scipy_walk(T, u, 10, 0.2)
        np.testing.assert_allclose(np.asarray(got.todense()).ravel(), want, rtol=1e-10, atol=1e-300)


def test_batched_walks_many_starts(gpu):
    from blp.walk import DeviceWalk

    rng = np.random.default_rng(4)
    n = 2000
    a = rng.integers(0, n, 15000)
    b = rng.integers(0, n, 15000)
    A = sp.coo_matrix((np.ones(2 * len(a)), (np.r_[a, b], np.r_[b, a])), shape=(n, n)).tocsr()
    A.data[:] = 1.0
    rs = np.asarray(A.sum(axis=1)).ravel()
    rs[rs == 0] = 1.0
    T = sp.diags(1.0 / rs) @ A
    starts = rng.choice(n, 70, replace=False)  # three batches of 32
    qs = np.repeat(np.arange(70), 25)
    qn = rng.integers(0, n, len(qs))
    got = DeviceWalk(T).run(starts, qs, qn, iterations=7, scale=0.8)
    for i, s in enumerate(starts):
        want = _scipy_walk(T, s, 7, 0.2)[qn[qs == i]]
        np.testing.assert_allclose(got[qs == i], want, rtol=1e-10, atol=1e-300)
