"""GPU parity of the truncated-SVD scorer (svd.py:7-31): reconstruction vs the reference's
stored factors and svd.json, random-factor pairs vs numpy, dense MFMA top-k vs numpy."""
import os
import shutil

import numpy as np
import pytest

import blp  # noqa: F401
import svd as S
from blp.factor import DeviceSVD
from helpers import GOLDEN, load

pytestmark = pytest.mark.gpu


def _flat(ex):
    return [(u, b) for u in ex for b in ex[u]]


@pytest.mark.parametrize("split", ["train", "test"])
def test_reconstruction_matches_reference_factors(gpu, split):
    d = os.path.join(GOLDEN, "bip", split)
    U, s, Vt = (np.load(os.path.join(d, f)) for f in ("svd_U.npy", "svd_s.npy", "svd_Vt.npy"))
    users = list(load(os.path.join(d, "user.json")))
    bus = list(load(os.path.join(d, "business.json")))
    row = {u: i for i, u in enumerate(users)}
    col = {b: i for i, b in enumerate(bus)}
    exp = load(os.path.join(d, "svd.json"))
    pairs = _flat(load(os.path.join(d, "examples.json")))
    dev = DeviceSVD(U * s, Vt.T)
    got = dev.score_pairs([row[u] for u, _ in pairs], [col[b] for _, b in pairs])
    want = np.array([exp[u][b] for u, b in pairs])
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("split", ["train", "test"])
def test_drop_in_svd_user_business(gpu, split, tmp_path, monkeypatch):
    shutil.copytree(os.path.join(GOLDEN, "bip", split), tmp_path / "data" / split)
    monkeypatch.chdir(tmp_path)
    S.svd_user_business(split, 8)
    got = load(str(tmp_path / "data" / split / "svd.json"))
    exp = load(os.path.join(GOLDEN, "bip", split, "svd.json"))
    assert list(got) == list(exp)
    for u in exp:
        assert list(got[u]) == list(exp[u])
        for b in exp[u]:
            assert isinstance(got[u][b], float)
            assert abs(got[u][b] - exp[u][b]) <= 1e-9 + 1e-6 * abs(exp[u][b])


@pytest.mark.parametrize("k", [8, 50, 64, 100])
def test_pairs_random_factors(gpu, k):
    rng = np.random.default_rng(k)
    us = rng.standard_normal((3000, k))
    v = rng.standard_normal((700, k))
    r = rng.integers(0, 3000, 20000)
    c = rng.integers(0, 700, 20000)
    got = DeviceSVD(us, v).score_pairs(r, c)
    want = np.einsum("ij,ij->i", us[r], v[c])
    scale = np.linalg.norm(us[r], axis=1) * np.linalg.norm(v[c], axis=1)
    assert np.all(np.abs(got - want) <= 1e-13 * scale)


def _np_topk(scores, topk, excl=None):
    out_c, out_s = [], []
    for i, row in enumerate(scores):
        cols = np.arange(len(row))
        keep = np.ones(len(row), bool)
        if excl is not None:
            keep[excl[i]] = False
        order = np.lexsort((cols[keep], -row[keep]))[:topk]
        out_c.append(cols[keep][order])
        out_s.append(row[keep][order])
    return np.array(out_c), np.array(out_s)


@pytest.mark.parametrize("k,n_cols,topk", [(64, 5003, 20), (50, 1200, 32), (16, 300, 7), (128, 2048, 20)])
def test_topk_vs_numpy(gpu, k, n_cols, topk):
    rng = np.random.default_rng(n_cols)
    us = rng.standard_normal((500, k))
    v = rng.standard_normal((n_cols, k))
    users = rng.choice(500, 150, replace=False).astype(np.int32)
    full = us[users] @ v.T
    ec, es = _np_topk(full, topk)
    dev = DeviceSVD(us, v)
    for prune in (True, False):
        dev.set_prune(prune)
        cols, sc = dev.topk(users, topk)
        np.testing.assert_array_equal(cols, ec)
        np.testing.assert_allclose(sc, es, rtol=1e-12, atol=1e-12)


def test_topk_ties_and_exclusions(gpu):
    rng = np.random.default_rng(9)
    # small integers: every dot product is exact in fp64, so ties are exact on both sides
    us = rng.integers(-3, 4, (64, 16)).astype(np.float64)
    base = rng.integers(-3, 4, (100, 16)).astype(np.float64)
    v = np.repeat(base, 5, axis=0)  # every score appears >= 5 times: ties broken by column
    users = np.arange(40, dtype=np.int32)
    excl = [np.sort(rng.choice(500, 30, replace=False)) for _ in users]
    off = np.r_[0, np.cumsum([len(e) for e in excl])]
    dev = DeviceSVD(us, v)
    full = us[users] @ v.T
    ec, es = _np_topk(full, 20, excl)
    for prune in (True, False):  # equal norms (repeated rows) and equal scores: column order decides
        dev.set_prune(prune)
        cols, sc = dev.topk(users, 20, exclude=(off, np.concatenate(excl)))
        np.testing.assert_array_equal(cols, ec)
    # more requested than available columns: trailing slots are -1
    small = DeviceSVD(us, v[:10])
    c2, _ = small.topk(users[:3], 15)
    assert (c2[:, 10:] == -1).all() and (c2[:, :10] >= 0).all()


def test_topk_device_matches_host_entry(gpu):
    """blp_svd_topk_device (device-resident inputs and outputs, handle-owned scratch) gives
    the lists of blp_svd_topk, with and without exclusions, across calls of different sizes."""
    import torch

    rng = np.random.default_rng(5)
    us = rng.standard_normal((300, 64))
    v = rng.standard_normal((2000, 64))
    dev = DeviceSVD(us, v)
    cuda = torch.device("cuda", 0)
    for n in (40, 150, 7):  # the scratch grows, then is reused
        users = rng.choice(300, n, replace=False).astype(np.int32)
        excl = [np.sort(rng.choice(2000, 12, replace=False)) for _ in users]
        off = np.r_[0, np.cumsum([len(e) for e in excl])].astype(np.int64)
        col = np.concatenate(excl).astype(np.int32)
        for ex in (None, (off, col)):
            hc, hs = dev.topk(users, 20, exclude=ex)
            dc = torch.empty((n, 20), dtype=torch.int32, device=cuda)
            ds = torch.empty((n, 20), dtype=torch.float64, device=cuda)
            dex = None if ex is None else (torch.from_numpy(off).to(cuda), torch.from_numpy(col).to(cuda))
            dev.topk_device(torch.from_numpy(users).to(cuda), 20, dc, ds, exclude=dex)
            dev.sync()
            np.testing.assert_array_equal(dc.cpu().numpy(), hc)
            np.testing.assert_array_equal(ds.cpu().numpy(), hs)


@pytest.mark.parametrize("n_cols,topk", [(30011, 20), (2500, 32), (2048 + 16, 5)])
def test_topk_pruned_equals_dense(gpu, n_cols, topk):
    """Norm pruning (blp_svd_set_prune, the default) gives the dense pass's lists bit for bit --
    scores and columns, with exclusions -- on factors whose column norms are skewed like a
    review graph's (a few popular businesses carry most of the mass), and scores far fewer
    MFMA tiles. Sizes: many pruned chunks; seed pass plus a short rest; one tile past the seed."""
    rng = np.random.default_rng(n_cols)
    k = 64
    us = rng.standard_normal((2000, k)) * rng.uniform(0.1, 3.0, (2000, 1))
    pop = 1.0 / np.arange(1, n_cols + 1) ** 0.8
    v = rng.standard_normal((n_cols, k)) * pop[rng.permutation(n_cols)][:, None]
    users = rng.choice(2000, 700, replace=False).astype(np.int32)
    excl = [np.sort(rng.choice(n_cols, int(rng.integers(0, 60)), replace=False)) for _ in users]
    off = np.r_[0, np.cumsum([len(e) for e in excl])].astype(np.int64)
    col = np.concatenate(excl).astype(np.int32)
    dev = DeviceSVD(us, v)
    dev.set_prune(False)
    dc, ds = dev.topk(users, topk, exclude=(off, col))
    dense_scored, dense_total = dev.tiles()
    assert dense_scored == dense_total > 0
    dev.set_prune(True)
    pc, ps = dev.topk(users, topk, exclude=(off, col))
    scored, total = dev.tiles()
    np.testing.assert_array_equal(pc, dc)
    np.testing.assert_array_equal(ps, ds)
    assert total == dense_total
    if n_cols > 20000:
        assert scored < 0.5 * total, (scored, total)
    full = us[users] @ v.T
    ec, es = _np_topk(full, topk, excl)
    np.testing.assert_array_equal(pc, ec)
    np.testing.assert_allclose(ps, es, rtol=1e-12, atol=1e-12)
