"""GPU truncated SVD (blp.factor.svds, csrc/factor.hip) vs scipy.sparse.linalg.svds -- the
reference's own factorisation (svd.py:24; SURVEY.md §8(f3): converged so that the
reconstructed scores agree far inside the 1e-5 bar; ARPACK agrees with itself to ~4e-10)."""
import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from blp import factor
from helpers import bipartite_edges

pytestmark = pytest.mark.gpu


def _matrix(seed, n_users, n_bus, draws):
    rng = np.random.default_rng(seed)
    u, b = bipartite_edges(rng, n_users, n_bus, draws)
    M = sp.csr_matrix((np.ones(len(u)), (u, b - n_users)), shape=(n_users, n_bus))
    M.sum_duplicates()
    M.data[:] = 1.0
    return M, rng


@pytest.mark.parametrize("k", [16, 50, 64])
def test_reconstruction_matches_arpack(gpu, k):
    M, rng = _matrix(1, 8000, 900, 80000)
    u, s, vt = spla.svds(M, k=k)
    ref_us = u * s
    st = factor.FactorStats()
    gu, gs, gvt = factor.svds(M, k=k, device=gpu, stats=st)
    assert st.iterations < 400 and st.converged_at is not None
    assert np.allclose(np.sort(gs), np.sort(s), rtol=1e-10, atol=0)
    rows = rng.integers(0, M.shape[0], 20000)
    cols = rng.integers(0, M.shape[1], 20000)
    ref = np.einsum("ij,ji->i", ref_us[rows], vt[:, cols])
    got = np.einsum("ij,ji->i", (gu * gs)[rows], gvt[:, cols])
    assert np.max(np.abs(got - ref)) <= 1e-9 * np.max(np.abs(ref))
    # right singular vectors orthonormal
    assert np.allclose(gvt @ gvt.T, np.eye(k), atol=1e-10)


@pytest.mark.parametrize("k", [16, 64])
def test_per_entry_parity_vs_arpack(gpu, k):
    """Every reconstructed entry of the GPU factorisation (the svd.py default) against the
    reference's ARPACK factorisation at 1e-5 relative per entry, with the exact-zero rule
    for empty rows / columns and the near-zero floor (blp_oracle.svd_entry_parity)."""
    import blp_oracle as O

    M, rng = _matrix(5, 6000, 700, 60000)
    # users and businesses with no reviews: their scores are exactly 0 (structural zeros)
    M = sp.vstack([M, sp.csr_matrix((40, M.shape[1]))]).tocsr()
    M = sp.hstack([M, sp.csr_matrix((M.shape[0], 9))]).tocsr()
    u, s, vt = spla.svds(M, k=k)
    ref_us = u * s
    gus, gs, gv = factor.svds(M, k=k, device=gpu, return_us=True)
    rows = np.r_[rng.integers(0, M.shape[0], 30000), np.arange(M.shape[0] - 40, M.shape[0])]
    cols = np.r_[rng.integers(0, M.shape[1], 30000), rng.integers(0, M.shape[1], 40)]
    cols[:50] = M.shape[1] - 1 - np.arange(50) % 9  # some empty columns
    ref = np.einsum("ij,ji->i", ref_us[rows], vt[:, cols])
    got = np.einsum("ij,ij->i", gus[rows], gv[cols])
    zero = (np.diff(M.indptr)[rows] == 0) | (np.diff(M.tocsc().indptr)[cols] == 0)
    r = O.svd_entry_parity(got, ref, zero)
    assert r["structural_zeros"] >= 80
    assert r["ok"], r


def test_return_us_layout_and_determinism(gpu):
    M, _ = _matrix(2, 5000, 600, 50000)
    us1, s1, v1 = factor.svds(M, k=32, device=gpu, return_us=True)
    us2, s2, v2 = factor.svds(M, k=32, device=gpu, return_us=True)
    assert np.array_equal(us1, us2) and np.array_equal(v1, v2) and np.array_equal(s1, s2)
    assert np.all(np.diff(s1) <= 0)  # descending
    assert np.allclose(M @ v1, us1, rtol=0, atol=1e-9 * np.abs(us1).max())  # us = M v


def test_rejects_bad_input(gpu):
    M, _ = _matrix(3, 300, 200, 3000)
    with pytest.raises(ValueError):
        factor.svds(M * 2.0, k=8, device=gpu)  # not binary
    with pytest.raises(ValueError):
        factor.svds(M[:, :100], k=8, device=gpu)  # fewer columns than the block


def test_svd_drop_in_gpu_factor_matches_host(gpu, tmp_path, monkeypatch):
    """svd.svd_user_business (svd.py:7-31) with the GPU factorisation vs the reference's own
    scipy ARPACK: the written svd.json scores agree to 1e-9 of the score scale."""
    import json

    import svd as S

    rng = np.random.default_rng(4)
    u, b = bipartite_edges(rng, 3000, 400, 30000)
    d = tmp_path / "data" / "t"
    d.mkdir(parents=True)
    users = [str(x) for x in rng.permutation(np.unique(u))]
    bus = [str(x) for x in rng.permutation(np.unique(b))]
    (d / "user.json").write_text(json.dumps({x: 1 for x in users}))
    (d / "business.json").write_text(json.dumps({x: 1 for x in bus}))
    (d / "graph.txt").write_text("".join("%d %d\n" % e for e in zip(u.tolist(), b.tolist())))
    ex = {}
    for x in users[:60]:
        ex[x] = {y: 0 for y in rng.choice(bus, 30, replace=False)}
    (d / "examples.json").write_text(json.dumps(ex))
    monkeypatch.chdir(tmp_path)
    got = S.svd_user_business("t", k=32, device=gpu, factor="gpu")
    (d / "examples.json").write_text(json.dumps(ex))
    ref = S.svd_user_business("t", k=32, device=gpu, factor="host")
    g = np.array([v for x in got for v in got[x].values()])
    r = np.array([v for x in ref for v in ref[x].values()])
    assert list(got) == list(ref)
    assert np.max(np.abs(g - r)) <= 1e-9 * np.max(np.abs(r))
