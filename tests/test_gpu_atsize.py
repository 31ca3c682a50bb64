"""At-size parity in the GPU suite for BASELINE.json configs 1, 3, 4 and 5 (config 2 is
tests/test_gpu_headline.py). Each test builds the config's own synthetic graph (SURVEY.md
§8(d)), asserts the launch geometry it claims to cover, and checks the engine bit-exact
against the C oracle (the reference algorithm, similarity.py:20-126) or fp64 numpy on the same
factors (svd.py:28-30). Marked `gpu`.

  config 1  similarity.main (similarity.py:11-18) on the Yelp-sized synthetic: every file
  config 3  full-candidate top-k on the 10M-edge graph (hop-3 set, dataset_maker.py:139)
  config 4  rank-64 SVD top-k on the 2M x 200K, 50M-draw matrix: dense MFMA and norm-pruned
  config 5  the 50M-user x 2M-business universe: 48 chunk-parallel 128 KiB chunks on the user
            side, the hash-set partition on the business side -- a fast geometry check on 100M
            of the draws, and the full 1B draws through the RCCL exchange (blp_multi_gather_csr)
"""
import os

import numpy as np
import pytest

import blp
import coracle
from blp import synth

pytestmark = pytest.mark.gpu

NT = max(1, len(os.sched_getaffinity(0)))


def _exact_topk(scores, ids, k):
    """Positions of the best k (score descending, then id ascending), ties included exactly."""
    n = len(scores)
    if n > k:
        vk = -np.partition(-scores, k - 1)[k - 1]
        cand = np.flatnonzero(scores >= vk)
    else:
        cand = np.arange(n)
    return cand[np.lexsort((ids[cand], -scores[cand]))][:k]


def _oracle(G):
    """C oracle over the engine graph's own edges, on its dense ids."""
    n0 = G.n_col0
    rows = np.repeat(np.arange(n0, dtype=np.int64), np.diff(G.row_ptr[: n0 + 1]))
    cols = G.col_idx[: G.row_ptr[n0]]
    return coracle.OracleGraph(G.n, rows.astype(np.int32), cols.astype(np.int32))


# ------------------------------------------------------------------------------ config 1
def test_config1_similarity_main_yelp_sized(gpu, tmp_path):
    """similarity.main from graph.txt + examples.json to the six files on the Yelp-sized
    synthetic (252,898 x 42,153, 1,125,458 draws; writeups/proposal.tex:93), 10K example users:
    every file's values equal the oracle's, ints and floats where the reference writes them
    (CN ints, AA int 0 for an empty sum, b_adamic only the missing-node zeros)."""
    import pandas as pd

    import similarity
    import util

    U, B, D = synth.CONFIGS["yelp"]
    a, b = synth.review_edges(U, B, D, seed=0)
    gpath = str(tmp_path / "graph.txt")
    pd.DataFrame({"u": a, "b": b}).to_csv(gpath, sep="\t", header=False, index=False)
    G = blp.DeviceGraph(a, b, device=gpu)
    ex_x, ex_y, ex_l = synth.make_examples(G, U, B, D, n_users=10_000, rate=0.01, seed=0)
    assert len(ex_x) > 500_000 and len(np.unique(ex_x)) > 9_000
    # two absent nodes: a user and a business that are not in graph.txt (similarity.py:59-60, 104-105)
    uid, bid = G.node_ids[ex_x].tolist(), G.node_ids[ex_y].tolist()
    examples = {}
    for u, v, l in zip(uid, bid, ex_l.tolist()):
        examples.setdefault(str(u), {})[str(v)] = int(l)
    first = next(iter(examples))
    examples[first][str(U + B + 7)] = 0
    examples[str(U + B + 9)] = {str(bid[0]): 1}
    epath = str(tmp_path / "examples.json")
    util.write_json(examples, epath)
    og = _oracle(G)
    present = [(int(u), int(v)) for u in examples for v in examples[u]]
    G.close()
    del G
    methods = ["common_neighbors", "jaccard", "adamic_adar"]
    uf = [str(tmp_path / f) for f in ("u_cn.json", "u_jaccard.json", "u_adamic.json")]
    bf = [str(tmp_path / f) for f in ("b_cn.json", "b_jaccard.json", "b_adamic.json")]
    similarity.main(epath, gpath, methods, uf, methods, bf)
    # the oracle on the file's own pair order; absent nodes -> int 0
    ids = np.unique(np.concatenate([a, b]))
    pos = {int(v): i for i, v in enumerate(ids)}
    ok = np.array([u in pos and v in pos for u, v in present])
    xo = np.array([pos.get(u, 0) for u, _ in present], np.int32)
    yo = np.array([pos.get(v, 0) for _, v in present], np.int32)
    n0 = int((ids < U).sum())
    assert np.all(xo[ok] < n0) and np.all(yo[ok] >= n0)
    # the oracle graph's ids are the engine's dense ids: users first, then businesses, ascending
    ucn, ujac, uaa, _ = og.score_pairs(xo[ok], yo[ok], 7, nthreads=NT)
    bcn, bjac, _, _ = og.score_pairs(yo[ok], xo[ok], 3, nthreads=NT)

    def expect(vals, int0):
        out, it = [], iter(vals.tolist())
        for p in ok:
            if not p:
                out.append(0)
            else:
                v = next(it)
                out.append(0 if int0 and v == 0.0 else v)
        return out

    for f, want in ((uf[0], expect(ucn, False)), (uf[1], expect(ujac, False)), (uf[2], expect(uaa, True)),
                    (bf[0], expect(bcn, False)), (bf[1], expect(bjac, False))):
        got = [v for u in util.load_json(f).values() for v in u.values()]
        assert got == want, f
        assert all(type(g) is type(w) for g, w in zip(got, want)), f
    bad = util.load_json(bf[2])  # the b_adamic bug (similarity.py:102): only the absent-node zeros
    assert sum(len(v) for v in bad.values()) == int((~ok).sum())
    assert all(v == 0 and type(v) is int for u in bad.values() for v in u.values())


# ------------------------------------------------------------------------------ config 3
@pytest.fixture(scope="module")
def c2_graph(request):
    dev = int(os.environ.get("BLP_DEVICE", "0"))
    U, B, D = synth.CONFIGS["c2"]
    a, b = synth.review_edges(U, B, D, seed=0)
    G = blp.DeviceGraph(a, b, device=dev)
    yield G
    G.close()


def test_config3_topk_at_size(gpu, c2_graph):
    """Config 3 on the 10M-edge config-2 graph: 64 sampled users' EVERY exact hop-3 business
    scored by blp.TopK (Jaccard + Adamic-Adar, k = 20); the handle's geometry (u32 / u16
    counter tiers, wedge rows, dense hot-target counts in play); lists, scores and |H3| equal
    the C oracle's (og_hop3 + the reference scorers, ranked score desc / id asc), and the AA
    values equal the pair kernel's."""
    from blp.topk import TopK

    G = c2_graph
    U = synth.CONFIGS["c2"][0]
    G.n_users_hint = U
    src = synth.sample_users(G, 64, seed=3)
    T = TopK(G, "user")
    info = T.info()
    assert info["tier32"] > 0 and info["tier16"] > 0 and info["wedge_entries"] > 0, info
    T.set_sources(src)
    T.run(20, blp.JACCARD | blp.ADAMIC)
    cj, sj, ncand = T.fetch("jaccard")
    ca, sa, _ = T.fetch("adamic_adar")
    assert T.stats(7)[1] > 0  # dense hot-target adds (the config-3 fast path) were taken
    og = _oracle(G)
    counts, mem = og.hop3(src)
    np.testing.assert_array_equal(ncand, counts)
    assert counts.sum() > 64 * 40_000  # ~70K of 100K businesses per user
    xrep = np.repeat(src, counts).astype(np.int32)
    _, jac, aa, _ = og.score_pairs(xrep, mem, 7, nthreads=NT)
    starts = np.r_[0, np.cumsum(counts)]
    for i in range(len(src)):
        s, e = starts[i], starts[i + 1]
        o = _exact_topk(jac[s:e], mem[s:e], 20)
        np.testing.assert_array_equal(cj[i], mem[s:e][o])
        np.testing.assert_array_equal(sj[i], jac[s:e][o])
        o = _exact_topk(aa[s:e], mem[s:e], 20)
        np.testing.assert_array_equal(ca[i], mem[s:e][o])
        np.testing.assert_array_equal(sa[i], aa[s:e][o])
    pair = G.score_pairs(np.repeat(src, 20).astype(np.int32), ca.reshape(-1).astype(np.int32), 7)["adamic"]
    np.testing.assert_array_equal(pair, sa.reshape(-1))
    # the block-round CN / Jaccard selection (BLP_TK_WAVESEL=0; the per-wave one is the default)
    # gives the same lists at size
    import os

    os.environ["BLP_TK_WAVESEL"] = "0"
    try:
        T.run(20, blp.JACCARD | blp.ADAMIC)
        for m, (c0, s0) in (("jaccard", (cj, sj)), ("adamic_adar", (ca, sa))):
            c1, s1, n1 = T.fetch(m)
            np.testing.assert_array_equal(c1, c0)
            np.testing.assert_array_equal(s1, s0)
            np.testing.assert_array_equal(n1, ncand)
    finally:
        del os.environ["BLP_TK_WAVESEL"]
    T.close()


# ------------------------------------------------------------------------------ config 4
def test_config4_svd_topk_at_size(gpu):
    """Config 4: the 2M x 200K binary matrix of 50M draws, rank-64 factors from the GPU
    factorisation (blp.factor.svds), 128 users' top-20 over all 200K businesses (own reviews
    excluded) on fp64 MFMA: the dense pass scores every 16 x 16 tile, the norm-pruned pass
    (the library default) skips most of them; both lists equal the exact fp64 numpy ranking on
    the same factors (np.dot(us[row], vt[:, col]), svd.py:28-30), bit for bit."""
    import scipy.sparse as sp

    from blp import factor as F
    from blp.factor import DeviceSVD

    U, B, D = synth.CONFIGS["c4"]
    u, b = synth.review_edges(U, B, D, seed=0)
    M = sp.csr_matrix((np.ones(len(u), np.float64), (u, b - U)), shape=(U, B))
    del u, b
    M.sum_duplicates()
    M.data[:] = 1.0
    assert M.shape == (2_000_000, 200_000) and M.nnz > 49_000_000
    us, s, v = F.svds(M, k=64, device=gpu, return_us=True)
    assert us.shape == (U, 64) and v.shape == (B, 64)
    rng = np.random.default_rng(4)
    deg = np.diff(M.indptr)
    users = np.sort(rng.choice(np.flatnonzero(deg > 0), 128, replace=False)).astype(np.int32)
    ex_off = np.r_[0, np.cumsum(deg[users])].astype(np.int64)
    ex_col = np.concatenate([M.indices[M.indptr[r]:M.indptr[r + 1]] for r in users]).astype(np.int32)
    S = DeviceSVD(us, np.ascontiguousarray(v), device=gpu)
    S.set_prune(False)
    S.tiles()
    dc, ds = S.topk(users, 20, exclude=(ex_off, ex_col))
    scored, dense = S.tiles()
    assert scored == dense > 0  # every MFMA tile
    S.set_prune(True)
    pc, ps = S.topk(users, 20, exclude=(ex_off, ex_col))
    scored, dense = S.tiles()
    assert scored < dense // 4, (scored, dense)  # pruning skipped most tiles
    np.testing.assert_array_equal(pc, dc)
    np.testing.assert_array_equal(ps, ds)
    full = us[users] @ np.ascontiguousarray(v.T)
    bids = np.arange(B)
    for i in range(len(users)):
        full[i, ex_col[ex_off[i]:ex_off[i + 1]]] = -np.inf
        o = _exact_topk(full[i], bids, 20)
        np.testing.assert_array_equal(dc[i], o)
        # the same 64-term dots summed in another order (MFMA vs BLAS): north_star's 1e-5 relative
        np.testing.assert_allclose(ds[i], full[i, o], rtol=1e-12, atol=0)


# ------------------------------------------------------------------------------ config 5
def test_config5_geometry_at_size(gpu):
    """Config 5's universe: 50M users x 2M businesses, 100M of the 1B draws (row-block
    generator, dist.block_review_edges, one block), the CSR built in HBM from device
    endpoints (the post-exchange path). 20 user sources' candidate pairs (every business
    outside N(u) kept at 0.01) run on the chunk-parallel scorer over 48 chunks of 128 KiB;
    their businesses, as business-side sources, run through the hash-set partition plus the
    chunk-parallel scorer. Every pair of both passes (the 20 user sources and their >100K
    business sources) is checked bit-exact against the C oracle over the same edges (CN,
    Jaccard, and AA on the user side)."""
    import torch

    from blp import dist as bd

    U, B, _ = synth.CONFIGS["c5"]
    D = 100_000_000
    u, b = bd.block_review_edges(U, B, D, 0, U, seed=0)
    ta = torch.from_numpy(u.astype(np.int32)).cuda(gpu)
    tb = torch.from_numpy(b.astype(np.int32)).cuda(gpu)
    G = blp.DeviceGraph.from_device_edges(ta.data_ptr(), tb.data_ptr(), len(u), U + B, U, device=gpu)
    del ta, tb
    torch.cuda.empty_cache()
    rng = np.random.default_rng(55)
    cand = np.flatnonzero(G.hop1_size[:U] >= 4)
    src = np.sort(rng.choice(cand, 20, replace=False)).astype(np.int32)
    ex_x, ex_y = synth.uniform_examples(G, src, rate=0.01, seed=5)
    assert len(ex_x) > 20 * 15_000
    ub, bb = G.batch(ex_x, ex_y), G.batch(ex_y, ex_x)
    pu, pb = ub.plan(), bb.plan()
    assert pu["chunks"] == -48 and pu["hi"] - pu["lo"] > 45_000_000, pu  # 48 x 128 KiB chunks
    assert pb["chunks"] < 0 and pb["hash_sources"] > 0, pb  # hash-set partition + chunk-parallel
    ub.score(7)
    bb.score(3)
    gu, gb = ub.fetch(7), bb.fetch(3)
    og = coracle.OracleGraph(U + B, u.astype(np.int32), b.astype(np.int32))
    del u, b
    cn, jac, aa, _ = og.score_pairs(ex_x, ex_y, 7, nthreads=NT)  # the 20 user sources: every pair
    np.testing.assert_array_equal(gu["cn"], cn)
    np.testing.assert_array_equal(gu["jaccard"], jac)
    np.testing.assert_array_equal(gu["adamic"], aa)
    assert pb["sources"] > 100_000
    cn, jac, _, _ = og.score_pairs(ex_y, ex_x, 3, nthreads=NT)  # every business source's pairs
    np.testing.assert_array_equal(gb["cn"], cn)
    np.testing.assert_array_equal(gb["jaccard"], jac)
    for bt in (ub, bb):
        bt.close()
    G.close()


def test_config5_full_1b_draws_through_rccl_exchange(gpu):
    """Config 5's own workload (BASELINE.json configs[4]): the 50M-user x 2M-business universe
    with ALL 1B draws (dataset_maker.py:139 / similarity.py:20-106 at that scale). The row-block
    generator (dist.block_review_edges) makes the partial of the whole user range -- world 1 --
    and it goes through the exchange the N-GPU bench runs: libblp's own RCCL communicator
    (blp_multi_gather_csr: counts, then the padded partials in one ncclAllGather, the CSR built
    in HBM), then the graph handle over that device CSR. Checked:
      - the gathered union CSR equals the C oracle's CSR of the same 1B edges (built on the host,
        independently: row pointers and every column id), so every duplicate was merged once;
      - the plan: 48 chunk-parallel 128 KiB chunks on the user side, the hash-set partition on
        the business side;
      - 24 user sources (every candidate pair: CN, Jaccard, AA), and 5,000 of the >100K business
        sources of the transposed list (every pair of each: CN, Jaccard), bit-exact against the
        oracle on that graph.
    Runtime on one MI355X box: see DESIGN.md §6 (config 5 parity in the suite)."""
    import time

    from blp import dist as bd
    from blp.multi import Multi

    U, B, D = synth.CONFIGS["c5"]
    t0 = time.time()
    u, b = bd.block_review_edges(U, B, D, 0, U, seed=0)
    u = u.astype(np.int32)
    b = b.astype(np.int32)
    assert len(u) == D
    t_gen = time.time() - t0
    with bd.stdout_to_stderr():  # RCCL's banner
        m = Multi(Multi.unique_id(), 1, 0, gpu)
    t0 = time.time()
    c = m.gather_csr(u, b, U + B)
    t_x = time.time() - t0
    assert m.bytes_in == 0  # world 1: nothing arrives from another rank
    m.close()
    G = blp.DeviceGraph.from_csr_handle(c, U + B, U, device=gpu)
    t0 = time.time()
    og = coracle.OracleGraph(U + B, u, b)
    t_og = time.time() - t0
    del u, b
    orp, oci = og.csr()
    assert G.nnz == len(oci) and G.nnz > 1_990_000_000
    np.testing.assert_array_equal(G.row_ptr, orp)
    assert np.array_equal(G.col_idx, oci)  # 2G column ids: the union CSR is the oracle's
    rng = np.random.default_rng(77)
    cand = np.flatnonzero(G.hop1_size[:U] >= 4)
    src = np.sort(rng.choice(cand, 24, replace=False)).astype(np.int32)
    ex_x, ex_y = synth.uniform_examples(G, src, rate=0.01, seed=11)
    assert len(ex_x) > 24 * 15_000
    ub, bb = G.batch(ex_x, ex_y), G.batch(ex_y, ex_x)
    pu, pb = ub.plan(), bb.plan()
    assert pu["chunks"] == -48 and pu["hi"] - pu["lo"] > 45_000_000, pu
    assert pb["chunks"] < 0 and pb["hash_sources"] > 0 and pb["sources"] > 100_000, pb
    t0 = time.time()
    G.score_batches([(ub, 7), (bb, 3)])
    gu, gb = ub.fetch(7), bb.fetch(3)
    t_sc = time.time() - t0
    t0 = time.time()
    cn, jac, aa, _ = og.score_pairs(ex_x, ex_y, 7, nthreads=NT)
    np.testing.assert_array_equal(gu["cn"], cn)
    np.testing.assert_array_equal(gu["jaccard"], jac)
    np.testing.assert_array_equal(gu["adamic"], aa)
    # business side: every pair of 5,000 sampled business sources (hash-set and chunk-parallel routes)
    bsrc = rng.choice(np.unique(ex_y), 5000, replace=False)
    sel = np.flatnonzero(np.isin(ex_y, bsrc))
    cn, jac, _, _ = og.score_pairs(ex_y[sel], ex_x[sel], 3, nthreads=NT)
    np.testing.assert_array_equal(gb["cn"][sel], cn)
    np.testing.assert_array_equal(gb["jaccard"][sel], jac)
    t_or = time.time() - t0
    print("config5 1B: generate %.1fs, exchange+CSR %.1fs, oracle graph %.1fs, score %.2fs, oracle score %.1fs, "
          "%d + %d pairs (%d business pairs checked)" % (t_gen, t_x, t_og, t_sc, t_or, len(ex_x), len(ex_y), len(sel)))
    for bt in (ub, bb):
        bt.close()
    G.close()
