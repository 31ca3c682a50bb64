"""GPU parity of the config-5 ingest path: device-resident endpoints ->
blp_csr_build_device -> blp_graph_create_from_csr (DeviceGraph.from_device_edges), against
the host CSR builder (blp_csr_from_edges, SNAP LoadEdgeList semantics, similarity.py:16)
and the C oracle; then the sharded-universe scorers on the resulting graph. Marked `gpu`.

The exchange itself (blp.dist.allgather_edges) runs here three ways: at world 1 on the
device without a process group; through RCCL (backend "nccl", all_gather_into_tensor) over a
one-rank process group, the same code N ranks run; and at world 2 with two processes sharing
the one GPU (gloo carries that exchange: RCCL refuses two ranks on one device)."""
import ctypes
import os
import socket

import numpy as np
import pytest

import blp
import coracle
from blp import dist as bd
from helpers import bipartite_edges, dense_edges

pytestmark = pytest.mark.gpu


def _host_csr(n, a, b):
    A = np.ascontiguousarray(a, np.int32)
    B = np.ascontiguousarray(b, np.int32)
    rp = np.zeros(n + 1, np.int64)
    ci = np.empty(max(2 * len(A), 1), np.int32)
    sl = np.zeros(max(n, 1), np.uint8)
    nnz = ctypes.c_int64(0)
    P = blp._lib.ptr
    blp._lib.check(blp.lib().blp_csr_from_edges(n, len(A), P(A), P(B), P(rp), P(ci), P(sl), ctypes.byref(nnz)))
    return rp, ci[: nnz.value], sl[:n]


def _on_device(*arrs):
    import torch

    out = [torch.from_numpy(np.ascontiguousarray(x, np.int32)).cuda() for x in arrs]
    return out


def _messy_edges(rng, n_users, n_bus, draws):
    """Review edges plus duplicates, reversed duplicates and self-loops (dense ids)."""
    u, b = bipartite_edges(rng, n_users, n_bus, draws)
    k = draws // 10
    i = rng.integers(0, draws, k)
    loops = rng.integers(0, n_users + n_bus, 25)
    a = np.concatenate([u, u[i], b[i[: k // 2]], loops])
    c = np.concatenate([b, b[i], u[i[: k // 2]], loops])
    perm = rng.permutation(len(a))
    return a[perm], c[perm]


@pytest.mark.parametrize("seed,n_users,n_bus,draws", [(0, 3000, 200, 20000), (1, 200000, 6000, 900000)])
def test_device_csr_equals_host_csr(gpu, seed, n_users, n_bus, draws):
    rng = np.random.default_rng(seed)
    a, c = _messy_edges(rng, n_users, n_bus, draws)
    n = n_users + n_bus
    rp, ci, sl = _host_csr(n, a, c)
    da, dc = _on_device(a, c)
    G = blp.DeviceGraph.from_device_edges(da.data_ptr(), dc.data_ptr(), len(a), n, n_users, device=gpu)
    assert np.array_equal(G.row_ptr, rp) and np.array_equal(G.col_idx, ci) and np.array_equal(G.self_loop, sl)
    assert sl.sum() > 0 and G.nnz == len(ci)
    assert set(G.build_times) == {"device_csr_s", "fetch_s", "host_half_s", "graph_create_s"}
    # the older entry point (host outputs) is the same builder
    rp2 = np.zeros(n + 1, np.int64)
    ci2 = np.empty(2 * len(a), np.int32)
    sl2 = np.zeros(n, np.uint8)
    nnz = ctypes.c_int64(0)
    P = blp._lib.ptr
    blp._lib.check(blp.lib().blp_csr_from_edges_device(gpu, ctypes.c_void_p(da.data_ptr()), ctypes.c_void_p(
        dc.data_ptr()), len(a), n, P(rp2), P(ci2), P(sl2), ctypes.byref(nnz)))
    assert np.array_equal(rp2, rp) and np.array_equal(ci2[: nnz.value], ci) and np.array_equal(sl2, sl)


def test_device_csr_rejects_out_of_range_ids(gpu):
    a = np.array([0, 1, 5], np.int32)
    c = np.array([3, 2, 9], np.int32)  # 9 >= n
    da, dc = _on_device(a, c)
    with pytest.raises(blp.BLPError) as e:
        blp.DeviceGraph.from_device_edges(da.data_ptr(), dc.data_ptr(), 3, 8, 4, device=gpu)
    assert e.value.code == -1  # BLP_E_ARG
    a[2] = -1
    c[2] = 3
    da, dc = _on_device(a, c)
    with pytest.raises(blp.BLPError) as e:
        blp.DeviceGraph.from_device_edges(da.data_ptr(), dc.data_ptr(), 3, 8, 4, device=gpu)
    assert e.value.code == -1


def test_device_csr_empty_and_loops_only(gpu):
    da, dc = _on_device(np.array([2, 2], np.int32), np.array([2, 2], np.int32))
    G = blp.DeviceGraph.from_device_edges(da.data_ptr(), dc.data_ptr(), 2, 5, 3, device=gpu)
    assert G.nnz == 0 and G.row_ptr.tolist() == [0] * 6 and G.self_loop.tolist() == [0, 0, 1, 0, 0]
    assert G.degree.tolist() == [0, 0, 1, 0, 0]


@pytest.mark.parametrize("knobs", [{}, {"BLP_SPLIT": "3"}, {"BLP_FORCE_GLOBAL": "1"}])
def test_device_graph_scores_match_oracle(gpu, knobs, monkeypatch):
    """Scores on the adopted device CSR: the default plan, the chunk-parallel scorer (the
    config-5 user side) and the HBM-bitmap scorer, vs the C oracle and vs a host-built graph."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(5)
    n_users, n_bus = 40000, 1200
    a, c = _messy_edges(rng, n_users, n_bus, 300000)
    n = n_users + n_bus
    da, dc = _on_device(a, c)
    G = blp.DeviceGraph.from_device_edges(da.data_ptr(), dc.data_ptr(), len(a), n, n_users, device=gpu)
    users = rng.choice(np.flatnonzero(G.hop1_size[:n_users] > 0), 120, replace=False)
    x = np.repeat(users, 25).astype(np.int32)
    y = rng.integers(n_users, n, len(x)).astype(np.int32)
    y = y[G.hop1_size[y] > 0]
    x = x[: len(y)]
    ids, oa, ob = dense_edges(a, c)
    og = coracle.OracleGraph(len(ids), oa, ob)
    for xs, ys, mask in ((x, y, 7), (y, x, 3)):
        got = G.score_pairs(xs, ys, mask)
        cn, jac, aa, _ = og.score_pairs(np.searchsorted(ids, xs), np.searchsorted(ids, ys), mask, nthreads=8)
        np.testing.assert_array_equal(got["cn"], cn)
        np.testing.assert_array_equal(got["jaccard"], jac)
        if mask & blp.ADAMIC:
            np.testing.assert_array_equal(got["adamic"], aa)  # exact sums: bit-exact
    if "BLP_SPLIT" in knobs:
        assert G.batch(x, y).plan()["chunks"] == -3
    if "BLP_FORCE_GLOBAL" in knobs:
        assert G.batch(x, y).plan()["chunks"] == 0
    # the same graph built from host arrays scores identically (Adamic-Adar included)
    H = blp.DeviceGraph.from_csr(G.row_ptr.copy(), G.col_idx.copy(), G.self_loop.copy(), n_users, device=gpu)
    for k, v in G.score_pairs(x, y, 7).items():
        np.testing.assert_array_equal(v, H.score_pairs(x, y, 7)[k])


@pytest.mark.parametrize("seed,sparse_ids", [(0, False), (1, True)])
def test_device_graph_from_ids_device_csr(gpu, seed, sparse_ids, monkeypatch):
    """DeviceGraph(a_ids, b_ids) -- similarity.main's graph.txt load -- builds large edge lists'
    CSR on the device (blp_csr_build_host): id map, CSR, degrees, weights and scores equal the
    host-CSR build of the same ids (duplicates, reversed duplicates, self-loops included)."""
    rng = np.random.default_rng(seed)
    n_users, n_bus = 30000, 900
    a, c = _messy_edges(rng, n_users, n_bus, 200000)
    if sparse_ids:  # original ids far apart: the sorted unique path and the searchsorted lookup
        a = a.astype(np.int64) * 7919 + 10**9
        c = c.astype(np.int64) * 7919 + 10**9
    else:
        a = a.astype(np.int64) + 12
        c = c.astype(np.int64) + 12
    monkeypatch.setenv("BLP_DEVICE_CSR_MIN", str(1 << 40))
    H = blp.DeviceGraph(a, c, device=gpu)
    monkeypatch.setenv("BLP_DEVICE_CSR_MIN", "1")
    G = blp.DeviceGraph(a, c, device=gpu)
    assert "device_csr_s" in G.build_times and "device_csr_s" not in H.build_times  # which path built each
    for k in ("node_ids", "row_ptr", "col_idx", "self_loop", "degree", "aa_weight"):
        assert np.array_equal(getattr(G, k), getattr(H, k)), k
    assert G.n_col0 == H.n_col0 and G.n == H.n and G.self_loop.sum() > 0
    users = rng.choice(G.node_ids[: G.n_col0][G.hop1_size[: G.n_col0] > 0], 60, replace=False)
    x = np.repeat(G.dense(users), 20).astype(np.int32)
    y = rng.integers(G.n_col0, G.n, len(x)).astype(np.int32)
    y = y[G.hop1_size[y] > 0]
    x = x[: len(y)]
    for xs, ys, mask in ((x, y, 7), (y, x, 7)):
        rg, rh = G.score_pairs(xs, ys, mask), H.score_pairs(xs, ys, mask)
        for k in rg:
            np.testing.assert_array_equal(rg[k], rh[k])


def test_csr_build_host_entry_point(gpu):
    """blp_csr_build_host: host endpoints -> device CSR, equal to the host builder; empty edge
    lists and self-loop-only lists; out-of-range ids rejected with BLP_E_ARG."""
    L, P = blp.lib(), blp._lib.ptr

    def build(a, c, n):
        A = np.ascontiguousarray(a, np.int32)
        C = np.ascontiguousarray(c, np.int32)
        h = ctypes.c_void_p()
        blp._lib.check(L.blp_csr_build_host(gpu, P(A) if len(A) else None, P(C) if len(C) else None, len(A), n,
                                            ctypes.byref(h)))
        try:
            nn, nnz = ctypes.c_int64(), ctypes.c_int64()
            blp._lib.check(L.blp_csr_info(h, ctypes.byref(nn), ctypes.byref(nnz)))
            rp = np.empty(n + 1, np.int64)
            ci = np.empty(max(nnz.value, 1), np.int32)
            sl = np.empty(max(n, 1), np.uint8)
            blp._lib.check(L.blp_csr_fetch(h, P(rp), P(ci), P(sl)))
            return rp, ci[: nnz.value], sl[:n]
        finally:
            L.blp_csr_destroy(h)

    rng = np.random.default_rng(11)
    a, c = _messy_edges(rng, 5000, 300, 40000)
    got = build(a, c, 5300)
    for g_, e_ in zip(got, _host_csr(5300, a, c)):
        assert np.array_equal(g_, e_)
    rp, ci, sl = build([], [], 4)
    assert rp.tolist() == [0] * 5 and len(ci) == 0 and sl.tolist() == [0] * 4
    rp, ci, sl = build([1, 3], [1, 3], 4)
    assert rp.tolist() == [0] * 5 and sl.tolist() == [0, 1, 0, 1]
    with pytest.raises(blp.BLPError) as e:
        build([0, 7], [1, 2], 5)
    assert e.value.code == -1


@pytest.mark.parametrize("device_csr,items", [(False, False), (True, False), (True, True)])
def test_wedge_rows_equal_host_construction(gpu, device_csr, items, monkeypatch):
    """The wedge-row index (gathered on the device, k_wedge_fill) equals its definition built
    here from the CSR: for every node whose neighbours' rows all hold <= 64 ids, the rows N(z),
    z in N(x), back to back, padded to whole vectors with the last id. Businesses here have
    ~400 neighbours, so one node spans several 256-neighbour rounds. items: the hub-node fill
    (k_wedge_fill_items: items of <= 4096 members, rows of a node in item order, padding a
    repeat of the node's first stored id) -- the same multiset per node."""
    monkeypatch.setenv("BLP_DEVICE_CSR_MIN", "1" if device_csr else str(1 << 40))
    if items:
        monkeypatch.setenv("BLP_WEDGE_ITEMS", "1")
    rng = np.random.default_rng(17)
    a, c = bipartite_edges(rng, 3000, 100, 40000)
    G = blp.DeviceGraph(a, c, device=gpu)
    nv = ctypes.c_int64()
    blp._lib.check(blp.lib().blp_graph_wedge(G.handle, ctypes.byref(nv), None, None))
    assert nv.value > 0
    wp = np.empty(G.n + 1, np.int64)
    wd = np.empty(4 * nv.value, np.int32)
    blp._lib.check(blp.lib().blp_graph_wedge(G.handle, ctypes.byref(nv), blp._lib.ptr(wp), blp._lib.ptr(wd)))
    rp, ci = G.row_ptr, G.col_idx
    deg = np.diff(rp)
    exp_wp = [0]
    exp = []
    for x in range(G.n):
        nb = ci[rp[x]: rp[x + 1]]
        row = []
        n_ids = 0
        if len(nb) and deg[nb].max() <= 64:
            for z in nb:
                row.extend(ci[rp[z]: rp[z + 1]].tolist())
            n_ids = len(row)
            row.extend([row[-1]] * (-len(row) % 4))
        if items and n_ids:
            got = wd[4 * wp[x]: 4 * wp[x + 1]]
            assert sorted(got[:n_ids].tolist()) == sorted(row[:n_ids]) and (got[n_ids:] == got[0]).all()
        exp.extend(row)
        exp_wp.append(exp_wp[-1] + len(row) // 4)
    assert np.array_equal(wp, np.array(exp_wp, np.int64))
    if not items:
        assert np.array_equal(wd, np.array(exp, np.int32))
    assert deg[G.n_col0:].max() > 256


def test_allgather_world1_on_device(gpu, monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    U, B, D = 5000, 300, 40000
    d = bd.Dist(exchange=True)
    u, b = bd.block_review_edges(U, B, D, 0, U, seed=3)
    a_all, b_all, counts = bd.allgather_edges(d, u, b)
    assert a_all.is_cuda and counts == [len(u)]
    G = blp.DeviceGraph.from_device_edges(a_all.data_ptr(), b_all.data_ptr(), len(a_all), U + B, U, device=gpu)
    rp, ci, _ = _host_csr(U + B, u, b)
    assert np.array_equal(G.row_ptr, rp) and np.array_equal(G.col_idx, ci)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


U2, B2, D2 = 30000, 800, 200000


def _rank(rank, world, port, outdir):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": "0", "BLP_EXCHANGE_BACKEND": "gloo"})
    d = bd.Dist(exchange=True)
    blocks = bd.user_blocks(U2, world)
    u, b = bd.block_review_edges(U2, B2, D2, blocks[rank], blocks[rank + 1], seed=9)
    a_all, b_all, counts = bd.allgather_edges(d, u, b)
    a_dev, b_dev = a_all.to("cuda:0"), b_all.to("cuda:0")
    G = blp.DeviceGraph.from_device_edges(a_dev.data_ptr(), b_dev.data_ptr(), len(a_dev), U2 + B2, U2, device=0)
    mine = np.arange(blocks[rank], blocks[rank + 1])
    src = np.random.default_rng(rank).choice(mine[G.hop1_size[mine] > 0], 40, replace=False)
    x = np.repeat(src, 20).astype(np.int32)
    y = np.random.default_rng(rank + 10).integers(U2, U2 + B2, len(x)).astype(np.int32)
    r = G.score_pairs(x, y, 7)
    np.savez(os.path.join(outdir, "r%d.npz" % rank), rp=G.row_ptr, ci=G.col_idx, u=u, b=b, x=x, y=y, **r)
    G.close()
    d.barrier()
    d.close()


def _rccl_world1(port, outdir):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": "0", "WORLD_SIZE": "1",
                       "LOCAL_RANK": "0", "BLP_EXCHANGE_BACKEND": "nccl"})
    d = bd.Dist(exchange=True, collective_at_world1=True)
    assert d.backend == "nccl" and d.td is not None
    u, b = bd.block_review_edges(U2, B2, D2, 0, U2, seed=9)
    a_all, b_all, counts = bd.allgather_edges(d, u, b)  # RCCL all_gather_into_tensor over one rank
    assert a_all.is_cuda and counts == [len(u)]
    G = blp.DeviceGraph.from_device_edges(a_all.data_ptr(), b_all.data_ptr(), len(a_all), U2 + B2, U2, device=0)
    src = np.random.default_rng(3).choice(np.flatnonzero(G.hop1_size[:U2] > 0), 40, replace=False)
    x = np.repeat(src, 20).astype(np.int32)
    y = np.random.default_rng(4).integers(U2, U2 + B2, len(x)).astype(np.int32)
    r = G.score_pairs(x, y, 7)
    rb = G.score_pairs(y, x, 7)
    np.savez(os.path.join(outdir, "w1.npz"), rp=G.row_ptr, ci=G.col_idx, u=u, b=b, x=x, y=y, backend=d.backend,
             **r, **{"b_" + k: v for k, v in rb.items()})
    G.close()
    d.barrier()
    d.close()


def test_rccl_allgather_world1(gpu, tmp_path):
    """The config-5 exchange through RCCL itself (backend "nccl", all_gather_into_tensor),
    run over a one-rank process group on the one-GPU box: the gathered device partials build
    the device CSR (equal to the host CSR of the edges) and both sides' scores equal the oracle
    (dist.py allgather_edges; similarity.py:20-106)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_rccl_world1, args=(_free_port(), str(tmp_path)))
    p.start()
    p.join(110)
    if p.exitcode is None:
        p.kill()
    assert p.exitcode == 0, p.exitcode
    r = np.load(os.path.join(tmp_path, "w1.npz"))
    assert str(r["backend"]) == "nccl"
    rp, ci, _ = _host_csr(U2 + B2, r["u"], r["b"])
    assert np.array_equal(r["rp"], rp) and np.array_equal(r["ci"], ci)
    ids, oa, ob = dense_edges(r["u"], r["b"])
    og = coracle.OracleGraph(len(ids), oa, ob)
    xs, ys = np.searchsorted(ids, r["x"]), np.searchsorted(ids, r["y"])
    for pre, (sx, sy) in (("", (xs, ys)), ("b_", (ys, xs))):
        cn, jac, aa, _ = og.score_pairs(sx, sy, 7)
        np.testing.assert_array_equal(r[pre + "cn"], cn)
        np.testing.assert_array_equal(r[pre + "jaccard"], jac)
        np.testing.assert_array_equal(r[pre + "adamic"], aa)


def test_two_ranks_share_the_gpu(gpu, tmp_path):
    """World 2 on one GPU: each rank generates its user block, the exchange gives both the
    union, each builds the device graph and scores its own users: CSRs equal the union's host
    CSR on both ranks, scores equal the oracle."""
    import torch.multiprocessing as mp

    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(110)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert codes == [0, 0], codes
    res = [np.load(os.path.join(tmp_path, "r%d.npz" % r)) for r in range(2)]
    u = np.concatenate([r["u"] for r in res])
    b = np.concatenate([r["b"] for r in res])
    rp, ci, _ = _host_csr(U2 + B2, u, b)
    ids, oa, ob = dense_edges(u, b)
    og = coracle.OracleGraph(len(ids), oa, ob)
    for r in res:
        assert np.array_equal(r["rp"], rp) and np.array_equal(r["ci"], ci)
        cn, jac, aa, _ = og.score_pairs(np.searchsorted(ids, r["x"]), np.searchsorted(ids, r["y"]), 7)
        np.testing.assert_array_equal(r["cn"], cn)
        np.testing.assert_array_equal(r["jaccard"], jac)
        np.testing.assert_array_equal(r["adamic"], aa)  # exact sums: bit-exact


def _capi_rank(rank, world, q, outdir, device_ptrs):
    """One rank of the C-ABI exchange (multi.hip): its user block's edges through
    blp_multi_gather_csr (libblp's own RCCL communicator), then its users' pairs scored."""
    import torch

    from blp import multi as bm

    if rank == 0:
        uid = bm.Multi.unique_id()
        for _ in range(world - 1):
            q.put(uid)
    else:
        uid = q.get(timeout=60)
    blocks = bd.user_blocks(U2, world)
    u, b = bd.block_review_edges(U2, B2, D2, blocks[rank], blocks[rank + 1], seed=9)
    dev = rank % blp.device_count()  # one GPU per rank where the box has them
    torch.cuda.set_device(dev)
    try:
        m = bm.Multi(uid, world, rank, dev)
    except blp.BLPError as e:
        if e.code == -6 and world > 1:  # RCCL refuses several ranks on one GPU
            open(os.path.join(outdir, "skip%d" % rank), "w").write(str(e))
            return
        raise
    if device_ptrs:
        ta = torch.as_tensor(u.astype(np.int32)).to("cuda:%d" % dev)
        tb = torch.as_tensor(b.astype(np.int32)).to("cuda:%d" % dev)
        G = m.gather_graph(ta.data_ptr(), tb.data_ptr(), U2 + B2, U2, m=len(u))
    else:
        G = m.gather_graph(u.astype(np.int32), b.astype(np.int32), U2 + B2, U2)
    tmax = m.allreduce(rank + 1.5, "max")
    tsum = m.allreduce(1.0, "sum")
    mine = np.arange(blocks[rank], blocks[rank + 1])
    src = np.random.default_rng(rank).choice(mine[G.hop1_size[mine] > 0], 40, replace=False)
    x = np.repeat(src, 20).astype(np.int32)
    y = np.random.default_rng(rank + 10).integers(U2, U2 + B2, len(x)).astype(np.int32)
    r = G.score_pairs(x, y, 7)
    np.savez(os.path.join(outdir, "c%d.npz" % rank), rp=G.row_ptr, ci=G.col_idx, u=u, b=b, x=x, y=y,
             bytes_in=m.bytes_in, tmax=tmax, tsum=tsum, **r)
    G.close()
    m.close()


def _run_capi(world, tmp_path, device_ptrs):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_capi_rank, args=(r, world, q, str(tmp_path), device_ptrs)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(110)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert codes == [0] * world, codes
    if any(os.path.exists(os.path.join(tmp_path, "skip%d" % r)) for r in range(world)):
        pytest.skip("RCCL: several ranks on one GPU refused (%s)" % open(
            [os.path.join(tmp_path, "skip%d" % r) for r in range(world)
             if os.path.exists(os.path.join(tmp_path, "skip%d" % r))][0]).read())
    res = [np.load(os.path.join(tmp_path, "c%d.npz" % r)) for r in range(world)]
    u = np.concatenate([r["u"] for r in res])
    b = np.concatenate([r["b"] for r in res])
    rp, ci, _ = _host_csr(U2 + B2, u, b)
    ids, oa, ob = dense_edges(u, b)
    og = coracle.OracleGraph(len(ids), oa, ob)
    m_max = max(len(r["u"]) for r in res)
    for r in res:
        assert np.array_equal(r["rp"], rp) and np.array_equal(r["ci"], ci)
        assert int(r["bytes_in"]) == 8 * m_max * (world - 1)
        assert float(r["tmax"]) == world - 1 + 1.5 and float(r["tsum"]) == world
        cn, jac, aa, _ = og.score_pairs(np.searchsorted(ids, r["x"]), np.searchsorted(ids, r["y"]), 7)
        np.testing.assert_array_equal(r["cn"], cn)
        np.testing.assert_array_equal(r["jaccard"], jac)
        np.testing.assert_array_equal(r["adamic"], aa)


@pytest.mark.parametrize("device_ptrs", [False, True])
def test_multi_capi_world1(gpu, tmp_path, device_ptrs):
    """The C-ABI exchange (blp_multi_*: libblp's own RCCL communicator, no torch.distributed)
    over one rank: host or device partials, the counts and padded partials all-gathered, the
    CSR built in HBM equals the host CSR of the edges, the all-reduce returns the rank's own
    value, and the scores equal the oracle (similarity.py:20-106)."""
    _run_capi(1, tmp_path, device_ptrs)


def test_multi_capi_two_ranks(gpu, tmp_path):
    """World 2 through the C-ABI, rank r on GPU r mod the device count: each rank passes its
    user block, both get the union's CSR (bytes_in = the other rank's padded partial), the
    max / sum all-reduces agree, and each rank's scores equal the oracle. On a one-GPU box
    both ranks share device 0, which RCCL refuses (ncclInvalidUsage): then skipped."""
    _run_capi(2, tmp_path, False)


@pytest.mark.parametrize("device_recv", [False, True])
def test_multi_compact_three_ranks(gpu, device_recv):
    """The post-gather compaction of the C-ABI exchange (blp_multi_compact_csr, the code
    blp_multi_gather_csr runs after its all-gather) at world 3 on one GPU: an all-gather
    receive buffer with uneven counts and a zero-count rank, its padding poisoned with
    out-of-range ids (read, they would fail the CSR build), host or device memory. The CSR
    equals the host CSR of the union, bytes_in = 8 * m_max * (world - 1), and the scores on it
    equal the oracle (similarity.py:20-61 over the union graph, similarity.py:16)."""
    from blp.multi import Multi

    rng = np.random.default_rng(5)
    n_users, n_bus = 40000, 3000
    blocks = [0, 15000, 15000, n_users]  # rank 1 owns no users: a zero-count partial
    parts = []
    for r in range(3):
        lo, hi = blocks[r], blocks[r + 1]
        k = {0: 90000, 1: 0, 2: 170000}[r]
        u = rng.integers(lo, max(hi, lo + 1), k)
        b = n_users + np.minimum((rng.pareto(1.2, k) * 40).astype(np.int64), n_bus - 1)
        parts.append((u.astype(np.int32), b.astype(np.int32)))
    counts = np.array([len(p[0]) for p in parts], np.int64)
    m_max = int(counts.max())
    recv = np.full((3, 2, m_max), 0x7FFFFFF0, np.int32)  # padding: ids far outside [0, n)
    for r, (u, b) in enumerate(parts):
        recv[r, 0, : len(u)] = u
        recv[r, 1, : len(b)] = b
    n = n_users + n_bus
    if device_recv:
        import torch

        t = torch.from_numpy(recv).cuda()
        c, bytes_in = Multi.compact_csr(t.data_ptr(), counts, n, device=gpu)
    else:
        c, bytes_in = Multi.compact_csr(recv, counts, n, device=gpu)
    assert bytes_in == 8 * m_max * 2
    G = blp.DeviceGraph.from_csr_handle(c, n, n_users, gpu)
    ua = np.concatenate([p[0] for p in parts])
    ub = np.concatenate([p[1] for p in parts])
    rp, ci, _ = _host_csr(n, ua, ub)
    assert np.array_equal(G.row_ptr, rp) and np.array_equal(G.col_idx, ci)
    ids, oa, ob = dense_edges(ua, ub)
    og = coracle.OracleGraph(len(ids), oa, ob)
    src = rng.choice(np.unique(ua), 60, replace=False)
    x = np.repeat(src, 25).astype(np.int32)
    y = rng.choice(np.unique(ub), len(x)).astype(np.int32)
    for xs, ys in ((x, y), (y, x)):
        got = G.score_pairs(xs, ys, 7)
        cn, jac, aa, _ = og.score_pairs(np.searchsorted(ids, xs), np.searchsorted(ids, ys), 7)
        np.testing.assert_array_equal(got["cn"], cn)
        np.testing.assert_array_equal(got["jaccard"], jac)
        np.testing.assert_array_equal(got["adamic"], aa)
    G.close()


def test_multi_compact_rejects_bad_counts(gpu):
    from blp.multi import Multi

    with pytest.raises(RuntimeError):
        Multi.compact_csr(np.zeros(8, np.int32), np.array([2, -1], np.int64), 10, device=gpu)


def _edges_load(path, device=None, csr_device=None):
    """Everything a blp_edges handle reports: through blp_edges_load_device (device given) or
    the host loader blp_edges_load; plus the CSR of blp_edges_csr when there is an id map."""
    L, P, check = blp.lib(), blp._lib.ptr, blp._lib.check
    h = ctypes.c_void_p()
    if device is None:
        check(L.blp_edges_load(str(path).encode(), 0, 1, ctypes.byref(h)))
    else:
        check(L.blp_edges_load_device(str(path).encode(), 0, 1, device, ctypes.byref(h)))
    try:
        v = [ctypes.c_int64() for _ in range(5)]
        check(L.blp_edges_info(h, *(ctypes.byref(x) for x in v)))
        m, n, n0, lo, span = (x.value for x in v)
        on = ctypes.c_int(7)
        check(L.blp_edges_device(h, ctypes.byref(on)))
        out = {"info": (m, n, n0, lo, span), "on": on.value}
        a, b = np.empty(m, np.int64), np.empty(m, np.int64)
        if span == 0:
            check(L.blp_edges_fetch(h, P(a), P(b), None, None, None, None))
            out.update(a=a, b=b)
            return out
        da, db = np.empty(m, np.int32), np.empty(m, np.int32)
        ids, idm = np.empty(n, np.int64), np.empty(span, np.int32)
        check(L.blp_edges_fetch(h, P(a), P(b), P(da), P(db), P(ids), P(idm)))
        out.update(a=a, b=b, da=da, db=db, node_ids=ids, id_map=idm)
        c = ctypes.c_void_p()
        check(L.blp_edges_csr(h, csr_device if csr_device is not None else 0, ctypes.byref(c)))
        try:
            nn, nnz = ctypes.c_int64(), ctypes.c_int64()
            check(L.blp_csr_info(c, ctypes.byref(nn), ctypes.byref(nnz)))
            rp = np.empty(n + 1, np.int64)
            ci = np.empty(max(nnz.value, 1), np.int32)
            sl = np.empty(max(n, 1), np.uint8)
            check(L.blp_csr_fetch(c, P(rp), P(ci), P(sl)))
            out["csr"] = (rp, ci[: nnz.value], sl[:n])
        finally:
            L.blp_csr_destroy(c)
        return out
    finally:
        L.blp_edges_destroy(h)


def _graph_txt(path, a, c, rng, shapes=("%d %d\n", "%d\t%d\r\n", "%d  %d \n", "%d\t \t%d\t\r\n", "%07d %d\n"),
               final_newline=False, extra=()):
    """graph.txt text of edges (a, c) with the line shapes the device parser takes; `extra`
    lines (index, text) spliced in."""
    pick = rng.integers(0, len(shapes), len(a))
    lines = [shapes[k] % (x, y) for k, x, y in zip(pick.tolist(), a.tolist(), c.tolist())]
    for i, t in extra:
        lines.insert(i, t)
    text = "".join(lines)
    if not final_newline:
        text = text.rstrip("\n").rstrip("\r")
    path.write_text(text)
    return path


def _same_load(d, h):
    assert d["info"] == h["info"]
    for k in ("a", "b", "da", "db", "node_ids", "id_map"):
        if k in h:
            assert np.array_equal(d[k], h[k]), k
    if "csr" in h:
        for x, y in zip(d["csr"], h["csr"]):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("chunk_kb", [None, "64", "12"])
@pytest.mark.parametrize("final_newline", [False, True])
def test_device_parse_equals_host_parse(gpu, tmp_path, final_newline, chunk_kb, monkeypatch):
    """blp_edges_load_device on a graph.txt of the reference's line shape (dataset_maker.py:197;
    tabs, CRLF, trailing blanks, leading zeros, duplicates, reversed duplicates, self-loops): the
    parse, id map and CSR run on the device and equal the host loader's, and the CSR equals the
    host CSR builder's on the dense endpoints. The text reaches HBM through the process's pinned
    staging ring (2 MiB slot fills by default; 64 KiB and 12 KiB fills wrap the ring many times,
    BLP_PARSE_CHUNK_KB)."""
    if chunk_kb:
        monkeypatch.setenv("BLP_PARSE_CHUNK_KB", chunk_kb)
    rng = np.random.default_rng(21)
    a, c = _messy_edges(rng, 60000, 2500, 150000)
    p = _graph_txt(tmp_path / "graph.txt", a + 5, c + 5, rng, final_newline=final_newline)
    assert p.stat().st_size >= 1 << 20
    d = _edges_load(p, device=gpu, csr_device=gpu)
    h = _edges_load(p, csr_device=gpu)
    assert d["on"] == gpu and h["on"] == -1
    _same_load(d, h)
    m, n, n0, lo, span = d["info"]
    assert m == len(a) and lo == 5 and span > 0
    rp, ci, sl = _host_csr(n, d["da"], d["db"])
    for x, y in zip(d["csr"], (rp, ci, sl)):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("draws,lo_mib,hi_mib", [(100000, 1, 4), (230000, 1, 4), (700000, 4, 64)])
@pytest.mark.parametrize("final_newline", [False, True])
def test_device_parse_sizes_repeated(gpu, tmp_path, draws, lo_mib, hi_mib, final_newline):
    """The round-5 driver fault (GPUTEST_r05: an illegal address at the graph.txt upload of a
    ~2 MB file) came from the upload's host buffer: a fresh 1-4 MiB malloc block or >= 4 MiB
    mapping, registered, copied, unregistered and freed on every call. The upload now goes through
    the process's pinned staging ring only. Files in the 1-4 MiB band and above it, with and without
    the final newline, each loaded three times in a row through the device parser (the ring and
    the device scratch blocks reused), every load equal to the host loader's."""
    rng = np.random.default_rng(draws + final_newline)
    a, c = _messy_edges(rng, 90000, 3000, draws)
    p = _graph_txt(tmp_path / "graph.txt", a + 1, c + 1, rng, final_newline=final_newline)
    assert (lo_mib << 20) <= p.stat().st_size < (hi_mib << 20)
    h = _edges_load(p, csr_device=gpu)
    for _ in range(3):
        d = _edges_load(p, device=gpu, csr_device=gpu)
        assert d["on"] == gpu
        _same_load(d, h)


@pytest.mark.parametrize("case", ["comment", "blank_line", "sign", "extra_column", "long_id", "sparse_ids", "small"])
def test_device_parse_falls_back_to_host(gpu, tmp_path, case):
    """Text outside the device parser's shape is parsed on the host, with the host loader's
    results: comments, blank lines, signs, extra columns, 19-digit ids, a non-compact id space,
    files under 1 MiB."""
    rng = np.random.default_rng(22)
    a, c = _messy_edges(rng, 60000, 2500, 150000)
    extra = {"comment": [(777, "# a comment\n")], "blank_line": [(5000, "\n")], "sign": [(9000, "+12 40\n")],
             "extra_column": [(100, "12 40 3\n")], "long_id": [(123, "1000000000000000000 7\n")]}.get(case, ())
    if case == "sparse_ids":
        a, c = a * 7919, c * 7919
    if case == "small":
        a, c = a[:1000], c[:1000]
    p = _graph_txt(tmp_path / "graph.txt", a, c, rng, extra=extra)
    d = _edges_load(p, device=gpu, csr_device=gpu)
    h = _edges_load(p, csr_device=gpu)
    assert d["on"] == -1
    _same_load(d, h)
    if case in ("sparse_ids", "long_id"):
        assert d["info"][4] == 0


def test_device_parse_out_of_memory_falls_back_to_host(gpu, tmp_path, monkeypatch):
    """A device parse that cannot get its HBM (BLP_PARSE_MEM_CAP: the reservations fail as out
    of memory) is not an error: the host parser takes the file, with the host loader's results
    (similarity.py:16, blp_edges_load_device)."""
    rng = np.random.default_rng(24)
    a, c = _messy_edges(rng, 60000, 2500, 150000)
    p = _graph_txt(tmp_path / "graph.txt", a, c, rng)
    monkeypatch.setenv("BLP_PARSE_MEM_CAP", "4096")
    d = _edges_load(p, device=gpu, csr_device=gpu)
    monkeypatch.delenv("BLP_PARSE_MEM_CAP")
    h = _edges_load(p, csr_device=gpu)
    assert d["on"] == -1
    _same_load(d, h)


def test_load_edge_list_device_parse(gpu, tmp_path):
    """blp.load_edge_list (similarity.py:16's snap.LoadEdgeList) on a device-parsed file gives
    the graph DeviceGraph builds from the host-parsed ids: ids, CSR, weights and scores."""
    rng = np.random.default_rng(23)
    a, c = _messy_edges(rng, 50000, 2000, 140000)
    p = _graph_txt(tmp_path / "graph.txt", a + 3, c + 3, rng)
    G = blp.load_edge_list(str(p), device=gpu)
    ra, rb = blp.parse_edge_list(str(p))
    H = blp.DeviceGraph(ra, rb, device=gpu)
    assert "device_csr_s" in G.build_times
    for k in ("node_ids", "row_ptr", "col_idx", "self_loop", "degree", "aa_weight"):
        assert np.array_equal(getattr(G, k), getattr(H, k)), k
    assert G.n_col0 == H.n_col0
    assert np.array_equal(G.dense(H.node_ids[:100]), np.arange(100))
    users = rng.choice(np.flatnonzero(G.hop1_size[: G.n_col0] > 0), 50, replace=False)
    x = np.repeat(users, 20).astype(np.int32)
    y = rng.integers(G.n_col0, G.n, len(x)).astype(np.int32)
    for k, v in G.score_pairs(x, y, 7).items():
        np.testing.assert_array_equal(v, H.score_pairs(x, y, 7)[k])
