"""Multi-GPU plumbing on CPU (gloo, world_size 2): the row-block sharded ingest and its one
exchange step, and the replica-mode reductions bench.py uses. The RCCL
("nccl") variant runs the same code with device tensors; it needs >= 2 GPUs (driver's
8-GPU run), so here the exchange goes over gloo (BLP_EXCHANGE_BACKEND=gloo)."""
import os
import socket

import numpy as np
import pytest

import blp
from blp import dist as bd
from blp import synth

U, B, D = 4000, 300, 30000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _csr(a, b):
    import ctypes

    n = U + B
    A = np.ascontiguousarray(a, np.int32)
    Bv = np.ascontiguousarray(b, np.int32)
    rp = np.zeros(n + 1, np.int64)
    ci = np.empty(max(2 * len(A), 1), np.int32)
    sl = np.zeros(n, np.uint8)
    nnz = ctypes.c_int64(0)
    P = blp._lib.ptr
    blp._lib.check(blp.lib().blp_csr_from_edges(n, len(A), P(A), P(Bv), P(rp), P(ci), P(sl), ctypes.byref(nnz)))
    return rp, ci[: nnz.value]


def _worker(rank, world, port, outdir):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank), "BLP_EXCHANGE_BACKEND": "gloo"})
    d = bd.Dist(exchange=True)
    assert d.backend == "gloo" and d.world == world
    blocks = bd.user_blocks(U, world)
    lo, hi = blocks[rank], blocks[rank + 1]
    u, b = bd.block_review_edges(U, B, D, lo, hi, seed=7)
    assert ((u >= lo) & (u < hi)).all()
    a_all, b_all, counts = bd.allgather_edges(d, u, b)
    assert sum(counts) == len(a_all) and counts[rank] == len(u)
    # the same CSR on every rank, built by the host twin of blp_csr_from_edges_device
    rp, ci = _csr(a_all.numpy(), b_all.numpy())
    np.savez(os.path.join(outdir, "r%d.npz" % rank), rp=rp, ci=ci, u=u, b=b,
             mx=d.max(rank + 1.5), sm=d.sum(rank + 1), ints=np.array(d.allgather_int(10 * rank + 3)),
             uid=np.frombuffer(d.broadcast_bytes(bytes(range(128)) if rank == 0 else None), np.uint8))
    d.barrier()
    d.close()


def _run(world, tmp_path):
    import torch.multiprocessing as mp

    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return [np.load(os.path.join(tmp_path, "r%d.npz" % r)) for r in range(world)]


def test_user_blocks_balance_work():
    b = bd.user_blocks(10, 3)
    assert b.tolist() == [0, 3, 6, 10]
    work = np.r_[np.full(10, 100.0), np.ones(90)]  # heavy head: the first block must be short
    wb = bd.user_blocks(100, 4, work)
    assert wb[0] == 0 and wb[-1] == 100 and (np.diff(wb) >= 0).all()
    per = [work[wb[i]:wb[i + 1]].sum() for i in range(4)]
    assert max(per) - min(per) <= 2 * 100.0  # within two of the largest items


def test_block_edges_cover_the_distribution():
    blocks = bd.user_blocks(U, 4)
    parts = [bd.block_review_edges(U, B, D, blocks[r], blocks[r + 1], seed=1) for r in range(4)]
    u = np.concatenate([p[0] for p in parts])
    b = np.concatenate([p[1] for p in parts])
    assert abs(len(u) - D) <= 4
    assert u.min() >= 0 and u.max() < U and b.min() >= U and b.max() < U + B
    # Zipf popularity: the most popular business gets ~p[0] of the draws
    p0 = synth.popularity(B)[0]
    assert abs((b == U).mean() - p0) < 5 * np.sqrt(p0 / len(b))


@pytest.mark.parametrize("world", [2])
def test_gloo_exchange_gives_every_rank_the_whole_graph(world, tmp_path):
    res = _run(world, tmp_path)
    u = np.concatenate([r["u"] for r in res])
    b = np.concatenate([r["b"] for r in res])
    rp, ci = _csr(u, b)  # the union of the partials, built in one process
    for r in res:
        assert np.array_equal(r["rp"], rp) and np.array_equal(r["ci"], ci)
    assert float(res[0]["mx"]) == world + 0.5 and float(res[1]["sm"]) == sum(range(1, world + 1))
    assert res[1]["ints"].tolist() == [10 * r + 3 for r in range(world)]
    # rank 0's communicator id (blp_multi_unique_id's 128 bytes) reaches every rank
    assert all(r["uid"].tolist() == list(range(128)) for r in res)
