"""GPU parity: the HIP pair scorer (via the drop-in similarity module and the C-ABI)
against the reference's golden outputs and the C oracle. Marked `gpu`."""
import math
import os

import numpy as np
import pytest

import blp
import coracle
import similarity
from helpers import (B_FILES, GOLDEN, METHODS, SIM_CASES, U_FILES, assert_same_scores, bipartite_edges, dense_edges,
                     golden, load)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", SIM_CASES)
def test_main_writes_reference_files(gpu, case, tmp_path):
    d = os.path.join(GOLDEN, case)
    uf = [str(tmp_path / f) for f in U_FILES]
    bf = [str(tmp_path / f) for f in B_FILES]
    similarity.main(os.path.join(d, "examples.json"), os.path.join(d, "graph.txt"), METHODS, uf, METHODS, bf)
    for m, f in zip(METHODS, U_FILES):
        assert_same_scores(load(str(tmp_path / f)), golden(case, f), m)
    for m, f in zip(METHODS, B_FILES):
        assert_same_scores(load(str(tmp_path / f)), golden(case, f), m)


@pytest.mark.parametrize("case", SIM_CASES)
def test_main_native_files_equal_dict_path(gpu, case, tmp_path):
    """similarity.main's native path (examples parsed into arrays, files written by
    blp_scores_write) produces byte-identical files to the dict + json.dumps path (which
    sidecar=True selects), including missing-node zeros and the b_adamic bug file."""
    d = os.path.join(GOLDEN, case)
    out = {}
    for mode in ("native", "dict"):
        uf = [str(tmp_path / (mode + f)) for f in U_FILES]
        bf = [str(tmp_path / (mode + f)) for f in B_FILES]
        similarity.main(os.path.join(d, "examples.json"), os.path.join(d, "graph.txt"), METHODS, uf, METHODS, bf,
                        sidecar=(mode == "dict"))
        out[mode] = [open(f).read() for f in uf + bf]
    assert out["native"] == out["dict"]


def _check_against_oracle(ga, gb, x, y, mask=7):
    """Device scores of dense-id pairs vs the C oracle on the same edge list."""
    G = blp.DeviceGraph(ga, gb)
    ids, da, db = dense_edges(ga, gb)
    og = coracle.OracleGraph(len(ids), da, db)
    # both sides use original ids; map to each engine's own dense ids
    xo, yo = G.node_ids[x], G.node_ids[y]
    got = G.score_pairs(x, y, mask)
    cn, jac, aa, _ = og.score_pairs(np.searchsorted(ids, xo), np.searchsorted(ids, yo), mask)
    np.testing.assert_array_equal(got["cn"], cn)
    if mask & blp.JACCARD:
        np.testing.assert_array_equal(got["jaccard"], jac)  # bit-exact
    if mask & blp.ADAMIC:
        np.testing.assert_array_equal(got["adamic"], aa)  # exact sums on both sides: bit-exact
    # the same pairs grouped by source (x non-decreasing): the run-head grouping path; the
    # exact sums make every score independent of pair order, so results are identical
    order = np.argsort(x, kind="stable")
    got_sorted = G.score_pairs(x[order], y[order], mask)
    for k, v in got.items():
        if v is not None:
            np.testing.assert_array_equal(got_sorted[k], v[order])
    return G


@pytest.mark.parametrize("no_runs", [False, True])
@pytest.mark.parametrize("n_users,n_bus,n_draws,seed", [
    (2000, 300, 20000, 0),     # small universe: SMALL block variant / short-row scorer
    (30000, 2000, 150000, 1),  # MED block variant
    (300000, 5000, 600000, 2), # LARGE block variant, long rows (popular businesses)
])
def test_user_and_business_side_vs_oracle(gpu, n_users, n_bus, n_draws, seed, no_runs, monkeypatch):
    if no_runs:
        monkeypatch.setenv("BLP_NO_RUNS", "1")  # bucket-sort grouping even for source-grouped lists
    rng = np.random.default_rng(seed)
    a, b = bipartite_edges(rng, n_users, n_bus, n_draws)
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    users = rng.choice(nu, size=min(200, nu), replace=False)
    x = np.repeat(users, 40).astype(np.int32)
    y = rng.integers(nu, G.n, len(x)).astype(np.int32)
    _check_against_oracle(a, b, x, y)          # user side
    _check_against_oracle(a, b, y, x)          # business side


def test_general_graph_exact_distance(gpu):
    rng = np.random.default_rng(5)
    a = rng.integers(0, 3000, 20000)
    b = rng.integers(0, 3000, 20000)
    a[:50] = b[:50]  # self-loops: SNAP degree +1, hop sets unchanged
    G = blp.DeviceGraph(a, b)
    x = rng.integers(0, G.n, 5000).astype(np.int32)
    y = rng.integers(0, G.n, 5000).astype(np.int32)
    _check_against_oracle(a, b, x, y)


@pytest.mark.parametrize("knobs", [
    {},
    {"BLP_CHUNK_BITS": "1024"},                         # wider than LDS: HBM-bitmap scorer
    {"BLP_CHUNK_BITS": "1024", "BLP_NO_GLOBAL": "1"},   # multi-chunk LDS bitmap universe
    {"BLP_FORCE_GLOBAL": "1"},                          # HBM-bitmap scorer on a small universe
    {"BLP_SPLIT": "3", "BLP_NO_HASH": "1"},                                 # chunk-parallel scorer, 3 chunks
    {"BLP_SPLIT": "3", "BLP_SPLIT_NOPK": "1", "BLP_NO_HASH": "1"},          # ... per-pair count in its own word (rows >= 2^24)
    {"BLP_SPLIT": "5", "BLP_SPLIT_BIG": "1", "BLP_SPLIT_NOPK": "1", "BLP_NO_HASH": "1"},
    {"BLP_SPLIT": "8", "BLP_HEAVY_WORK": "50", "BLP_NO_HASH": "1"},         # ... 8 chunks, heavy sources pre-built
    {"BLP_SPLIT": "2", "BLP_HOT_MIN": "8", "BLP_NO_HASH": "1"},             # ... dense rows OR-ed per chunk
    {"BLP_SPLIT": "40", "BLP_NO_HASH": "1"},                                # ... many chunks, some empty
    {"BLP_SPLIT": "3", "BLP_SPLIT_BIG": "1", "BLP_NO_HASH": "1"},           # ... 128 KiB chunks, one workgroup per CU
    {"BLP_SPLIT": "3", "BLP_SPLIT_BIG": "1", "BLP_SPLIT_SHORT": "0", "BLP_NO_HASH": "1"},  # ... no thread-per-slice short path
    {"BLP_SPLIT": "2", "BLP_SPLIT_BIG": "1", "BLP_SPLIT_SHORT": "4", "BLP_NO_HASH": "1"},  # ... short path only below 5 ids
    {"BLP_SPLIT": "24", "BLP_SPLIT_BIG": "1", "BLP_NO_HASH": "1"},          # ... same, many chunks
    {"BLP_SPLIT": "3", "BLP_SPLIT_BIG": "1", "BLP_NO_HASH": "1", "BLP_NO_WEDGE": "1"},  # ... members' rows from the CSR, not wedge rows
    {"BLP_SPLIT": "3", "BLP_SPLIT_BIG": "1", "BLP_HASH_WORK": "600", "BLP_NO_WEDGE": "1"},  # hash-set build from the CSR
    {"BLP_SPLIT": "3", "BLP_HASH_BIG": "1"},                                # 128 KiB hash tables (1024 threads)
    {"BLP_SPLIT": "3", "BLP_HASH_BIG": "1", "BLP_NO_WEDGE": "1"},           # ... built from the CSR
    {"BLP_HEAVY_WORK": "50"},                           # heavy sources pre-built by k_heavy
    {"BLP_HEAVY_WORK": "1"},                            # one row per heavy item
    {"BLP_CHUNK_BITS": "2048", "BLP_HEAVY_WORK": "50", "BLP_NO_GLOBAL": "1"},  # multi-chunk: no heavy path
    {"BLP_HOT_MIN": "8"},                               # dense-row index OR-ed into H2
    {"BLP_VARIANT": "2"},                               # LARGE variant (row-chunk loops) on the small graph
    {"BLP_VARIANT": "2", "BLP_WCODES": "3"},            # ... few weight codes: code-0 ids gather aaw
    {"BLP_HOT_MIN": "8", "BLP_CHUNK_BITS": "1024", "BLP_NO_GLOBAL": "1"},  # dense rows across chunks
    {"BLP_HOT_MIN": "8", "BLP_HEAVY_WORK": "50"},
    {"BLP_HOT_MIN": "1", "BLP_HOT_DENSITY": "100000000"},  # > HOT_LIST dense rows: sparse fallback
    {"BLP_VARIANT": "1"},                               # 64 KiB-bitmap scorer (no hint table)
    {"BLP_VARIANT": "2"},                               # 136 KiB-bitmap scorer (row-chunk loops)
    {"BLP_VARIANT": "2", "BLP_NO_SHORT": "1"},          # ... short rows through the row-chunk loops
    {"BLP_VARIANT": "2", "BLP_WCODES": "3"},            # ... coded and gathered weights mixed
    {"BLP_VARIANT": "2", "BLP_HOT_MIN": "8"},           # ... dense rows skipped: empty build rows
    {"BLP_VARIANT": "2", "BLP_CHUNK_BITS": "1024", "BLP_NO_GLOBAL": "1"},  # ... several LDS chunks
    {"BLP_VARIANT": "2", "BLP_NO_PKO": "1"},            # ... the general large scorer (per-pair counts, 512-pair segments)
    {"BLP_VARIANT": "2", "BLP_NO_PKO": "1", "BLP_NO_SHORT": "1"},
    {"BLP_NO_SHORT_KERNEL": "1"},                       # short rows through the general block scorer
    {"BLP_WCODES": "0"},                                # every AA weight gathered per node
    {"BLP_WCODES": "3"},                                # coded and gathered weights mixed
    {"BLP_NO_WCODES": "1"},                             # scorers on the plain id stream
    {"BLP_WCODES": "3", "BLP_SPLIT": "3"},
    {"BLP_WCODES": "3", "BLP_SPLIT": "3", "BLP_SPLIT_BIG": "1", "BLP_NO_HASH": "1"},  # short slices: code-0 hits gather aaw
    {"BLP_NO_WCODES": "1", "BLP_SPLIT": "3", "BLP_SPLIT_BIG": "1", "BLP_NO_HASH": "1"},  # ... every hit gathers (plain ids)
    {"BLP_WCODES": "3", "BLP_FORCE_GLOBAL": "1"},
    {"BLP_WCODES": "3", "BLP_HEAVY_WORK": "50", "BLP_HOT_MIN": "8"},
    {"BLP_NO_WEDGE": "1"},                              # short-row build from CSR, not wedge rows
    {"BLP_NO_WEDGE": "1", "BLP_HEAVY_WORK": "50"},      # ... heavy items as CSR ranges
    {"BLP_WEDGE": "0", "BLP_HEAVY_WORK": "50"},         # graph built without wedge rows
    {"BLP_WEDGE_MAX_X": "0.5"},                         # wedge rows over budget: not built
    {"BLP_HEAVY_WORK": "7"},                            # wedge slices of 1 vector, uneven tails
    {"BLP_HEAVY_WORK": "7", "BLP_NO_WBM_BATCH": "1"},   # ... through k_heavy, not the graph's wedge-row bitmaps
    {"BLP_NO_WBM_BATCH": "1"},                          # every business source built from its wedge row
    {"BLP_WBM_MIN_X": "40"},                            # bitmaps for the longest wedge rows only
    {"BLP_SPLIT": "3", "BLP_SPLIT_BIG": "1", "BLP_HASH_WORK": "600"},  # hash-set scorer for light sources, split for the rest
    {"BLP_SPLIT": "2", "BLP_SPLIT_BIG": "1", "BLP_HASH_WORK": "100000"},  # every source on the hash-set scorer (knob clamped to HT - 1)
    {"BLP_SPLIT": "4", "BLP_HASH_WORK": "400"},          # ... beside the 64 KiB chunk scorer
    {"BLP_NO_WEDGE": "1", "BLP_HEAVY_WORK": "7"},       # short-row batches on the segment scorer (k_score SHORT)
    {"BLP_NO_WSET": "1"},                               # business side on the grouped short-row scorer (k_score_short)
    {"BLP_NO_WSET": "1", "BLP_HEAVY_WORK": "7"},        # ... with wedge slices of heavy sources
    {"BLP_WSET_MB": "0"},                               # wedge-set index over budget: the grouped path
    {"BLP_ITEM_NB": "1"},                               # one interleaved bucket (or the fewest that keep <= 1024 keys)
    {"BLP_ITEM_NB": "4", "BLP_GROUP_NBLK": "3"},        # few buckets, few scatter workgroups
    {"BLP_LPT": "0"},                                   # run-grouped sources queued in id order (default: largest work first)
    {"BLP_NO_YDIRECT": "1"},                            # run-grouped block scorer on gathered row starts / lengths
    {"BLP_NO_RUN_FAST": "1"},                           # run grouping by tile counts, scan and writes (four launches)
    {"BLP_VARIANT": "2", "BLP_NO_YDIRECT": "1"},        # ... the large scorer on gathered rows (so no two-launch grouping)
    {"BLP_VARIANT": "2", "BLP_NO_RUN_FAST": "1"},       # ... the large scorer after the four-launch grouping
    {"BLP_LPT": "3"},                                   # ... and item-grouped ones
    {"BLP_LPT": "3", "BLP_SPLIT": "3", "BLP_HASH_WORK": "600"},  # ... with the hash-set partition of the queue
])
def test_kernel_paths_vs_oracle(gpu, knobs, monkeypatch):
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(11)
    a, b = bipartite_edges(rng, 6000, 400, 40000)
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    x = np.repeat(rng.choice(nu, 60, replace=False), 30).astype(np.int32)
    y = rng.integers(nu, G.n, len(x)).astype(np.int32)
    _check_against_oracle(a, b, x, y)
    _check_against_oracle(a, b, y, x)
    if "BLP_HEAVY_WORK" in knobs and "BLP_CHUNK_BITS" not in knobs:
        plan = G.batch(y, x).plan()  # heavy business sources: k_heavy, or the graph's wedge-row bitmaps
        assert plan["heavy"] > 0 or plan["wedge_bitmaps"]
        if "BLP_NO_WBM_BATCH" in knobs:
            assert plan["heavy"] > 0 and not plan["wedge_bitmaps"]
    if "BLP_FORCE_GLOBAL" in knobs or ("BLP_CHUNK_BITS" in knobs and "BLP_NO_GLOBAL" not in knobs):
        assert G.batch(x, y).plan()["chunks"] == 0  # HBM-bitmap scorer
    if "BLP_SPLIT" in knobs:
        assert G.batch(x, y).plan()["chunks"] == -int(knobs["BLP_SPLIT"])  # chunk-parallel scorer


@pytest.mark.parametrize("variant", [None, "1", "2", "split", "split_big", "split_nopk", "split_noshort", "split_hash"])
def test_many_pairs_per_source_vs_oracle(gpu, variant, monkeypatch):
    # > SEG pairs per source and > SEG rows in N(x): the segment-chunk loops; batches of more
    # than one block step: the segment hint tables. Chunk-parallel scorer: several pair batches
    # per (source, chunk) item, so the next batch's metadata comes from the in-flight prefetch
    knobs = {"split": {"BLP_SPLIT": "3", "BLP_NO_HASH": "1"}, "split_big": {"BLP_SPLIT": "4", "BLP_SPLIT_BIG": "1", "BLP_NO_HASH": "1"},
             "split_nopk": {"BLP_SPLIT": "4", "BLP_SPLIT_BIG": "1", "BLP_SPLIT_NOPK": "1", "BLP_NO_HASH": "1"},
             "split_noshort": {"BLP_SPLIT": "4", "BLP_SPLIT_BIG": "1", "BLP_SPLIT_SHORT": "0", "BLP_NO_HASH": "1"},
             "split_hash": {"BLP_SPLIT": "4", "BLP_SPLIT_BIG": "1", "BLP_HASH_WORK": "100000"}}
    if variant in knobs:
        for k, v in knobs[variant].items():
            monkeypatch.setenv(k, v)
    elif variant:
        monkeypatch.setenv("BLP_VARIANT", variant)
    rng = np.random.default_rng(12)
    a, b = bipartite_edges(rng, 20000, 1500, 200000)
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    users = rng.choice(nu, 6, replace=False)
    x = np.repeat(users, 1400).astype(np.int32)
    y = rng.integers(nu, G.n, len(x)).astype(np.int32)
    _check_against_oracle(a, b, x, y)
    _check_against_oracle(a, b, y, x)   # popular businesses: N(x) has thousands of rows


def test_single_run_and_tile_edges(gpu):
    # grouped input: one source for every pair, and run heads on scan-tile boundaries
    rng = np.random.default_rng(14)
    a, b = bipartite_edges(rng, 20000, 1500, 200000)
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    y = rng.integers(nu, G.n, 5000).astype(np.int32)
    _check_against_oracle(a, b, np.full(len(y), rng.integers(0, nu), np.int32), y)
    x = np.sort(rng.choice(nu, 4096 * 3 + 7, replace=True)).astype(np.int32)
    x[4095:4097] = x[4094] + np.array([0, 1])  # heads at and around a tile boundary
    x = np.maximum.accumulate(x)
    _check_against_oracle(a, b, x, rng.integers(nu, G.n, len(x)).astype(np.int32))


def test_unsorted_pair_order_vs_oracle(gpu):
    # grouping must not assume any input order (runs of x broken up)
    rng = np.random.default_rng(13)
    a, b = bipartite_edges(rng, 20000, 1500, 200000)
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    x = np.repeat(rng.choice(nu, 100, replace=False), 50).astype(np.int32)
    y = rng.integers(nu, G.n, len(x)).astype(np.int32)
    perm = rng.permutation(len(x))
    _check_against_oracle(a, b, x[perm], y[perm])


@pytest.mark.parametrize("mode", ["items", "buckets"])
def test_skewed_unsorted_grouping_vs_oracle(gpu, mode, monkeypatch):
    # ungrouped pair lists with one hot source (> several GI_PAIRS items of its own) and a run
    # of popular neighbouring ids, over a wide id range (hundreds of keys per bucket)
    if mode == "buckets":
        monkeypatch.setenv("BLP_GROUP_BUCKETS", "1")
    rng = np.random.default_rng(15)
    a, b = bipartite_edges(rng, 300000, 2000, 400000)
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    hot = int(rng.integers(0, nu))
    x = np.concatenate([np.full(18000, hot), rng.integers(0, 64, 6000), rng.integers(0, nu, 9000)]).astype(np.int32)
    y = rng.integers(nu, G.n, len(x)).astype(np.int32)
    perm = rng.permutation(len(x))
    _check_against_oracle(a, b, x[perm], y[perm])
    _check_against_oracle(a, b, y[perm], x[perm])


def test_batch_repeat_is_deterministic(gpu):
    rng = np.random.default_rng(3)
    a, b = bipartite_edges(rng, 20000, 1000, 100000)
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    x = np.repeat(rng.choice(nu, 100, replace=False), 50).astype(np.int32)
    y = rng.integers(nu, G.n, len(x)).astype(np.int32)
    bt = G.batch(x, y)
    bt.score(7)
    r1 = bt.fetch(7)
    for _ in range(3):
        bt.score(7)
    r2 = bt.fetch(7)
    for k in r1:
        np.testing.assert_array_equal(r1[k], r2[k])
    ms, launches = G.stats(blp._lib.K_SCORE)
    assert launches == 4 and ms > 0


def test_graph_score_totals_follow_the_batch_timers(gpu):
    # the graph's score / group totals are the batches' own timers (no timing events of their
    # own): launches and milliseconds add up, a destroyed batch's times stay in the totals, and
    # batches scored from two host threads at once are each counted
    import threading

    rng = np.random.default_rng(5)
    a, b = bipartite_edges(rng, 20000, 1000, 100000)
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    x = np.repeat(rng.choice(nu, 100, replace=False), 50).astype(np.int32)
    y = rng.integers(nu, G.n, len(x)).astype(np.int32)
    G.stats_reset()
    bx, by = G.batch(x, y), G.batch(y, x)
    for _ in range(2):
        bx.score(7)
    by.score(3)
    bx.fetch(7)
    by.fetch(3)
    ms, launches = G.stats(blp._lib.K_SCORE)
    mx, nx = bx.stats(0)
    my, ny = by.stats(0)
    assert (launches, nx, ny) == (3, 2, 1)
    assert ms == pytest.approx(mx + my, rel=1e-6) and ms > 0
    gms, gl = G.stats(blp._lib.K_GROUP)
    assert gl == bx.stats(1)[1] + by.stats(1)[1]
    by.close()
    assert G.stats(blp._lib.K_SCORE) == (pytest.approx(ms, rel=1e-6), 3)
    bz = G.batch(y, x)

    def run(bt, m):
        for _ in range(5):
            bt.score(m)

    reads = []

    def watch():  # the graph's totals read while both batches score (the timers' lock)
        for _ in range(20):
            reads.append(G.stats(blp._lib.K_SCORE)[1])

    th = [threading.Thread(target=run, args=(bx, 7)), threading.Thread(target=run, args=(bz, 3)),
          threading.Thread(target=watch)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert reads == sorted(reads) and all(3 <= r <= 13 for r in reads)
    bx.fetch(7)
    bz.fetch(3)
    assert G.stats(blp._lib.K_SCORE)[1] == 13
    bx.close()
    bz.close()
    assert G.stats(blp._lib.K_SCORE)[1] == 13


def test_empty_and_zero_division(gpu):
    G = blp.DeviceGraph(np.array([0, 2]), np.array([1, 3]))
    r = G.score_pairs(np.zeros(0, np.int32), np.zeros(0, np.int32))
    assert len(r["cn"]) == 0
    # x = 0 has H2 = {} (its only neighbour 1 has no other neighbour); y = 3 has N = {2};
    # union non-empty -> 0.0
    d0, d3 = G.dense([0, 3])
    r = G.score_pairs(np.array([d0], np.int32), np.array([d3], np.int32))
    assert r["cn"][0] == 0 and r["jaccard"][0] == 0.0 and r["adamic"][0] == 0.0
    # a node whose only edge is a self-loop has an empty hop-1 set: union of two empty sets
    G2 = blp.DeviceGraph(np.array([5, 6]), np.array([5, 7]))
    d5 = G2.dense([5])[0]
    with pytest.raises(ZeroDivisionError):
        G2.score_pairs(np.array([d5], np.int32), np.array([d5], np.int32))


def test_business_fix_adamic_matches_oracle(gpu):
    import blp_oracle as O

    d = os.path.join(GOLDEN, "bip", "train")
    ex = golden("bip/train", "examples.json")
    G = blp.load_edge_list(os.path.join(d, "graph.txt"))
    got = similarity.business(ex, G, ["adamic_adar"], [None], fix_adamic=True)[0]
    adj = O.load_edge_list(os.path.join(d, "graph.txt"))
    exp = O.business(ex, adj, [O.BUGGY_B_ADAMIC])[0]
    assert_same_scores(got, exp, "adamic_adar")


@pytest.mark.parametrize("variant", [None, "2"])
def test_coscheduled_passes_match_single_passes(gpu, variant, monkeypatch):
    # blp_batches_score: the user and business passes of one step run concurrently on their
    # own streams (the large-universe scorer held to a share of the CUs); results must equal
    # each pass scored alone, repeated steps included
    if variant:
        monkeypatch.setenv("BLP_VARIANT", variant[0])  # the large-universe block scorer on this graph
    rng = np.random.default_rng(21)
    a, b = bipartite_edges(rng, 20000, 1500, 200000)
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    x = np.repeat(rng.choice(nu, 300, replace=False), 40).astype(np.int32)
    y = rng.integers(nu, G.n, len(x)).astype(np.int32)
    alone_u = G.score_pairs(x, y, 7)
    alone_b = G.score_pairs(y, x, 3)
    ub, bb = G.batch(x, y), G.batch(y, x)
    for _ in range(3):
        G.score_batches([(ub, 7), (bb, 3)])
    got_u, got_b = ub.fetch(7), bb.fetch(3)
    for k in ("cn", "jaccard", "adamic"):
        np.testing.assert_array_equal(got_u[k], alone_u[k])
    for k in ("cn", "jaccard"):
        np.testing.assert_array_equal(got_b[k], alone_b[k])
    _check_against_oracle(a, b, x, y)


def test_adamic_exact_on_hub_pairs(gpu):
    """Adamic-Adar sums are exact (two-word integer sums of w * 2^58, blp_internal.h), so a pair
    with ~100K common neighbours -- far past where a 64-bit 2^-40 fixed point would wrap
    (Σw >= 2^23) for larger hubs -- still equals the correctly rounded sum of the reference's
    terms: math.fsum of (log deg)^-1 over H2(x) ∩ N(y) (similarity.py:116-126), bit for bit."""
    rng = np.random.default_rng(31)
    # two hub businesses reviewed by most of 120K users, plus background reviews
    nu = 120000
    users = np.arange(nu)
    a = np.concatenate([users, users[: nu * 9 // 10], rng.integers(0, nu, 200000)])
    b = np.concatenate([np.full(nu, nu), np.full(nu * 9 // 10, nu + 1), nu + 2 + rng.integers(0, 500, 200000)])
    G = blp.DeviceGraph(a, b)
    x = G.dense(np.array([0, 1, 2, 3], np.int64)).astype(np.int32)   # users
    y = G.dense(np.array([nu + 1, nu + 1, nu, nu + 2], np.int64)).astype(np.int32)  # hub targets
    got = G.score_pairs(x, y, 7)
    assert got["cn"][:3].min() > 100000  # hub pairs
    _check_against_oracle(a, b, x, y)  # bit-exact vs the C oracle's 128-bit sums
    # the same value from math.fsum over the reference's own terms
    deg = G.degree
    for i in range(len(x)):
        h2 = set(np.flatnonzero(_h2_mask(G, int(x[i]))))
        nb = set(G.col_idx[G.row_ptr[y[i]]:G.row_ptr[y[i] + 1]].tolist())
        terms = [math.log(int(deg[w])) ** -1 for w in h2 & nb if deg[w] > 1]
        assert got["adamic"][i] == math.fsum(terms)


def _h2_mask(G, x):
    """Exact distance-2 membership of every dense node (host-side BFS over the CSR mirror)."""
    rp, ci = G.row_ptr, G.col_idx
    d1 = ci[rp[x]:rp[x + 1]]
    m = np.zeros(G.n, bool)
    for z in d1:
        m[ci[rp[z]:rp[z + 1]]] = True
    m[d1] = False
    m[x] = False
    return m


def test_adamic_scale_and_weight_range(gpu):
    rng = np.random.default_rng(2)
    a, b = bipartite_edges(rng, 2000, 300, 20000)
    G = blp.DeviceGraph(a, b)
    assert G.aa_shift == 58
    # a custom weight table outside [0, 64) is refused (exactness bound, blp_internal.h)
    from blp._lib import lib, ptr
    import ctypes
    for bad in (-1.0, 2.0, float("nan")):
        w = np.array(G.aa_weight, np.float64)
        w[3] = bad
        h = ctypes.c_void_p()
        rc = lib().blp_graph_create(ptr(G.row_ptr), ptr(G.col_idx), G.n, ptr(w), 0, ctypes.byref(h))
        assert rc == -1 and "aa_weight" in lib().blp_last_error().decode()  # BLP_E_ARG


def test_concurrent_short_row_batches_share_wedge_bitmaps(gpu):
    """similarity.main creates its user and business batches on two host threads at once
    (similarity._score_both_ids). On a graph where every row is short, BOTH batches take the
    short-row scorer and ask the graph for its wedge-row bitmaps over their own universe, so
    the graph's bitmap cache is built from two threads concurrently (blp::wedge_bitmaps holds
    the graph's lock across lookup-or-build). Repeated on fresh graphs; every batch's scores
    must equal the oracle (similarity.py:20-106)."""
    from concurrent.futures import ThreadPoolExecutor

    rng = np.random.default_rng(11)
    seen_wbm = 0
    for rep in range(6):
        n_users, n_bus = 300, 200  # ~10 reviews per user, ~15 members per business: every row short
        u, b = bipartite_edges(rng, n_users, n_bus, 3000, zipf=0.0)
        G = blp.DeviceGraph(u, b, device=gpu)
        nu = G.n_col0
        x = rng.integers(0, nu, 6000).astype(np.int32)
        y = rng.integers(nu, G.n, len(x)).astype(np.int32)
        with ThreadPoolExecutor(2) as ex:
            fu = ex.submit(G.batch, x, y)
            fb = ex.submit(G.batch, y, x)
            ub, bb = fu.result(), fb.result()
        seen_wbm += sum(bt.plan().get("wedge_bitmaps", 0) for bt in (ub, bb))
        G.score_batches([(ub, 7), (bb, 7)])
        ids, oa, ob = dense_edges(u, b)
        og = coracle.OracleGraph(len(ids), oa, ob)
        for bt, xs, ys in ((ub, x, y), (bb, y, x)):
            got = bt.fetch(7)
            cn, jac, aa, _ = og.score_pairs(np.searchsorted(ids, G.node_ids[xs]), np.searchsorted(ids, G.node_ids[ys]), 7)
            np.testing.assert_array_equal(got["cn"], cn)
            np.testing.assert_array_equal(got["jaccard"], jac)
            np.testing.assert_array_equal(got["adamic"], aa)
        G.close()
    assert seen_wbm > 0  # the bitmaps were actually in play


def test_node2_planning_with_empty_row_runs(gpu):
    """The per-node two-hop statistics (node2.hip, computed on the device at graph creation) that
    blp_batch_create plans from and the wedge index sizes with: a graph whose dense ids hold a
    run of 200K isolated users between two populated blocks, so one CSR tile spans far more
    rows than its LDS table (the direct-atomic path). The batch universe equals the host
    computation over N(y) and N(N(x)), the wedge rows equal their host construction, and the
    scores equal the oracle (similarity.py:20-106)."""
    import ctypes

    rng = np.random.default_rng(21)
    n_users, n_bus = 300_000, 600
    users = np.concatenate([rng.integers(0, 1000, 6000), rng.integers(200_000, 201_000, 6000)])
    bus = n_users + (rng.pareto(1.0, len(users)) * 20).astype(np.int64) % n_bus
    n = n_users + n_bus
    A = np.ascontiguousarray(users, np.int32)
    Bv = np.ascontiguousarray(bus, np.int32)
    rp = np.zeros(n + 1, np.int64)
    ci = np.empty(2 * len(A), np.int32)
    sl = np.zeros(n, np.uint8)
    nnz = ctypes.c_int64(0)
    P = blp._lib.ptr
    blp._lib.check(blp.lib().blp_csr_from_edges(n, len(A), P(A), P(Bv), P(rp), P(ci), P(sl), ctypes.byref(nnz)))
    ci = ci[: nnz.value].copy()
    G = blp.DeviceGraph.from_csr(rp, ci, sl, n_users, device=gpu)
    present_u = np.flatnonzero(np.diff(rp)[:n_users] > 0)
    x = np.repeat(rng.choice(present_u, 80, replace=False), 15).astype(np.int32)
    y = rng.integers(n_users, n, len(x)).astype(np.int32)

    def universe(xs, ys):
        lo, hi = 1 << 62, -1
        for v in np.unique(ys):
            if rp[v + 1] > rp[v]:
                lo, hi = min(lo, ci[rp[v]]), max(hi, ci[rp[v + 1] - 1] + 1)
        for u in np.unique(xs):
            for z in ci[rp[u]:rp[u + 1]]:
                if rp[z + 1] > rp[z]:
                    lo, hi = min(lo, ci[rp[z]]), max(hi, ci[rp[z + 1] - 1] + 1)
        return lo & ~127, hi

    ids = np.arange(n)
    og = coracle.OracleGraph(n, A, Bv)
    for xs, ys in ((x, y), (y, x)):
        bt = G.batch(xs, ys)
        plan = bt.plan()
        assert (plan["lo"], plan["hi"]) == universe(xs, ys), plan
        bt.score(7)
        got = bt.fetch(7)
        cn, jac, aa, _ = og.score_pairs(xs, ys, 7)
        np.testing.assert_array_equal(got["cn"], cn)
        np.testing.assert_array_equal(got["jaccard"], jac)
        np.testing.assert_array_equal(got["adamic"], aa)
        bt.close()
    # wedge rows: x holds one when every neighbour row has <= 64 ids (wedge.hip), N(N(x)) back to back
    nv = ctypes.c_int64(0)
    blp._lib.check(blp.lib().blp_graph_wedge(G.handle, ctypes.byref(nv), None, None))
    if nv.value > 0:
        wp = np.empty(n + 1, np.int64)
        wedge = np.empty(4 * nv.value, np.int32)
        blp._lib.check(blp.lib().blp_graph_wedge(G.handle, ctypes.byref(nv), P(wp), P(wedge)))
        deg = np.diff(rp)
        for v in rng.choice(n, 400, replace=False):
            nbr = ci[rp[v]:rp[v + 1]]
            ok = len(nbr) > 0 and deg[nbr].max() <= 64
            assert (wp[v + 1] > wp[v]) == ok
            if ok:
                want = np.concatenate([ci[rp[z]:rp[z + 1]] for z in nbr])
                got_w = wedge[4 * wp[v]:4 * wp[v + 1]]
                np.testing.assert_array_equal(np.unique(got_w), np.unique(want))
                assert len(got_w) == (len(want) + 3) // 4 * 4
    G.close()


@pytest.mark.parametrize("knobs", [
    {},
    {"BLP_HEAVY_WORK": "50"},
    {"BLP_HEAVY_WORK": "50", "BLP_NO_WEDGE": "1"},
    {"BLP_HEAVY_WORK": "50000", "BLP_NO_WBM_BATCH": "1"},
    {"BLP_SPLIT": "3", "BLP_SPLIT_BIG": "1", "BLP_HASH_WORK": "600"},
    {"BLP_FORCE_GLOBAL": "1"},
])
def test_device_plan_scores_vs_oracle(gpu, knobs, monkeypatch):
    """blp_batch_create's planning pass on the device (k_plan_pairs / k_plan_sources: bounds, the
    universe, runs, the sources, build work, heavy and hash-set routing; the host planning loops
    were removed in round 6) on both sides, for source-grouped and shuffled pair lists: the plan
    is the same for a list and its shuffle where the runs do not matter, and every score equals
    the C oracle's (similarity.py:20-106)."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(21)
    a, b = bipartite_edges(rng, 30000, 1500, 300000)
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    x = np.repeat(np.sort(rng.choice(nu, 120, replace=False)), 40).astype(np.int32)
    y = rng.integers(nu, G.n, len(x)).astype(np.int32)
    perm = rng.permutation(len(x))
    ids, da, db = dense_edges(a, b)
    og = coracle.OracleGraph(len(ids), da, db)
    for xs, ys in ((x, y), (y, x), (x[perm], y[perm])):
        dev = G.batch(xs, ys)
        dev.score(7)
        rd = dev.fetch(7)
        cn, jac, aa, _ = og.score_pairs(np.searchsorted(ids, G.node_ids[xs]), np.searchsorted(ids, G.node_ids[ys]), 7)
        np.testing.assert_array_equal(rd["cn"], cn)
        np.testing.assert_array_equal(rd["jaccard"], jac)
        np.testing.assert_array_equal(rd["adamic"], aa)
        dev.close()
    _check_against_oracle(a, b, y[perm], x[perm])


def test_batch_pair_equals_two_batches(gpu):
    """blp_batch_create_pair (one upload, the business batch copies the user batch's device
    arrays swapped) gives the two batches blp_batch_create gives, scores and plans alike, for a
    source-grouped list and a shuffled one (similarity.main's two passes, similarity.py:20-106)."""
    rng = np.random.default_rng(23)
    a, b = bipartite_edges(rng, 30000, 1500, 300000)
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    x = np.repeat(np.sort(rng.choice(nu, 150, replace=False)), 30).astype(np.int32)
    y = rng.integers(nu, G.n, len(x)).astype(np.int32)
    perm = rng.permutation(len(x))
    for xs, ys in ((x, y), (x[perm], y[perm]), (x[:0], y[:0])):
        ub, bb = G.batch_pair(xs, ys)
        u1, b1 = G.batch(xs, ys), G.batch(ys, xs)
        assert ub.plan() == u1.plan() and bb.plan() == b1.plan()
        G.score_batches([(ub, 7), (bb, 3)])
        G.score_batches([(u1, 7), (b1, 3)])
        for p, q, m in ((ub, u1, 7), (bb, b1, 3)):
            rp, rq = p.fetch(m), q.fetch(m)
            for k in rp:
                np.testing.assert_array_equal(rp[k], rq[k])
        for bt in (ub, bb, u1, b1):
            bt.close()
    _check_against_oracle(a, b, x[perm], y[perm])


@pytest.mark.parametrize("cache_mb", ["0", "1", "8192"])
def test_device_scratch_cache_budgets(gpu, cache_mb):
    """The device scratch cache (released DevBuf blocks kept for reuse, graph.hip): no cache (0),
    a budget too small for most blocks (1 MiB: freed as before), and the default. In a child
    process (the budget is read once): both passes scored repeatedly through create / score /
    destroy cycles that reuse the cached blocks, every score equal to the C oracle's."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r'''
import os, sys
import numpy as np
sys.path[:0] = [os.path.join(ROOT, "bipartite-link-prediction_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import blp, coracle
from helpers import bipartite_edges, dense_edges
rng = np.random.default_rng(7)
a, b = bipartite_edges(rng, 40000, 2000, 300000)
G = blp.DeviceGraph(a, b)
ids, oa, ob = dense_edges(a, b)
og = coracle.OracleGraph(len(ids), oa, ob)
nu = G.n_col0
for rep in range(3):
    x = np.repeat(rng.choice(nu, 100 + 50 * rep, replace=False), 25).astype(np.int32)
    y = rng.integers(nu, G.n, len(x)).astype(np.int32)
    for xs, ys in ((x, y), (y, x)):
        got = G.score_pairs(xs, ys, 7)
        cn, jac, aa, _ = og.score_pairs(np.searchsorted(ids, G.node_ids[xs]), np.searchsorted(ids, G.node_ids[ys]), 7)
        assert np.array_equal(got["cn"], cn) and np.array_equal(got["jaccard"], jac) and np.array_equal(got["adamic"], aa)
G.close()
print("OK")
'''
    env = dict(os.environ, BLP_DEV_CACHE_MB=cache_mb)
    r = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % root + code], env=env, cwd=root, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])


def test_prewarm_concurrent_with_batches(gpu):
    """blp_stream_prewarm on other threads while batches are created, scored and destroyed (the
    pool's latch: stream_take waits while a prewarm creates streams; similarity.main prewarms on
    a spare thread): no deadlock, and every score equal to the single-threaded ones."""
    import threading

    rng = np.random.default_rng(29)
    a, b = bipartite_edges(rng, 20000, 1000, 150000)
    G = blp.DeviceGraph(a, b)
    nu = G.n_col0
    x = np.repeat(np.sort(rng.choice(nu, 80, replace=False)), 20).astype(np.int32)
    y = rng.integers(nu, G.n, len(x)).astype(np.int32)
    ref = G.score_pairs(x, y, 7)
    errs = []

    def warm():
        try:
            for _ in range(3):
                blp.prewarm(gpu, 16)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=warm) for _ in range(2)]
    for t in th:
        t.start()
    for _ in range(4):
        ub, bb = G.batch_pair(x, y)
        G.score_batches([(ub, 7), (bb, 3)])
        got = ub.fetch(7)
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k])
        ub.close()
        bb.close()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th) and not errs, errs


@pytest.mark.parametrize("mask", [3, 7])
def test_wedge_set_path_equals_grouped_path(gpu, mask, monkeypatch):
    """The business side on the graph's dense wedge-set index (k_score_wset, round 6: CN(x, y) =
    #{c in N(y), c != x : x in N(N(c))}, pair by pair in caller order, no grouping) gives the
    grouped short-row scorer's values bit for bit, and the C oracle's (similarity.py:63-106):
    pairs grouped by user and shuffled, repeated pairs, and pairs whose user reviewed the business
    (c == x in N(y) must not count). mask 7 is the fix_adamic business pass (exact AA words)."""
    rng = np.random.default_rng(5)
    a, b = bipartite_edges(rng, 9000, 700, 70000)
    G = blp.DeviceGraph(a, b)
    nu = G.n - len(np.unique(b))
    users = np.repeat(rng.choice(nu, 150, replace=False), 40).astype(np.int32)
    bus = rng.integers(nu, G.n, len(users)).astype(np.int32)
    rp, ci = G.row_ptr, G.col_idx
    own = np.array([ci[rp[u]] for u in users[:200:10]], np.int32)  # businesses the user reviewed
    users = np.concatenate([users, users[:200:10], users[:50]])
    bus = np.concatenate([bus, own, bus[:50]])
    for order in ("grouped", "shuffled"):
        if order == "shuffled":
            p = rng.permutation(len(users))
            users, bus = users[p], bus[p]
        got = G.batch(bus, users)
        assert got.kernel(mask) == "k_score_wset<%s>" % ("true" if mask & 4 else "false"), got.kernel(mask)
        got.score(mask)
        rw = got.fetch(mask)
        monkeypatch.setenv("BLP_NO_WSET", "1")
        ref = G.batch(bus, users)
        monkeypatch.delenv("BLP_NO_WSET")
        assert ref.kernel(mask).startswith("k_score_short"), ref.kernel(mask)
        ref.score(mask)
        rs = ref.fetch(mask)
        for k in ("cn", "jaccard") + (("adamic",) if mask & 4 else ()):
            np.testing.assert_array_equal(rw[k], rs[k], err_msg=k)
        got.close()
        ref.close()
    _check_against_oracle(a, b, bus, users, mask)


@pytest.mark.parametrize("extra", ["user-user", "business-business"])
def test_wedge_set_path_refuses_non_bipartite(gpu, extra):
    """The wedge-set path rests on N(x) lying outside the sets' range (distance 1 never in the
    universe) -- a bipartite graph. A review graph with a few user-user or business-business
    edges puts distance-2 users, or a business's business neighbours, in play; the batch must
    take the grouped path, and its scores must equal the C oracle's (similarity.py:63-106)."""
    rng = np.random.default_rng(8)
    a, b = bipartite_edges(rng, 5000, 400, 30000)
    users, bus = np.unique(a), np.unique(b)
    k = 40
    if extra == "user-user":
        ea, eb = rng.choice(users, k), rng.choice(users, k)
    else:
        ea, eb = rng.choice(bus, k), rng.choice(bus, k)
    a2, b2 = np.concatenate([a, ea]), np.concatenate([b, eb])
    G = blp.DeviceGraph(a2, b2)
    dense = {int(v): i for i, v in enumerate(G.node_ids)}  # original id -> dense id
    u_src = np.array([dense[int(v)] for v in rng.choice(users, 80, replace=False)], np.int32)
    x = np.repeat(u_src, 25).astype(np.int32)
    y = np.array([dense[int(v)] for v in rng.choice(bus, len(x))], np.int32)
    bt = G.batch(y, x)
    assert not bt.kernel(3).startswith("k_score_wset"), bt.kernel(3)
    bt.close()
    _check_against_oracle(a2, b2, y, x, 3)
    _check_against_oracle(a2, b2, y, x, 7)
