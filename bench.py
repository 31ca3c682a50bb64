"""Benchmark: candidate (user, business) pairs scored per second on MI355X.

Workload (BASELINE.json configs[1], "config 2"): synthetic review graph of 1M users x
100K businesses from 10M draws (9,947,457 unique edges), 10K example
users per GPU, their exact distance-3 candidates sampled at 1% (dataset_maker.py:137-144)
-> ~7M (user, business) pairs per GPU. One step = the device work of similarity.main on
that batch (similarity.py:17-18): the user side (u_cn, u_jaccard, u_adamic fused) and the
business side (b_cn, b_jaccard; b_adamic is the reference's empty bug file), each pass
grouping the raw pair list by source on the device and scoring every pair. Inputs are in
HBM before the timed region; results stay in HBM.

Multi-GPU: one process per GPU (torchrun); every rank holds a replica of the graph and
scores its own 10K users (weak scaling, no data-path collective, SURVEY.md §8(e) "small
configs may use replicas"). Timing: barrier + device sync on both sides, max over ranks.

Prints ONE JSON line (rank 0). Extras: roofline of the dominant kernel (user-side scorer,
HIP events on its stream), the CPU baseline (C oracle, 1 thread, bounded sample) and a
parity spot-check plus AUCs of the scores.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "bipartite-link-prediction_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import blp  # noqa: E402
from blp import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "candidate (user,business) pairs scored/sec at 1/2/4/8 GPUs; AUC parity vs ref"


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


from blp.dist import Dist  # noqa: E402  (torch.distributed plumbing: barrier, max/sum, exchange)


def _device(dist):
    """The rank's GPU: LOCAL_RANK (one process per GPU). BLP_DEVICE overrides it -- used only
    to rehearse the multi-rank path with several ranks on a one-GPU box."""
    return int(os.environ.get("BLP_DEVICE", dist.local))


def alg_bytes(G, x, y, mask, cn=None):
    """SURVEY.md §8(d) algorithmic bytes of one scorer pass over pairs (x -> y).

    per source x:  16 + 4 d_x + sum_{z in N(x)} (16 + 4 d_z)     (build H2(x))
    per pair:      8 (pair ids) + 16 + 4 d_y (scan N(y)) + 8 CN (AA weights, if AA)
                   + 4 (cn) + 8 (jaccard, if J) + 8 (adamic, if AA)"""
    d = G.hop1_size.astype(np.int64)
    src = np.unique(x)
    rp, ci = G.row_ptr, G.col_idx
    dz = d[ci]  # degree of each neighbour entry
    csum = np.concatenate([[0], np.cumsum(dz)])
    nbr_deg_sum = csum[rp[src + 1]] - csum[rp[src]]
    per_src = (16 + 4 * d[src] + 16 * d[src] + 4 * nbr_deg_sum).sum()
    per_pair = len(x) * (8 + 16 + 4) + 4 * d[y].sum()
    if mask & blp.JACCARD:
        per_pair += 8 * len(x)
    if mask & blp.ADAMIC:
        per_pair += 8 * len(x) + 8 * int(cn.astype(np.int64).sum())
    return int(per_src + per_pair)


def wset_alg_bytes(G, x, y, mask):
    """Algorithmic bytes of the wedge-set scorer (k_score_wset) over pairs
    (x business, y user), in caller order with no grouping:
    per pair:  8 (pair ids) + 16 (rp[y], rp[y + 1]) + 4 d_y (N(y), coded ids)
               + 4 d_y (the word of x in W(c) for each c in N(y)) + 4 (|H2(x)|)
               + 4 (cn) + 8 (jaccard, if J) + 8 (adamic, if AA)"""
    d = G.hop1_size.astype(np.int64)
    per_pair = len(x) * (8 + 16 + 4 + 4) + 8 * int(d[y].sum())
    if mask & blp.JACCARD:
        per_pair += 8 * len(x)
    if mask & blp.ADAMIC:
        per_pair += 8 * len(x)
    return int(per_pair)


def pmc_fields(kernel, pattern, sec=None):
    """HBM-side bytes per launch of `kernel` from the newest committed PMC summary matching
    `pattern` under profiles/ (written by profiles/summarize.py from separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of the same command): newest round first (rNN_ prefix),
    then the highest _vM, then the name. Reported side by side, because MI355X_MICROARCH.md
    (HBM) calibrates FETCH_SIZE only for wide coalesced streaming reads (exactly half the
    bytes) and these kernels also gather:
      traffic      = 2 x FETCH_SIZE + WRITE_SIZE (the guide's streaming correction)
      traffic_raw  = FETCH_SIZE + WRITE_SIZE     (uncorrected)
    frac_dram (over the same kernel time `sec`) is given for both; traffic_source names the
    file and its measured kernel time (avg over its launches)."""
    import glob
    import re

    def key(f):
        b = os.path.basename(f)
        r = re.match(r"r(\d+)_", b)
        v = re.search(r"_v(\d+)", b)
        return (int(r.group(1)) if r else -1, int(v.group(1)) if v else -1, b)

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), key=key, reverse=True):
        try:
            rows = json.load(open(f))
        except Exception:
            continue
        for r in rows if isinstance(rows, list) else []:
            if kernel in r.get("kernel", "") and r.get("fetch_kb_raw") and r.get("write_kb") is not None:
                fetch, write = 1024.0 * r["fetch_kb_raw"], 1024.0 * r["write_kb"]
                out = {"traffic": 2 * fetch + write, "traffic_raw": fetch + write,
                       "traffic_source": "%s (kernel avg %.3f ms there)" % (os.path.relpath(f, ROOT),
                                                                             r["avg_us"] / 1e3),
                       "profile_kernel_ms": r["avg_us"] / 1e3}
                if sec:
                    out["frac_dram"] = out["traffic"] / sec / 1e9 / HBM_PEAK_GBS
                    out["frac_dram_raw"] = out["traffic_raw"] / sec / 1e9 / HBM_PEAK_GBS
                return out
    return {"traffic": None, "traffic_source": "no committed PMC summary for %s matching profiles/%s" % (kernel, pattern)}


def pmc_limiter(kernel, pattern):
    """What bounds `kernel`, from the newest committed counter summary matching `pattern` under
    profiles/ (profiles/pmc_report.py output of separate SQ / TCC --pmc passes): the share of
    wave cycles spent waiting, the share of LDS-active cycles lost to bank conflicts, and the L2
    hit rate. None when no summary names the kernel."""
    import glob
    import re

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)),
                   key=lambda f: (int((re.match(r"r(\d+)_", os.path.basename(f)) or [0, -1])[1]), f), reverse=True)
    for f in files:
        c, cur = {}, None
        for line in open(f):
            if not line.startswith(" "):
                cur = kernel in line
                continue
            if cur:
                parts = line.split()
                if len(parts) == 2:
                    c[parts[0]] = float(parts[1])
        if c.get("SQ_WAVE_CYCLES"):
            def ratio(a, b):
                return c.get(a, 0.0) / c[b] if c.get(b) else float("nan")
            hit = c.get("TCC_HIT_sum", 0.0)
            miss = c.get("TCC_MISS_sum", 0.0)
            return ("latency: waves wait %.0f%% of their cycles; %.0f%% of LDS-active cycles are bank conflicts; "
                    "L2 hit %.0f%% (%s)" % (100 * ratio("SQ_WAIT_ANY", "SQ_WAVE_CYCLES"),
                                             100 * ratio("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"),
                                             100 * hit / (hit + miss) if hit + miss else float("nan"),
                                             os.path.relpath(f, ROOT)))
    return None


def cpu_baseline(og, ex_x, ex_y, target_s=15.0):
    """C oracle (oracle/oracle.c), 1 thread, on a bounded sample of the same workload:
    all pairs of a subset of the example users (user side) and all pairs of a subset of
    the candidate businesses (business side); rate = 1 / (1/r_user + 1/r_business)."""
    rng = np.random.default_rng(123)

    def side_rate(src_arr, dst_arr, mask, budget):
        srcs = np.unique(src_arr)
        rng.shuffle(srcs)
        k = max(1, min(len(srcs), 8))
        done_pairs, spent, used = 0, 0.0, 0
        while spent < budget and used < len(srcs):
            pick = srcs[used:used + k]
            used += len(pick)
            sel = np.isin(src_arr, pick)
            t = time.perf_counter()
            og.score_pairs(src_arr[sel], dst_arr[sel], mask, nthreads=1)
            spent += time.perf_counter() - t
            done_pairs += int(sel.sum())
            k = min(k * 2, 4096)
        return done_pairs / spent, done_pairs, used, spent

    ru, pu, su, tu = side_rate(ex_x, ex_y, 7, target_s / 2)
    rb, pb, sb, tb = side_rate(ex_y, ex_x, 3, target_s / 2)
    rate = 1.0 / (1.0 / ru + 1.0 / rb)
    return {"value": rate, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": "C oracle (oracle/oracle.c, reference algorithm: per-source exact BFS 2-hop set, per-pair "
                      "N(y) scan), 1 thread: user side %d pairs of %d users in %.1fs (%.0f pairs/s), business "
                      "side %d pairs of %d businesses in %.1fs (%.0f pairs/s); combined = harmonic" %
                      (pu, su, tu, ru, pb, sb, tb, rb)}


def oracle_full(og, ex_x, ex_y, b_mask=3):
    """Every pair of the step scored by the C oracle on all of this host's cores (OpenMP,
    dynamic per source): the full-workload parity reference AND the multicore CPU baseline
    (SURVEY.md §8(d)(ii)). Same arithmetic as similarity.py:108-126."""
    nt = max(1, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0)))
    t0 = time.perf_counter()
    ucn, ujac, uaa, _ = og.score_pairs(ex_x, ex_y, 7, nthreads=nt)
    tu = time.perf_counter() - t0
    t0 = time.perf_counter()
    bcn, bjac, baa, _ = og.score_pairs(ex_y, ex_x, b_mask, nthreads=nt)
    tb = time.perf_counter() - t0
    res = {"user": {"cn": ucn, "jaccard": ujac, "adamic": uaa}, "business": {"cn": bcn, "jaccard": bjac}}
    if b_mask & 4:
        res["business"]["adamic"] = baa
    multi = {"value": len(ex_x) / (tu + tb), "unit": "pairs/s", "cores": nt, "kind": "port",
             "sample": "C oracle, %d OpenMP threads, the WHOLE step: user side %d pairs (CN+J+AA) in %.2fs, business "
                       "side %d pairs (CN+J) in %.2fs" % (nt, len(ex_x), tu, len(ex_x), tb)}
    return res, multi


def full_parity(ex_l, gpu, ora):
    """All pairs of both sides, bit-exact: CN, Jaccard (correctly rounded quotient) and
    Adamic-Adar (the correctly rounded sum of the reference's terms on both sides -- the
    engine's two-word integer sums and the C oracle's 128-bit sums, blp_internal.h;
    similarity.py:108-126). AUC (eval.py:26) of the GPU scores and of the oracle scores side
    by side: identical, ties included, because the scores are."""
    import importlib

    ev = importlib.import_module("eval")
    out = {"pairs_checked": int(len(ex_l)) * 2, "pairs_per_side": int(len(ex_l))}
    ok = True
    auc = {}
    for side, keys in (("user", ("cn", "jaccard", "adamic")), ("business", ("cn", "jaccard", "adamic"))):
        for k in keys:
            if k not in ora[side] or gpu[side].get(k) is None:
                continue
            g, o = gpu[side][k], ora[side][k]
            same = bool(np.array_equal(g, o))
            out["%s_%s_exact" % (side[0], k)] = same
            ok &= same
            name = "%s_%s" % (side[0], k)
            ag, ao = ev.roc_auc(ex_l, g), ev.roc_auc(ex_l, o)
            auc[name] = {"gpu": ag, "oracle": ao, "equal": bool(ag == ao)}
            ok &= ag == ao
    out["auc"] = auc
    out["auc_equal"] = all(v["equal"] for v in auc.values())
    out["ok"] = bool(ok)
    return out


def _build_elems(G, x):
    """sum over distinct sources x of sum_{z in N(x)} |N(z)|: elements read to build the H2 bitmaps."""
    d = G.hop1_size.astype(np.int64)
    src = np.unique(x)
    csum = np.concatenate([[0], np.cumsum(d[G.col_idx])])
    return int((csum[G.row_ptr[src + 1]] - csum[G.row_ptr[src]]).sum())


def _dense_edges(G):
    """Edge list (dense ids, each undirected edge once, self-loops restored) from the CSR."""
    rows = np.repeat(np.arange(G.n, dtype=np.int32), np.diff(G.row_ptr))
    keep = rows < G.col_idx
    a = rows[keep]
    b = G.col_idx[keep]
    loops = np.flatnonzero(G.self_loop).astype(np.int32)
    return np.concatenate([a, loops]), np.concatenate([b, loops])


# FP64 MFMA ceiling, MEASURED on this chip (MI355X_MICROARCH.md lists no FP64 rate): the probe
# profiles/scripts/mfma_f64_peak.hip sustains 75 TF/s of v_mfma_f64_16x16x4f64 with independent
# accumulation chains on every SIMD (profiles/r01_mfma_f64_peak.txt); AMD's spec value is 78.6.
FP64_MFMA_PEAK_TFS = 75.0
FP64_MFMA_PEAK_SOURCE = "measured: profiles/r01_mfma_f64_peak.txt (v_mfma_f64_16x16x4f64, independent chains)"


def run_svd(args):
    """Config 4 (BASELINE.json configs[3]): rank-64 truncated SVD of the binary 2M x 200K
    matrix of a 50M-draw review graph. Host ARPACK factorisation (svd.py:24), timed apart;
    the timed step is the GPU reconstruction: every business scored for 10K users on fp64
    MFMA with a fused top-k (plus the candidate-pair kernel as an extra line item)."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla

    from blp.factor import DeviceSVD

    dist = Dist()
    dev = _device(dist)
    blp.lib()
    U, B, D = synth.CONFIGS["c4"]
    t0 = time.time()
    u, b = synth.review_edges(U, B, D, seed=0)
    M = sp.csr_matrix((np.ones(len(u)), (u, b - U)), shape=(U, B))
    M.sum_duplicates()
    M.data[:] = 1.0
    del u, b
    log("matrix %dx%d, %d nnz in %.1fs" % (U, B, M.nnz, time.time() - t0))
    from blp import factor as F

    st = F.FactorStats()
    t0 = time.time()
    us_g, s_g, v_g = F.svds(M, k=64, device=dev, stats=st, return_us=True)
    fact_s = time.time() - t0
    log("GPU svds k=64: %d iterations (Ritz settled at %s) in %.2fs (SpMM %.0f ms, dense %.0f ms)" %
        (st.iterations, st.converged_at, fact_s, st.spmm_ms, st.dense_ms))
    arpack_s = None
    if dist.rank == 0 and not args.no_cpu_baseline:
        t0 = time.time()
        uu, ss, vt = spla.svds(M, k=64)
        arpack_s = time.time() - t0
        log("host ARPACK svds k=64 in %.1fs" % arpack_s)
    else:
        uu, ss, vt = None, None, None
    us = us_g
    vt_g = np.ascontiguousarray(v_g.T)
    rng = np.random.default_rng(dist.rank)
    deg = np.diff(M.indptr)
    users = np.sort(rng.choice(np.flatnonzero(deg > 0), size=args.users, replace=False)).astype(np.int32)
    ex_off = M.indptr[users.astype(np.int64) + 1] - M.indptr[users]
    ex_off = np.r_[0, np.cumsum(ex_off)].astype(np.int64)
    ex_col = np.concatenate([M.indices[M.indptr[r]:M.indptr[r + 1]] for r in users]).astype(np.int32)
    S = DeviceSVD(us, np.ascontiguousarray(v_g), device=dev)
    # inputs resident in HBM before the timed region; outputs stay there (read back after it)
    import torch

    cuda = torch.device("cuda", dev)
    d_users = torch.from_numpy(users).to(cuda)
    d_ex = (torch.from_numpy(ex_off).to(cuda), torch.from_numpy(ex_col).to(cuda))
    d_cols = torch.empty((len(users), args.topk), dtype=torch.int32, device=cuda)
    d_scores = torch.empty((len(users), args.topk), dtype=torch.float64, device=cuda)
    torch.cuda.synchronize(cuda)
    # the headline step is the dense reconstruction: every (user, business) score on fp64 MFMA
    # (the norm-pruned top-k, the library default, is timed after it as its own line)
    S.set_prune(False)
    for _ in range(args.warmup):
        S.topk_device(d_users, args.topk, d_cols, d_scores, exclude=d_ex)
    S.sync()
    ms0, n0 = S.stats(1)
    dist.barrier()
    blp.device_sync(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        S.topk_device(d_users, args.topk, d_cols, d_scores, exclude=d_ex)
    S.sync()
    blp.device_sync(dev)
    wall = time.perf_counter() - t_start
    cols, scores = d_cols.cpu().numpy(), d_scores.cpu().numpy()
    dist.barrier()
    ms1, n1 = S.stats(1)
    kern_s = (ms1 - ms0) / 1e3 / max(n1 - n0, 1)
    # the host entry point (blp_svd_topk: uploads, sync, downloads) must give the same lists
    hc, hs = S.topk(users[:64], args.topk, exclude=(ex_off[:65], ex_col[:ex_off[64]]))
    host_same = bool(np.array_equal(hc, cols[:64]) and np.array_equal(hs, scores[:64]))
    t_max = dist.max(wall) / args.steps
    # the norm-pruned top-k (blp_svd_set_prune, default on): same lists, far fewer MFMA tiles
    S.set_prune(True)
    p_cols = torch.empty_like(d_cols)
    p_scores = torch.empty_like(d_scores)
    for _ in range(max(args.warmup, 1)):
        S.topk_device(d_users, args.topk, p_cols, p_scores, exclude=d_ex)
    S.sync()
    S.tiles()
    pm0, pn0 = S.stats(1)
    dist.barrier()
    blp.device_sync(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        S.topk_device(d_users, args.topk, p_cols, p_scores, exclude=d_ex)
    S.sync()
    p_wall = dist.max(time.perf_counter() - t_start) / args.steps
    pm1, pn1 = S.stats(1)
    t_scored, t_dense = S.tiles()
    pruned = {"ms_per_step": 1e3 * p_wall, "kernel_ms": (pm1 - pm0) / max(pn1 - pn0, 1),
              "pairs_ranked_per_s": dist.sum(len(users) * B) / p_wall,
              "tiles_scored_fraction": t_scored / max(t_dense, 1),
              "lists_equal_dense": bool(np.array_equal(p_cols.cpu().numpy(), cols) and
                                        np.array_equal(p_scores.cpu().numpy(), scores)),
              "note": "exact top-k by the norm bound |us[u].v[b]| <= ||us[u]|| ||v[b]||: businesses in "
                      "||v|| descending order, a block of 16 users stops once the bound falls below all "
                      "its k-th scores; value counts pairs ranked, not pairs reconstructed"}
    scored = len(users) * B
    flops = 2.0 * len(users) * B * 64
    # candidate-pair reconstruction (svd.py:28-30 shape): 750 random businesses per user
    pr = np.repeat(users, 750)
    pc = rng.integers(0, B, len(pr)).astype(np.int32)
    S.score_pairs(pr, pc)
    p0, q0 = S.stats(0)
    for _ in range(args.steps):
        S.score_pairs(pr, pc)
    p1, q1 = S.stats(0)
    pair_s = (p1 - p0) / 1e3 / max(q1 - q0, 1)
    pair_bytes = len(users) * 64 * 8 + len(pr) * (64 * 8 + 8 + 8)
    # parity of the top-k on >= 1000 users: fp64 numpy on the same factors, 64 users per chunk
    n_chk = len(users) if args.svd_parity_users <= 0 else min(len(users), args.svd_parity_users)
    ok = True
    bids = np.arange(B)
    for c0 in range(0, n_chk, 64):
        c1 = min(n_chk, c0 + 64)
        full = us[users[c0:c1]] @ vt_g
        for i in range(c0, c1):
            full[i - c0, ex_col[ex_off[i]:ex_off[i + 1]]] = -np.inf
            ok &= bool(np.array_equal(exact_topk(full[i - c0], bids, args.topk), cols[i]))
    del full
    svd_pmc = pmc_fields("k_svd_topk", "r*_svd_c4*.json")  # HBM bytes per launch (PMC)
    svd_pmc.pop("frac_dram", None)
    out = {
        "metric": METRIC, "value": dist.sum(scored) / t_max, "unit": "pairs/s", "n_gpus": dist.world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * t_max, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "config4: svd.py rank-64 truncated SVD, synthetic 2M users x 200K businesses, 50M draws "
                               "(%d unique edges); step = every business scored for %d users on fp64 MFMA + fused "
                               "top-%d (own reviews excluded); rank-64 factorisation on the GPU (blp.factor.svds) "
                               "%.2fs, not in the step" % (M.nnz, len(users), args.topk, fact_s),
                   "global_batch": int(dist.sum(scored)), "parallelism": "replicas x%d" % dist.world},
        "roofline": {"bound": "mfma", "achieved": flops / kern_s / 1e12, "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                     "frac": flops / kern_s / 1e12 / FP64_MFMA_PEAK_TFS, "peak_source": FP64_MFMA_PEAK_SOURCE,
                     "frac_of_spec_78.6": flops / kern_s / 1e12 / 78.6,
                     "kernel": "k_svd_topk<64> + k_svd_merge", "kernel_ms": 1e3 * kern_s, **svd_pmc},
        "pairs_kernel": {"pairs": int(len(pr)), "ms": 1e3 * pair_s, "pairs_per_s": len(pr) / pair_s,
                         "alg_GBps": pair_bytes / pair_s / 1e9},
        "parity": {"topk_users_checked": int(n_chk), "exact": bool(ok), "host_entry_point_same": host_same},
        "pruned_topk": pruned,
        "factorization": {"gpu_s": fact_s, "create_s": st.create_s, "iterations": st.iterations,
                          "ritz_settled_at": st.converged_at,
                          "spmm_ms": st.spmm_ms, "dense_ms": st.dense_ms},
    }
    if arpack_s is not None:
        # the reference's own factorisation (svd.py:24) on the host, and the agreement of the
        # two rank-64 reconstructions on random (user, business) pairs
        import blp_oracle

        ref = np.einsum("ij,ji->i", (uu * ss)[pr[:200000]], vt[:, pc[:200000]])
        got = np.einsum("ij,ji->i", us[pr[:200000]], vt_g[:, pc[:200000]])
        cdeg = np.diff(M.tocsc().indptr)
        zero = (deg[pr[:200000]] == 0) | (cdeg[pc[:200000]] == 0)
        out["factorization"].update({"host_arpack_s": arpack_s, "speedup": arpack_s / fact_s,
                                     "host_arpack_note": "scipy.sparse.linalg.svds(M, k=64) on the same matrix "
                                                         "(svd.py:24, the reference's own call), host BLAS threads"})
        # per-entry 1e-5 relative, exact-zero rule for empty rows/columns, near-zero floor
        out["parity"]["gpu_factor_vs_arpack"] = blp_oracle.svd_entry_parity(got, ref, zero)
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = svd_cpu_baseline(us, vt_g, users, B, args.cpu_seconds)
    if dist.rank == 0:
        print(json.dumps(out), flush=True)


def svd_cpu_baseline(us, vt, users, n_cols, target_s=15.0):
    """The reference's reconstruction loop (svd.py:28-30: examples[u][b] = np.dot(us[row],
    vt[:, col]) per pair) restated on the same factors, 1 thread, over a bounded sample of the
    step's own pairs: the sampled users' rows against every business, in the step's order, for
    about target_s seconds. pairs/s, the unit of the bench line."""
    done, t0 = 0, time.perf_counter()
    vt = np.ascontiguousarray(vt)
    i = 0
    while time.perf_counter() - t0 < target_s:
        row = us[users[i % len(users)]]
        for col in range(0, n_cols, 1):
            np.dot(row, vt[:, col])
            done += 1
            if done % 65536 == 0 and time.perf_counter() - t0 >= target_s:
                break
        i += 1
    spent = time.perf_counter() - t0
    return {"value": done / spent, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": "svd.py:28-30 restated: np.dot(us[row], vt[:, col]) per (user, business) pair on the step's "
                      "factors, users in the step's order against every business, 1 thread: %d pairs in %.1fs" %
                      (done, spent)}


def topk_alg_bytes(G, src, h2_sum, push_sum, k, n_methods, dense_adds=0, dense_add_bytes=0):
    """SURVEY.md §8(d) "Full-candidate top-k (user)": per user the H2 bytes
    (16 + 4 d_u + sum_{b in N(u)} (16 + 4 d_b)) + sum_{w in H2(u)} (16 + 4 d_w) + 12 k per list.
    The last sum comes from the kernel's own work counters. push_sum is the row entries the
    kernel actually pushes (stats 6: the walk plus the dense corrections, not the 10.27G of the
    whole H2 volume -- the hot targets' counts are precomputed at topk_create), and each dense
    hot-target add reads its precomputed counts and fused AA words (stats 7 x stats 8)."""
    d = G.hop1_size.astype(np.int64)
    csum = np.concatenate([[0], np.cumsum(d[G.col_idx])])
    nbr = csum[G.row_ptr[src + 1]] - csum[G.row_ptr[src]]
    h2_bytes = int((16 + 4 * d[src] + 16 * d[src] + 4 * nbr).sum())
    return h2_bytes + 16 * h2_sum + 4 * push_sum + dense_adds * dense_add_bytes + 12 * k * n_methods * len(src)


def _oracle_graph(G):
    """C oracle over the same edges, on the engine's dense ids (identity id maps)."""
    import coracle

    ident = np.arange(G.n, dtype=np.int32)
    return coracle.OracleGraph(G.n, *_dense_edges(G)), ident, ident


def exact_topk(scores, ids, k):
    """Positions of the best k of `scores` (score descending, then id ascending), exactly: the
    k-th largest value by partition, then a sort of everything at or above it (ties included)."""
    n = len(scores)
    if n > k:
        vk = -np.partition(-scores, k - 1)[k - 1]
        cand = np.flatnonzero(scores >= vk)
    else:
        cand = np.arange(n)
    return cand[np.lexsort((ids[cand], -scores[cand]))][:k]


def topk_parity(G, src, k, res, n_users=200, batch=250):
    """Not timed: for `n_users` users (all of them with --topk-parity-users 0) the C oracle
    enumerates the exact hop-3 set, scores every candidate (all host cores) and ranks them
    (score desc, id asc), `batch` users at a time; the Jaccard lists must match exactly, so must
    the Adamic-Adar lists (exact sums on both sides; their values also equal the pair
    kernel's), and |H3(u)| must equal the kernel's candidate count."""
    og, to_o, from_o = _oracle_graph(G)
    nt = max(1, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0)))
    n_users = len(src) if n_users <= 0 else min(n_users, len(src))
    pick = np.sort(np.random.default_rng(5).choice(len(src), n_users, replace=False))
    ok_j = ok_a = ok_n = True
    n_cand = 0
    pair_x, pair_y, pair_v = [], [], []
    for b0 in range(0, len(pick), batch):
        pb = pick[b0:b0 + batch]
        xs_o = to_o[src[pb]]
        counts, mem = og.hop3(xs_o)
        n_cand += int(counts.sum())
        ok_n &= bool(np.array_equal(res["ncand"][pb], counts))
        xrep = np.repeat(xs_o, counts).astype(np.int32)
        _, jac, aa, _ = og.score_pairs(xrep, mem, 7, nthreads=nt)
        starts = np.r_[0, np.cumsum(counts)]
        for j, i in enumerate(pb):
            s_, e_ = starts[j], starts[j + 1]
            dense = from_o[mem[s_:e_]]
            o = exact_topk(jac[s_:e_], dense, k)
            ok_j &= bool(np.array_equal(res["jaccard"][0][i][:len(o)], dense[o]) and
                         np.array_equal(res["jaccard"][1][i][:len(o)], jac[s_:e_][o]))
            # Adamic-Adar: exact sums on both sides (blp_internal.h), so the lists match exactly too
            oa = exact_topk(aa[s_:e_], dense, k)
            ok_a &= bool(np.array_equal(res["adamic_adar"][0][i][:len(oa)], dense[oa]) and
                         np.array_equal(res["adamic_adar"][1][i][:len(oa)], aa[s_:e_][oa]))
            cols, sc = res["adamic_adar"][0][i], res["adamic_adar"][1][i]
            v = cols >= 0
            pair_x.append(np.full(int(v.sum()), src[i], np.int32))
            pair_y.append(cols[v])
            pair_v.append(sc[v])
        del mem, xrep, jac, aa
    pair = G.score_pairs(np.concatenate(pair_x), np.concatenate(pair_y), 7)["adamic"]
    ok_a &= bool(np.array_equal(pair, np.concatenate(pair_v)))
    return {"users_checked": int(len(pick)), "candidates_checked": n_cand, "jaccard_exact": ok_j,
            "adamic_exact_and_pair_kernel_equal": ok_a, "n_candidates_exact": ok_n}


def topk_cpu_baseline(G, src, k, target_s=15.0):
    """C oracle, 1 thread: exact hop-3 candidates of a few users (og_hop3), every candidate
    scored (og_score_pairs: CN, Jaccard, Adamic-Adar), top-k by sort; candidate pairs/s."""
    og, to_oracle, _ = _oracle_graph(G)
    done, spent, used = 0, 0.0, 0
    while spent < target_s and used < len(src):
        x = to_oracle[src[used]]
        used += 1
        t = time.perf_counter()
        counts, members = og.hop3([x])
        xs = np.full(len(members), x, np.int32)
        cn, jac, aa, _ = og.score_pairs(xs, members, 7, nthreads=1)
        for sc in (jac, aa):
            np.lexsort((members, -sc))[:k]
        spent += time.perf_counter() - t
        done += len(members)
    return {"value": done / spent, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": "C oracle (oracle/oracle.c), 1 thread: exact hop-3 candidate set of %d users (%d pairs) "
                      "scored with CN+Jaccard+AA and sorted for top-%d, %.1fs" % (used, done, k, spent)}


def run_topk(args):
    """Config 3 (BASELINE.json configs[2]): the config-2 graph; for 10K users per GPU EVERY
    exact-distance-3 business is scored with Jaccard and Adamic-Adar and the top-k kept
    (k = 20, eval.py:10). One step = one blp_topk_run over all users. value = candidate
    pairs scored (sum |H3(u)|) per second."""
    from blp.topk import TopK

    dist = Dist()
    dev = _device(dist)
    blp.lib()
    U, B, D = synth.CONFIGS[args.config]
    t0 = time.time()
    a, b = synth.review_edges(U, B, D, seed=0)
    G = blp.DeviceGraph(a, b, device=dev)
    del a, b
    graph_s = time.time() - t0
    log("graph: %d nodes, %d unique edges, built in %.1fs" % (G.n, G.nnz // 2, graph_s))
    G.n_users_hint = U  # the same users make_examples samples for config 2
    src = synth.sample_users(G, args.users, seed=dist.rank)
    t0 = time.time()
    T = TopK(G, "user")  # the handle's graph indexes: permuted rows, wedge rows, hot-target dense counts
    create_s = time.time() - t0
    T.set_sources(src)
    log("top-k engine: %s in %.1fs" % (T.info(), time.time() - t0))
    mask = args.topk_mask
    for _ in range(args.warmup):
        T.run(args.topk, mask)
    blp.device_sync(dev)
    T.stats_reset()
    dist.barrier()
    blp.device_sync(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        T.run(args.topk, mask)
    blp.device_sync(dev)
    t_local = time.perf_counter() - t_start
    dist.barrier()
    t_max = dist.max(t_local) / args.steps
    kms, kn = T.stats(0)
    kern_s = kms / 1e3 / max(kn, 1)
    first = [m for m, bit in (("common_neighbors", 1), ("jaccard", 2), ("adamic_adar", 4)) if mask & bit][0]
    ncand = T.fetch(first)[2]
    pairs = int(ncand.sum())
    h2_sum, push_sum = T.stats(3)[1], T.stats(4)[1]
    hash_src, direct_src = T.stats(1)[1], T.stats(2)[1]
    pushed, dense_adds = T.stats(6)[1], T.stats(7)[1]
    add_bytes = T.stats(8)[1]
    byts = topk_alg_bytes(G, src, h2_sum, pushed, args.topk, bin(mask).count("1"), dense_adds, add_bytes)
    byts_h2 = topk_alg_bytes(G, src, h2_sum, push_sum, args.topk, bin(mask).count("1"))
    out = {
        "metric": METRIC, "value": dist.sum(pairs) / t_max, "unit": "pairs/s", "n_gpus": dist.world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * t_max, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int32", "data": "synthetic",
        "config": {"workload": "config3: config-2 graph (%d unique edges); %d users/GPU, every exact hop-3 business "
                               "scored (%s), top-%d per method" % (G.nnz // 2, len(src), "+".join(
                                   n for n, bit in (("CN", 1), ("Jaccard", 2), ("Adamic-Adar", 4)) if mask & bit),
                                   args.topk),
                   "pairs_per_gpu": pairs, "global_batch": int(dist.sum(pairs)),
                   "parallelism": "replicas x%d (graph replicated, users split, no collective)" % dist.world},
        "roofline": {"bound": "hbm", "achieved": byts / kern_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": byts / kern_s / 1e9 / HBM_PEAK_GBS, "kernel": "k_topk", "kernel_ms": 1e3 * kern_s,
                     "alg_bytes_per_launch": byts,
                     "priced_on": "the pushes the kernel performs (%d) plus %d dense hot-target adds of %d B; "
                                  "the whole H2 volume (%d pushes) would give frac %.3f" %
                                  (pushed, dense_adds, add_bytes, push_sum, byts_h2 / kern_s / 1e9 / HBM_PEAK_GBS),
                     **pmc_fields("k_topk", "r*_topk_*.json", kern_s),
                     "limiter": pmc_limiter("k_topk", "r*_topk_*_pmc.txt")},
        "work": {"sum_h2": h2_sum, "sum_push": push_sum, "pushed": pushed, "dense_target_adds": dense_adds,
                 "aa_hash_sources": hash_src, "aa_direct_sources": direct_src},
        # off the clock, once per graph (independent of the sources): the synthetic graph and the
        # top-k handle (permuted rows, wedge rows, the hot targets' dense counts)
        "setup_s": {"graph_build": round(graph_s, 3), "topk_create": round(create_s, 3),
                    # once per graph, off the clock; its cost in steps of this line
                    "topk_create_in_steps": round(create_s / t_max, 1)},
    }
    if dist.rank == 0 and not args.no_parity and mask == blp.JACCARD | blp.ADAMIC:
        cols_j, sc_j, _ = T.fetch("jaccard")
        cols_a, sc_a, _ = T.fetch("adamic_adar")
        out["parity"] = topk_parity(G, src, args.topk, {"jaccard": (cols_j, sc_j), "adamic_adar": (cols_a, sc_a),
                                                        "ncand": ncand}, n_users=args.topk_parity_users)
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = topk_cpu_baseline(G, src, args.topk, args.cpu_seconds)
    if dist.rank == 0:
        print(json.dumps(out), flush=True)


XGMI_LINK_GBS = 153.0  # per-direction xGMI link rate (MI355X_MICROARCH.md), 7 links per GPU


def run_sharded(args):
    """Config 5 (BASELINE.json configs[4]): row-block sharded ingest. Rank r generates only the
    edges of its user block, ONE RCCL all-gather over xGMI gives every rank the full edge list
    in HBM, libblp builds the CSR on the device, and each rank scores its own users' pairs
    (rank-local, no further collective). The exchange is timed apart from the scoring step;
    value = candidate pairs scored per second over all ranks (weak scaling)."""
    from blp import dist as bd

    # the process group is formed even for one rank, so the exchange below is RCCL's own
    # all_gather_into_tensor at every world size (dist.py, allgather_edges)
    capi = args.exchange == "capi"
    # capi: the exchange through libblp's own RCCL communicator (blp_multi_*, multi.hip); the
    # torch group is then gloo only (barrier, max / sum of the timings)
    d = Dist(exchange=not capi, collective_at_world1=not args.no_collective_at_world1 and not capi)
    dev = _device(d)
    blp.lib()
    U, B, D = synth.CONFIGS[args.config]
    blocks = bd.user_blocks(U, d.world)
    lo, hi = int(blocks[d.rank]), int(blocks[d.rank + 1])
    t0 = time.time()
    u, b = bd.block_review_edges(U, B, D, lo, hi, seed=0)
    gen_s = time.time() - t0
    log("rank %d: users [%d, %d), %d draws generated in %.1fs" % (d.rank, lo, hi, len(u), gen_s))
    import torch

    torch.cuda.set_device(dev)
    d.barrier()
    torch.cuda.synchronize()
    if capi:
        from blp.multi import Multi

        with bd.stdout_to_stderr():  # RCCL's banner goes to stdout
            mc = Multi(d.broadcast_bytes(Multi.unique_id() if d.rank == 0 else None), d.world, d.rank, dev)
        d.barrier()
        t0 = time.perf_counter()
        # ONE call: counts + padded partials all-gathered over RCCL, padding dropped, CSR built in HBM
        c = mc.gather_csr(u.astype(np.int32), b.astype(np.int32), U + B)
        exch_local = time.perf_counter() - t0
        d.barrier()
        exch_s = d.max(exch_local)
        recv_bytes = mc.bytes_in  # padded partials of the other ranks
        gathered_bytes = recv_bytes + 8 * len(u)
        del u, b
        t0 = time.perf_counter()
        G = blp.DeviceGraph.from_csr_handle(c, U + B, U, device=dev)
        build_s = time.perf_counter() - t0
        mc.close()
    else:
        t0 = time.perf_counter()
        a_all, b_all, counts = bd.allgather_edges(d, u, b)
        torch.cuda.synchronize()
        exch_local = time.perf_counter() - t0
        d.barrier()
        exch_s = d.max(exch_local)
        recv_bytes = 8 * (sum(counts) - counts[d.rank])
        gathered_bytes = 8 * max(counts) * d.world  # the all-gather's output tensor (padded partials)
        del u, b
        if not a_all.is_cuda:  # gloo exchange (rehearsal without RCCL): the partials arrive on the host
            a_all, b_all = a_all.to("cuda:%d" % dev), b_all.to("cuda:%d" % dev)
        t0 = time.perf_counter()
        # the CSR is built in HBM from the gathered endpoints and stays there (no host round trip)
        G = blp.DeviceGraph.from_device_edges(a_all.data_ptr(), b_all.data_ptr(), len(a_all), U + B, U, device=dev)
        build_s = time.perf_counter() - t0
        del a_all, b_all
    torch.cuda.empty_cache()
    log("rank %d: graph %d nodes, %d unique edges; exchange %.2fs (%.2f GB in), device CSR build %.1fs %s" %
        (d.rank, G.n, G.nnz // 2, exch_local, recv_bytes / 1e9, build_s, G.build_times))
    # scoring ownership: contiguous user blocks balanced by WORK (SURVEY.md §8(e) step 1:
    # sum_{b in N(u)} d_b per user, from the full CSR every rank now holds -- identical on all ranks)
    end_u = int(G.row_ptr[U])  # user rows come first: only their entries are summed
    csum = np.zeros(end_u + 1, np.int64)
    np.cumsum(G.hop1_size[G.col_idx[:end_u]], out=csum[1:])
    work = (csum[G.row_ptr[1:U + 1]] - csum[G.row_ptr[:U]]).astype(np.float64)
    del csum
    sblocks = bd.user_blocks(U, d.world, work)
    lo, hi = int(sblocks[d.rank]), int(sblocks[d.rank + 1])
    rng = np.random.default_rng(d.rank)
    mine = np.arange(lo, hi)
    mine = mine[G.hop1_size[lo:hi] > 0]
    src = np.sort(rng.choice(mine, size=min(args.users, len(mine)), replace=False)).astype(np.int32)
    ex_x, ex_y = synth.uniform_examples(G, src, rate=args.rate, seed=d.rank)
    passes = [("user", G.batch(ex_x, ex_y), args.user_mask)] if args.sides != "business" else []
    if args.sides != "user":
        passes.append(("business", G.batch(ex_y, ex_x), 7 if getattr(args, "fix_adamic", False) else 3))
    for name, bt, _ in passes:
        log("plan %s: %s" % (name, bt.plan()))
    # each pass on its own stream (they overlap where the grids leave room); --cosched-passes:
    # both through blp_batches_score (holding each chunk-parallel grid to a CU share was measured
    # slower: 1951 / 864 / 903 ms at proportional / 176 / 128 user CUs against 743 ms,
    # profiles/r03_bench_sharded_c5_cosched*.json, and was removed)
    def step():
        if len(passes) > 1 and args.cosched_passes:
            G.score_batches([(bt, mask) for _, bt, mask in passes])
        else:
            for _, bt, mask in passes:
                bt.score(mask)

    for _ in range(args.warmup):
        step()
    blp.device_sync(dev)
    for _, bt, _ in passes:
        bt.stats_reset()
    d.barrier()
    blp.device_sync(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    blp.device_sync(dev)
    t_local = time.perf_counter() - t_start
    if os.environ.get("BLP_PROF_READ"):  # experiment library built with -DBLP_PROF: phase clocks
        import ctypes

        buf = (ctypes.c_ulonglong * 16)()
        blp.lib().blp_prof_read(buf)
        v = np.array(buf[:9], np.float64)
        log("prof %s" % {i: "%.1f%%" % (100 * x / max(v.sum(), 1)) for i, x in enumerate(v)})
    d.barrier()
    t_max = d.max(t_local)
    pairs_total = d.sum(len(ex_x))
    name0, bt0, mask0 = passes[0]
    ms, n = bt0.stats(0)
    sec = ms / 1e3 / max(n, 1)
    cn0 = bt0.fetch(mask0)["cn"]
    byts = alg_bytes(G, *((ex_x, ex_y) if name0 == "user" else (ex_y, ex_x)), mask0, cn0)
    # ring all-gather: each rank receives (G-1)/G of the data; bound by one link per direction
    xgmi_bound_s = recv_bytes / (XGMI_LINK_GBS * 1e9) if d.world > 1 else 0.0
    out = {
        "metric": METRIC, "value": pairs_total * args.steps / t_max, "unit": "pairs/s", "n_gpus": d.world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * t_max / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32", "data": "synthetic",
        "config": {"workload": "config5-style row-block sharded: %d users x %d businesses, %d draws (%d unique edges); "
                               "%d users/GPU from the rank's own block, businesses outside N(u) kept at %g; step = %s"
                               % (U, B, D, G.nnz // 2, len(src), args.rate,
                                  "user side CN+J+AA + business side CN+J" if args.sides == "both" else
                                  args.sides + " side only"),
                   "pairs_per_gpu": int(len(ex_x)), "global_batch": int(pairs_total),
                   "parallelism": "row-block sharded ingest x%d + RCCL all-gather (%s), rank-local scoring"
                                  % (d.world, d.backend or "single rank")},
        "exchange": {"backend": "rccl (libblp blp_multi_gather_csr; seconds include the device CSR build)" if capi
                     else d.backend,
                     "collective": "ncclAllGather" if capi else
                     "all_gather_into_tensor" if d.td is not None else None,
                     "gathered_bytes_per_rank": int(gathered_bytes),
                     "seconds": exch_s, "bytes_in_per_rank": int(recv_bytes),
                     "GBps_in_per_rank": recv_bytes / exch_s / 1e9 if exch_s > 0 and recv_bytes else None,
                     "xgmi_one_link_bound_s": xgmi_bound_s, "device_csr_build_s": build_s, "generate_s": gen_s,
                     "device_csr_phases_s": G.build_times,
                     "scoring_blocks": "work-balanced (sum of d_b over N(u)); block work max/mean %.3f" %
                                       (max(work[sblocks[r]:sblocks[r + 1]].sum() for r in range(d.world)) /
                                        (work.sum() / d.world))},
        "roofline": {"bound": "hbm", "achieved": byts / sec / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": byts / sec / 1e9 / HBM_PEAK_GBS, "kernel": "%s-side scorer (%s)" % (name0, C5_KERNEL),
                     "kernel_ms": 1e3 * sec, "alg_bytes_per_launch": byts, "plan": bt0.plan()},
    }
    out["roofline"].update(pmc_fields(C5_KERNEL, "r*_c5_*.json", sec))
    out["roofline"]["limiter"] = pmc_limiter(C5_KERNEL, "r*_c5_*_pmc.txt")
    if not args.no_parity:
        out["parity"] = sharded_parity(args, d, U, B, D, passes, ex_x, ex_y)
    if d.rank == 0:
        print(json.dumps(out), flush=True)
    d.close()


C5_KERNEL = "k_score_split"


def sharded_parity(args, d, U, B, D, passes, ex_x, ex_y):
    """Config 5 at its own scale, not timed: on every rank, all pairs of `--parity-sources`
    sampled user sources (user pass, CN + Jaccard + Adamic-Adar) and as many sampled business
    sources (business pass, CN + Jaccard) are gathered to rank 0, which regenerates the union
    of every rank's edge partial independently of the exchange (block_review_edges, the same
    seeds), builds the C oracle's graph over the full 1B edges (oracle.c og_create: SNAP
    LoadEdgeList semantics) and scores them with the reference algorithm
    (similarity.py:20-106 / :108-126). Bit-exact: CN, the Jaccard quotient and the correctly
    rounded Adamic-Adar sum."""
    import coracle

    from blp import dist as bd

    rng = np.random.default_rng(100 + d.rank)
    mine = {}
    for name, bt, mask in passes:
        xs, ys = (ex_x, ex_y) if name == "user" else (ex_y, ex_x)
        srcs = np.unique(xs)
        pick = rng.choice(srcs, size=min(args.parity_sources, len(srcs)), replace=False)
        sel = np.flatnonzero(np.isin(xs, pick))
        res = bt.fetch(mask)
        mine[name] = {"x": xs[sel], "y": ys[sel], "mask": mask,
                      **{k: v[sel] for k, v in res.items() if v is not None}}
    allr = [mine]
    if d.world > 1:
        allr = [None] * d.world if d.rank == 0 else None
        d.td.gather_object(mine, allr, dst=0, group=d.cpu_group)
    if d.rank != 0:
        return None
    t0 = time.time()
    blocks = bd.user_blocks(U, d.world)
    parts = [bd.block_review_edges(U, B, D, int(blocks[r]), int(blocks[r + 1]), seed=0) for r in range(d.world)]
    a = np.concatenate([p[0] for p in parts]).astype(np.int32)
    b = np.concatenate([p[1] for p in parts]).astype(np.int32)
    del parts
    og = coracle.OracleGraph(U + B, a, b)
    del a, b
    build_s = time.time() - t0
    nt = max(1, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0)))
    out = {"ranks_checked": len(allr), "oracle_graph_build_s": round(build_s, 1), "ok": True}
    t0 = time.time()
    for name in mine:
        n_pairs = n_src = 0
        same = {}
        for r in allr:
            m = r[name]
            cn, jac, aa, _ = og.score_pairs(m["x"], m["y"], m["mask"], nthreads=nt)
            for k, want in (("cn", cn), ("jaccard", jac), ("adamic", aa)):
                if k in m:
                    same[k] = same.get(k, True) and bool(np.array_equal(m[k], want))
            n_pairs += len(m["x"])
            n_src += len(np.unique(m["x"]))
        out[name] = {"sources": n_src, "pairs": n_pairs, **{k + "_exact": v for k, v in same.items()}}
        out["ok"] &= all(same.values()) and n_pairs > 0
    out["oracle_score_s"] = round(time.time() - t0, 1)
    return out


def run_e2e(args):
    """Config 1 (Yelp-sized synthetic, BASELINE.json configs[0]) and config 2 end to end: the
    drop-in similarity.main (similarity.py:11-18) from graph.txt + examples.json to the six
    JSON files (parse + id lookup + device step + dict assembly + json.dumps, util.py:18-21),
    one run, phases timed. Beside it: the device-only step on the same pairs, the C oracle's
    reference-algorithm scoring of every pair (1 thread and all host threads), and every
    score file checked against the oracle (CN / Jaccard / Adamic-Adar bit-exact)."""
    import importlib
    import shutil
    import tempfile

    import pandas as pd

    import coracle

    sim = importlib.import_module("similarity")
    util = importlib.import_module("util")
    dist = Dist()
    dev = _device(dist)
    blp.lib()
    U, B, D = synth.CONFIGS[args.config]
    work = tempfile.mkdtemp(prefix="blp_e2e_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        t0 = time.time()
        a, b = synth.review_edges(U, B, D, seed=0)
        gpath = os.path.join(work, "graph.txt")
        pd.DataFrame({"u": a, "b": b}).to_csv(gpath, sep="\t", header=False, index=False)
        G = blp.DeviceGraph(a, b, device=dev)
        del a, b
        ex_x, ex_y, ex_l = synth.make_examples(G, U, B, D, n_users=args.users, rate=args.rate, seed=0)
        uid, bid = G.node_ids[ex_x].tolist(), G.node_ids[ex_y].tolist()
        examples = {}
        for u, v, l in zip(uid, bid, ex_l.tolist()):
            examples.setdefault(str(u), {})[str(v)] = int(l)
        epath = os.path.join(work, "examples.json")
        util.write_json(examples, epath)
        n_ex_users = len(examples)
        del examples, uid, bid  # the harness's own 7.5M-entry dict and id lists: not alive while main runs
        log("e2e inputs: %d edges in graph.txt (%.0f MB), %d pairs of %d users, in %.1fs" %
            (D, os.path.getsize(gpath) / 2**20, len(ex_x), n_ex_users, time.time() - t0))
        # the device-only step on the same pairs (both passes, concurrent), for reference
        ub, bb = G.batch(ex_x, ex_y), G.batch(ex_y, ex_x)
        step = [(ub, 7), (bb, 3)]
        G.score_batches(step)
        blp.device_sync(dev)
        t = time.perf_counter()
        for _ in range(5):
            G.score_batches(step)
        blp.device_sync(dev)
        dev_ms = (time.perf_counter() - t) / 5 * 1e3
        og = coracle.OracleGraph(G.n, *_dense_edges(G))
        ub.close()
        bb.close()
        G.close()
        del G
        # timed: similarity.main end to end
        uf = [os.path.join(work, f) for f in ("u_cn.json", "u_jaccard.json", "u_adamic.json")]
        bf = [os.path.join(work, f) for f in ("b_cn.json", "b_jaccard.json", "b_adamic.json")]
        methods = ["common_neighbors", "jaccard", "adamic_adar"]
        ph = {}
        import gc

        gc.collect()  # the harness's garbage is collected before the timed call, not during it
        t = time.perf_counter()
        sim.main(epath, gpath, methods, uf, methods, bf, timings=ph)
        t_back = time.perf_counter()
        e2e = t_back - t
        ph["call_overhead"] = ph.pop("_clock_entry") - t
        ph["return_overhead"] = t_back - ph.pop("_clock_exit")
        n = ph["pairs"]
        # the C oracle (reference algorithm) on every pair of both sides
        cpu = {}
        nt = max(1, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0)))
        for threads in (1, nt):
            t = time.perf_counter()
            ucn, ujac, uaa, _ = og.score_pairs(ex_x, ex_y, 7, nthreads=threads)
            bcn, bjac, _, _ = og.score_pairs(ex_y, ex_x, 3, nthreads=threads)
            cpu["%dt" % threads] = {"seconds": time.perf_counter() - t, "pairs_per_s": n / (time.perf_counter() - t)}
        # every score file against the oracle, in the files' own order (= examples order)
        par = {}
        for f, want in ((uf[0], ucn), (uf[1], ujac), (uf[2], uaa), (bf[0], bcn), (bf[1], bjac)):
            got = [v for u in util.load_json(f).values() for v in u.values()]
            w = want.tolist()
            if f.endswith("_adamic.json"):
                w = [0 if x == 0.0 else x for x in w]
            par[os.path.basename(f)] = bool(got == w and all(type(g) is type(x) for g, x in zip(got, w)))
        out = {"metric": "similarity.main end to end (graph.txt -> 6 JSON files), pairs/s", "value": n / e2e,
               "unit": "pairs/s", "n_gpus": 1, "higher_is_better": True, "data": "synthetic",
               "config": {"workload": "%s: synthetic %d users x %d businesses, %d draws; %d example users, hop-3 "
                                      "candidates kept at %g; u_methods = b_methods = CN, Jaccard, AA (the reference's "
                                      "__main__ call, similarity.py:129-135)" % (args.config, U, B, D, n_ex_users,
                                                                                  args.rate), "pairs": n},
               "e2e_s": e2e, "phases_s": {k: v for k, v in ph.items() if k not in ("pairs", "graph_detail")},
               "graph_phase_detail_s": ph.get("graph_detail"),
               "device_step_ms": dev_ms, "device_pairs_per_s": n / (dev_ms / 1e3),
               "cpu_reference_algorithm": {"kind": "port", "what": "C oracle scoring of every pair of both sides "
                                           "(graph already built; no file I/O)", **cpu},
               "files_equal_oracle": par, "ok": all(par.values())}
        if dist.rank == 0:
            print(json.dumps(out), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


def exchange_check(dist, dev, a, b, U, B, G, timeout_s=120.0):
    """One run of the multi-GPU exchange (blp_multi_gather_csr, csrc/multi.hip)
    after the timed step, over this job's ranks: rank r sends the edges of its user block
    (user_blocks by count) of the config-2 graph every replica generated; ONE RCCL all-gather
    moves the counts, then the padded partials; the padding is dropped on the device and the
    union's CSR is built in HBM. The union is the whole graph, so its CSR must equal the
    replica's (checked). Reported beside the headline, never part of it. A watchdog bounds the
    collective: if it has not returned in timeout_s, rank 0 still prints its line (exchange
    marked as timed out) and every rank exits with status 3 (main)."""
    import threading

    from blp import dist as bd
    from blp.multi import Multi

    lo, hi = (int(v) for v in bd.user_blocks(U, dist.world)[dist.rank:dist.rank + 2])
    sel = (a >= lo) & (a < hi)
    pa, pb = a[sel].astype(np.int32), b[sel].astype(np.int32)
    box = {}

    def run():
        try:
            with bd.stdout_to_stderr():  # RCCL's banner goes to stdout
                uid = dist.broadcast_bytes(Multi.unique_id() if dist.rank == 0 else None)
                mc = Multi(uid, dist.world, dist.rank, dev)
            dist.barrier()
            t0 = time.perf_counter()
            c = mc.gather_csr(pa, pb, U + B)
            sec = time.perf_counter() - t0
            rp, ci = Multi.fetch_csr(c)
            t_max = mc.allreduce(sec, "max")
            box["res"] = (mc.bytes_in, sec, t_max, rp, ci)
            mc.close()
        except Exception as e:  # reported in the line, the headline stands
            box["err"] = "%s: %s" % (type(e).__name__, e)

    th = threading.Thread(target=run, daemon=True)
    th.start()
    th.join(timeout_s)
    if th.is_alive():
        return {"error": "exchange did not return within %.0f s" % timeout_s, "timed_out": True}
    if "err" in box:
        return {"error": box["err"]}
    bytes_in, sec, t_max, rp, ci = box["res"]
    dense = G.n == U + B and np.array_equal(G.node_ids, np.arange(U + B))
    same = bool(dense and np.array_equal(rp, G.row_ptr) and np.array_equal(ci, G.col_idx)) if dense else \
        int(len(ci)) == int(G.nnz)
    return {"backend": "rccl (libblp blp_multi_gather_csr)", "collective": "ncclAllGather (counts, then padded partials)",
            "edges_sent": int(sel.sum()), "bytes_in_per_rank": int(bytes_in),
            "seconds_max_over_ranks": t_max, "seconds_include": "count exchange + all-gather + device CSR build",
            "GBps_in_per_rank": bytes_in / t_max / 1e9 if t_max > 0 and bytes_in else None,
            "xgmi_one_link_bound_s": bytes_in / (XGMI_LINK_GBS * 1e9),
            "union_csr_equals_replica": same}


def _free_port():
    import socket

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def relaunch_if_needed(args):
    """`python bench.py --gpus N` with N > 1 and no torchrun environment: start N ranks under
    torch.distributed.run as a CHILD process (nothing here has touched the GPU yet) and exit
    with its status. Under torchrun (the driver's own launch), WORLD_SIZE must equal --gpus."""
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        if args.gpus <= 1:
            return
        import subprocess

        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               os.path.abspath(__file__)] + sys.argv[1:]
        log("launching %d ranks: %s" % (args.gpus, " ".join(cmd)))
        sys.exit(subprocess.call(cmd))
    if int(world) != args.gpus:
        sys.exit("bench.py: WORLD_SIZE=%s but --gpus %d" % (world, args.gpus))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(synth.CONFIGS))
    ap.add_argument("--users", type=int, default=10_000)
    ap.add_argument("--rate", type=float, default=0.01)
    ap.add_argument("--sides", default="both", choices=["both", "user", "business"])
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--user-mask", type=int, default=7, help="methods of the user pass (1 CN, 2 J, 4 AA)")
    ap.add_argument("--business-first", action="store_true", help="enqueue the business pass before the user pass")
    ap.add_argument("--fix-adamic", action="store_true",
                    help="business pass with Adamic-Adar too (similarity.business(..., fix_adamic=True); the "
                         "reference's own business pass never computes it, similarity.py:102)")
    ap.add_argument("--mode", default="similarity", choices=["similarity", "topk", "svd", "sharded", "e2e"],
                    help="similarity: config 2 (default); topk: config 3 full-candidate Jaccard + Adamic-Adar "
                         "top-k; svd: config 4 rank-64 truncated-SVD scorer; sharded: config 5 row-block "
                         "sharded ingest + RCCL all-gather, then rank-local scoring (--config c5); e2e: "
                         "similarity.main from graph.txt to the 6 files (--config yelp = config 1, or c2)")
    ap.add_argument("--cosched-passes", action="store_true", help="--mode sharded: both passes through blp_batches_score")
    ap.add_argument("--parity-sources", type=int, default=50,
                    help="--mode sharded: sampled sources per side and rank checked against the C oracle")
    ap.add_argument("--exchange", choices=["torch", "capi"], default="torch",
                    help="sharded mode: config 5's exchange through torch.distributed (RCCL) or through "
                         "libblp's own RCCL communicator (blp_multi_gather_csr)")
    ap.add_argument("--no-collective-at-world1", action="store_true",
                    help="--mode sharded: at one rank, skip the process group (no RCCL call; the local partial)")
    ap.add_argument("--no-exchange", action="store_true",
                    help="similarity mode: skip the post-step exchange run (blp_multi_gather_csr over the ranks)")
    ap.add_argument("--topk", type=int, default=20)
    ap.add_argument("--svd-parity-users", type=int, default=1000,
                    help="--mode svd: users whose top-k is checked against numpy (0: every user)")
    ap.add_argument("--topk-parity-users", type=int, default=200,
                    help="--mode topk: users whose lists are checked against the C oracle (0: every user)")
    ap.add_argument("--topk-mask", type=int, default=6, help="methods of --mode topk (default Jaccard + AA)")
    args = ap.parse_args()
    relaunch_if_needed(args)
    if args.mode == "svd":
        return run_svd(args)
    if args.mode == "topk":
        return run_topk(args)
    if args.mode == "sharded":
        return run_sharded(args)
    if args.mode == "e2e":
        return run_e2e(args)

    dist = Dist()
    dev = _device(dist)
    blp.lib()
    U, B, D = synth.CONFIGS[args.config]
    t0 = time.time()
    a, b = synth.review_edges(U, B, D, seed=0)
    t_gen = time.time() - t0
    t0 = time.time()
    G = blp.DeviceGraph(a, b, device=dev)  # CSR, weights, coded ids, dense-row index, wedge rows
    t_graph = time.time() - t0
    log("graph: %d nodes, %d unique edges, generated in %.1fs, built in %.1fs" % (G.n, G.nnz // 2, t_gen, t_graph))
    t0 = time.time()
    ex_x, ex_y, ex_l = synth.make_examples(G, U, B, D, n_users=args.users, rate=args.rate, seed=dist.rank)
    t_ex = time.time() - t0
    hop3_ms, hop3_n = G.stats(blp._lib.K_HOP3)  # the candidate kernel (k_hop3_wedge), HIP events
    log("examples: %d pairs for %d users (%d positives) in %.1fs (hop-3 kernel %.2f ms)" %
        (len(ex_x), len(np.unique(ex_x)), int(ex_l.sum()), t_ex, hop3_ms / max(hop3_n, 1)))

    passes = []
    # the kernels' code objects and the pooled streams, as similarity.main's prewarm thread loads
    # them: a one-off cost of the process, not of a pair list
    if not os.environ.get("BLP_BENCH_NO_PREWARM"):  # (A/B knob)
        blp.prewarm(dev, 3)
    t0 = time.time()
    b_mask = 7 if getattr(args, "fix_adamic", False) else 3
    if args.sides == "both":  # one upload of the pairs for both passes (blp_batch_create_pair)
        ub_, bb_ = G.batch_pair(ex_x, ex_y)
        passes += [("user", ub_, args.user_mask), ("business", bb_, b_mask)]
    elif args.sides == "user":
        passes.append(("user", G.batch(ex_x, ex_y), args.user_mask))
    else:
        passes.append(("business", G.batch(ex_y, ex_x), b_mask))
    t_batch = time.time() - t0
    if args.business_first:  # enqueue order of the two concurrent passes
        passes.reverse()
    for name, bt, _ in passes:
        log("plan %s: %s" % (name, bt.plan()))

    step = [(bt, mask) for _, bt, mask in passes]  # one concurrent step (blp_batches_score)
    for _ in range(args.warmup):
        G.score_batches(step)
    blp.device_sync(dev)
    for _, bt, _ in passes:
        bt.stats_reset()

    dist.barrier()
    blp.device_sync(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        G.score_batches(step)
    blp.device_sync(dev)
    t_local = time.perf_counter() - t_start
    dist.barrier()
    t_max = dist.max(t_local)
    pairs_total = dist.sum(len(ex_x))

    # per-kernel device times (HIP events on the graph stream, same launches as timed)
    ktimes = {}
    for name, bt, _ in passes:
        ms, n = bt.stats(0)
        gms, gn = bt.stats(1)
        ktimes[name] = {"score_ms": ms / max(n, 1), "group_ms": gms / max(gn, 1)}
    res = {name: bt.fetch(mask) for name, bt, mask in passes}
    # after the timed step: config 5's exchange (blp_multi_gather_csr: counts + padded partials in
    # ONE RCCL all-gather, CSR built in HBM) over this job's ranks, on the config-2 edge partials
    exchange = None if args.no_exchange else exchange_check(dist, dev, a, b, U, B, G)
    del a, b

    out = {
        "metric": METRIC,
        "value": pairs_total * args.steps / t_max,
        "unit": "pairs/s",
        "n_gpus": dist.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * t_max / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {
            "workload": "config2: synthetic %dK users x %dK businesses, %dM draws (%d unique edges); %d example "
                        "users/GPU, exact hop-3 candidates kept at %g (+held-out positives); step = similarity.main "
                        "device work: %s" % (U // 1000, B // 1000, D // 10**6, G.nnz // 2, len(np.unique(ex_x)),
                                             args.rate, "user side CN+Jaccard+AA fused + business side CN+Jaccard" +
                                             (" + AA (fix_adamic)" if args.fix_adamic else "")
                                             if args.sides == "both" else args.sides + " side"),
            "pairs_per_gpu": int(len(ex_x)),
            "global_batch": int(pairs_total),
            "parallelism": "replicas x%d (graph replicated, users split, no collective)" % dist.world,
        },
        "kernels_ms": ktimes,
        # a NEW pair list's rate: planning both batches (blp_batch_create: upload + device planning
        # pass) plus one step, as similarity.main pays it once per call (never `value`)
        "including_batch_create": {"batch_create_s": round(t_batch, 4),
                                   "seconds": t_batch + t_max / args.steps,
                                   "pairs_per_s": len(ex_x) / (t_batch + t_max / args.steps)},
        "exchange": exchange,
        # outside the timed step (once per graph / per example set), reported for completeness
        "setup_s": {"edge_generation": round(t_gen, 3), "graph_build": round(t_graph, 3),
                    "examples_hop3": round(t_ex, 3), "hop3_kernel_ms": round(hop3_ms / max(hop3_n, 1), 3),
                    "batch_create": round(t_batch, 3)},
        "work": {name: {"build_elems": _build_elems(G, xs_), "scan_elems": int(G.hop1_size[ys_].astype(np.int64).sum()),
                        "hits": int(res[name]["cn"].astype(np.int64).sum()), "sources": int(len(np.unique(xs_)))}
                 for name, xs_, ys_ in [("user", ex_x, ex_y), ("business", ex_y, ex_x)] if name in res},
    }
    # roofline of the dominant kernel: the user-side scorer (falls back to the first pass); and
    # (both sides) a second entry for the business pass -- its scorer and its per-step grouping,
    # the chain that runs beside the user scorer on the remaining CUs
    def roofline_of(name, bt, mask):
        xs, ys = (ex_x, ex_y) if name == "user" else (ex_y, ex_x)
        kname = bt.kernel(mask)
        byts = (wset_alg_bytes(G, xs, ys, mask) if kname.startswith("k_score_wset")
                else alg_bytes(G, xs, ys, mask, res[name]["cn"]))
        sec = ktimes[name]["score_ms"] / 1e3
        r = {"bound": "hbm", "achieved": byts / sec / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
             # basis: the kernel's in-step average (HIP events around every timed launch, on the
             # batch's own stream); frac_profile below uses the committed profile's average instead
             "frac": byts / sec / 1e9 / HBM_PEAK_GBS, "frac_basis": "in-step HIP-event average (%.4f ms)" % (1e3 * sec),
             # the counters' HBM-side bytes over the same kernel time: what DRAM actually moved
             **pmc_fields(kname, "r*_v*_bench.json", sec),
             "kernel": "%s (%s side)" % (kname, name), "alg_bytes_per_launch": byts,
             # what the counters name as the bound ("What bounds the user scorer"),
             # from the newest committed counter summary of this kernel
             "limiter": pmc_limiter(kname, "r*_v*_bench_pmc.txt")}
        if r.get("profile_kernel_ms"):
            r["frac_profile"] = byts / (r["profile_kernel_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS
        if alone.get(name):
            r["kernel_alone_ms"] = alone[name]
            r["frac_alone"] = byts / (alone[name] / 1e3) / 1e9 / HBM_PEAK_GBS
        return r

    # each pass by itself, after the timed loop (5 launches each; never `value`): in the step the
    # user scorer starts while the business launch still holds part of the chip, so its in-step
    # average (the `frac` basis) includes that sharing; kernel_alone_ms / frac_alone exclude it
    alone = {}
    for name, bt, mask in passes:
        bt.stats_reset()
        for _ in range(5):
            bt.score(mask)
        blp.device_sync(dev)
        ms, n = bt.stats(0)
        alone[name] = ms / max(n, 1)

    name0, bt0, mask0 = sorted(passes, key=lambda p: p[0] != "user")[0]
    out["roofline"] = roofline_of(name0, bt0, mask0)
    for name, bt, mask in passes:
        if name == "business" and name0 == "user":
            rb = roofline_of(name, bt, mask)
            # the business grouping per step (bucket sort into item order): read (x, y), gather
            # rp[y] and rp[y + 1], write the grouped metadata (caller index 4 B, row start 8 B,
            # row length 4 B) -- 40 B per pair
            gb = 40 * len(ex_x)
            gsec = ktimes[name]["group_ms"] / 1e3
            rb["grouping"] = ({"alg_bytes_per_step": gb, "ms": 1e3 * gsec, "achieved": gb / gsec / 1e9,
                               "frac": gb / gsec / 1e9 / HBM_PEAK_GBS} if gsec > 0 else
                              {"ms": 0.0, "note": "none: the wedge-set scorer reads the pairs in caller order"})
            rb["chain_ms"] = 1e3 * (gsec + ktimes[name]["score_ms"] / 1e3)
            if rb.get("frac_alone"):
                # the business launch is enqueued beside the user pass and, once the user scorer's
                # persistent grid holds the chip, waits for its workgroups to retire: its in-step
                # window is mostly queueing (it fills the user scorer's tail). Its own rate is the
                # launch alone, after the timed loop; the in-step figure is kept beside it
                rb["frac_in_step"], rb["frac_basis_in_step"] = rb["frac"], rb["frac_basis"]
                rb["frac"] = rb["frac_alone"]
                rb["frac_basis"] = ("the launch alone after the timed loop (%.4f ms, 5 launches); in the step "
                                    "it waits behind the user scorer and fills its tail" % rb["kernel_alone_ms"])
            out["roofline_business"] = rb
    if dist.rank == 0 and args.sides == "both" and not (args.no_parity and args.no_cpu_baseline):
        import coracle

        og = coracle.OracleGraph(G.n, *_dense_edges(G))
        ora, multi = oracle_full(og, ex_x, ex_y, 7 if args.fix_adamic else 3)
        if not args.no_parity:
            out["parity"] = full_parity(ex_l, res, ora)
        if dist.world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(og, ex_x, ex_y, args.cpu_seconds)
            out["cpu_baseline"]["multicore"] = multi
    if dist.rank == 0:
        print(json.dumps(out), flush=True)
    if exchange and exchange.get("timed_out"):
        # a collective still blocked in RCCL: do not wait for it, and do not report success -- the
        # line above stands, but a hung exchange on an N-GPU run must read as a failed job
        log("exchange watchdog fired: exiting with status 3")
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(3)


if __name__ == "__main__":
    main()
