"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the reference's hot path, used as the *checker* for the
HIP engine. Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it; the product (``bipartite-link-prediction_amd/``)
never does, and fails loudly when its HIP library is missing.

Pinning: every function here is checked against the golden fixtures in
``tests/golden/`` (outputs of the reference's own code, see
``tests/golden/make_golden.py``) by ``tests/test_oracle.py``. The SNAP calls
(``LoadEdgeList``, ``GetNodesAtHop``, ``GetDeg``) are restated from SNAP's documented
semantics; SNAP itself is absent (``.MISSING_LARGE_BLOBS:1-3``), so that boundary is
"parity unpinned" beyond the fixtures.

Pure-Python loops: small cases only. ``oracle/oracle.c`` is the C restatement of the
same pair scorers for larger cases and the CPU baseline.
"""
import math
from collections import defaultdict, deque

import numpy as np

BUGGY_B_ADAMIC = "Beginning adamic adar coefficient computation"  # similarity.py:102


# --------------------------------------------------------------------------- graph (SNAP)
def load_edge_list(path, c0=0, c1=1):
    """snap.LoadEdgeList(snap.PUNGraph, path, 0, 1) as used at similarity.py:16.

    Undirected simple graph; '#' lines skipped; duplicate edges dropped; a self-loop
    is stored once in the node's own neighbour set (TUNGraph::AddEdge), so GetDeg
    counts it once."""
    adj = {}
    with open(path) as f:
        for line in f:
            if line.startswith("#"):
                continue
            cols = line.split()
            if len(cols) <= max(c0, c1):
                continue
            a, b = int(cols[c0]), int(cols[c1])
            adj.setdefault(a, set()).add(b)
            adj.setdefault(b, set()).add(a)
    return adj


def nodes_at_hop(adj, start, hop):
    """snap.GetNodesAtHop(G, start, hop, v, True): nodes at EXACT BFS distance `hop`."""
    dist = {start: 0}
    q = deque([start])
    while q:
        n = q.popleft()
        if dist[n] == hop:
            continue
        for w in adj[n]:
            if w not in dist:
                dist[w] = dist[n] + 1
                q.append(w)
    return {n for n, d in dist.items() if d == hop}


def degree(adj, n):
    """G.GetNI(n).GetDeg() (similarity.py:121)."""
    return len(adj[n])


# --------------------------------------------------------------------------- scorers
def common_neighbors(s1, s2):  # similarity.py:113-114
    return len(s1.intersection(s2))


def jaccard(s1, s2):  # similarity.py:108-111
    return float(len(s1.intersection(s2))) / float(len(s1.union(s2)))


def adamic_adar(s1, s2, adj):  # similarity.py:116-126 (int 0 when nothing is added)
    total = 0
    for i in s1.intersection(s2):
        d = degree(adj, i)
        if d > 1:
            total += math.log(d) ** -1
        else:
            total += 0
    return total


def users(examples, adj, methods):
    """similarity.users (similarity.py:20-61) -> {method_index: u_sim}."""
    hop2s, neighbors = {}, {}
    for u in examples:
        if int(u) in adj:
            hop2s[int(u)] = nodes_at_hop(adj, int(u), 2)
    for u in examples:
        for v in examples[u]:
            if int(v) not in neighbors and int(v) in adj:
                neighbors[int(v)] = nodes_at_hop(adj, int(v), 1)
    out = []
    for m in methods:
        sim = defaultdict(dict)
        for u in examples:
            for v in examples[u]:
                if int(u) in adj and int(v) in adj:
                    if m == "common_neighbors":
                        sim[u][v] = common_neighbors(hop2s[int(u)], neighbors[int(v)])
                    elif m == "jaccard":
                        sim[u][v] = jaccard(hop2s[int(u)], neighbors[int(v)])
                    elif m == "adamic_adar":
                        sim[u][v] = adamic_adar(hop2s[int(u)], neighbors[int(v)], adj)
                else:
                    sim[u][v] = 0
        out.append(dict(sim))
    return out


def business(examples, adj, methods):
    """similarity.business (similarity.py:63-106), including the AA branch that only
    fires for the string at similarity.py:102."""
    hop2s, neighbors = {}, {}
    for u in examples:
        for v in examples[u]:
            if int(v) not in hop2s and int(v) in adj:
                hop2s[int(v)] = nodes_at_hop(adj, int(v), 2)
    for u in examples:
        if int(u) not in neighbors and int(u) in adj:
            neighbors[int(u)] = nodes_at_hop(adj, int(u), 1)
    out = []
    for m in methods:
        sim = defaultdict(dict)
        for u in examples:
            for v in examples[u]:
                if int(u) in adj and int(v) in adj:
                    if m == "common_neighbors":
                        sim[u][v] = common_neighbors(hop2s[int(v)], neighbors[int(u)])
                    elif m == "jaccard":
                        sim[u][v] = jaccard(hop2s[int(v)], neighbors[int(u)])
                    elif m == BUGGY_B_ADAMIC:
                        sim[u][v] = adamic_adar(hop2s[int(v)], neighbors[int(u)], adj)
                else:
                    sim[u][v] = 0
        out.append(dict(sim))
    return out


# --------------------------------------------------------------------------- svd.py
def svd_pair_scores(us, vt, rows, cols):
    """svd.py:28-30: np.dot(us[row, :], vt[:, col]) per pair."""
    return np.array([np.dot(us[r, :], vt[:, c]) for r, c in zip(rows, cols)], dtype=np.float64)


# --------------------------------------------------------------------------- random_walks.py
def svd_entry_parity(got, ref, structural_zero, rtol=1e-5, floor_frac=1e-6, zero_atol_frac=1e-12):
    """Per-entry comparison of two rank-k reconstructions (SURVEY.md §7 hard part 3; the
    north star's 1e-5 relative bar on svd.py:28-30 scores).

    * structural zeros -- pairs whose user row or business column of M is empty, so
      us[row] . vt[:, col] is 0 in exact arithmetic: `got` must be exactly 0.0 and `ref`
      within zero_atol_frac * scale (ARPACK's vectors of an empty row are 0 up to rounding);
    * every other entry: |got - ref| <= rtol * max(|ref|, floor), floor = floor_frac * scale
      (scale = max |ref|). The floor is the near-zero rule: an entry that cancels to below
      one millionth of the score scale carries no relative digits in either factorisation.
    Returns a dict with the verdict, the worst entry and the band counts."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    z = np.asarray(structural_zero, bool)
    scale = float(np.max(np.abs(ref))) if len(ref) else 0.0
    floor = floor_frac * scale
    zero_ok = bool(np.all(got[z] == 0.0) and np.all(np.abs(ref[z]) <= zero_atol_frac * scale))
    nz = ~z
    den = np.maximum(np.abs(ref[nz]), floor) if nz.any() else np.zeros(0)
    err = np.abs(got[nz] - ref[nz]) / np.where(den > 0, den, 1.0)
    worst = int(np.argmax(err)) if len(err) else -1
    idx = np.flatnonzero(nz)
    return {
        "entries": int(len(ref)), "structural_zeros": int(z.sum()), "structural_zeros_exact": zero_ok,
        "near_zero_band": int(np.sum(np.abs(ref[nz]) < floor)), "rtol": rtol, "floor": floor,
        "worst_rel_err": float(err[worst]) if worst >= 0 else 0.0,
        "worst_entry": {"index": int(idx[worst]), "got": float(got[idx[worst]]), "ref": float(ref[idx[worst]])}
        if worst >= 0 else None,
        "ok": bool(zero_ok and (len(err) == 0 or err[worst] <= rtol)),
    }


def random_walk_scores(edges, examples, iterations=10, jump_p=0.2):
    """random_walks.py:9-53 restated densely (small graphs only).

    Row order = first appearance in graph.txt (nx.read_edgelist, :14); the start
    vector and the scores are indexed by the integer node id (:36, :44-45)."""
    order = {}
    for a, b in edges:
        for x in (a, b):
            if x not in order:
                order[x] = len(order)
    n = len(order)
    A = np.zeros((n, n))
    for a, b in edges:
        A[order[a], order[b]] = 1.0
        A[order[b], order[a]] = 1.0
    T = A / A.sum(axis=1, keepdims=True)
    out = {}
    for u in examples:
        p = np.zeros(n)
        p[int(u)] = 1.0
        for _ in range(iterations):
            p = p @ T
            p *= 1 - jump_p
        out[u] = {b: p[int(b)] for b in examples[u]}
    return out


# --------------------------------------------------------------------------- eval.py
def roc_auc(ys, ps):
    """sklearn.roc_auc_score (eval.py:26) = tie-averaged Mann-Whitney U / (P*N)."""
    ys = np.asarray(ys, dtype=np.float64)
    ps = np.asarray(ps, dtype=np.float64)
    order = np.argsort(ps, kind="mergesort")
    sp = ps[order]
    ranks = np.empty(len(ps))
    i = 0
    while i < len(sp):
        j = i
        while j + 1 < len(sp) and sp[j + 1] == sp[i]:
            j += 1
        ranks[order[i : j + 1]] = 0.5 * (i + j) + 1.0
        i = j + 1
    npos = ys.sum()
    nneg = len(ys) - npos
    return (ranks[ys == 1].sum() - npos * (npos + 1) / 2.0) / (npos * nneg)


def precision_at(examples, predictions, k=20):
    """eval.py:17-31: stable sort by score desc, top min(k, len) per user, / len(examples)."""
    total = 0.0
    for u in predictions:
        pairs = [(examples[u][b], predictions[u][b]) for b in predictions[u]]
        n = min(k, len(pairs))
        top = sorted(pairs, key=lambda t: t[1], reverse=True)[:n]
        total += sum(t[0] for t in top) / float(n)
    return total / len(examples)


# --------------------------------------------------------------------------- dataset_maker.py
def hop3_candidates(adj, u):
    """dataset_maker.py:138-139: snap.GetNodesAtHop(G, u, 3)."""
    return nodes_at_hop(adj, u, 3)


# --------------------------------------------------------------------------- full-candidate top-k
def adamic_adar_exact(s1, s2, adj):
    """adamic_adar (similarity.py:116-126) with the terms added exactly and rounded once
    (math.fsum): the value the engine returns (blp_internal.h). The reference adds the same
    terms in Python set order with a rounding per add, so it agrees to a few ulps; keeps the
    reference's int 0 when nothing is added."""
    terms = []
    for w in s1.intersection(s2):
        d = degree(adj, w)
        if d > 1:
            terms.append(math.log(d) ** -1)
    return math.fsum(terms) if terms else 0


def topk_full_candidates(adj, x, k, method):
    """BASELINE.json configs[2]: score EVERY node b at exact distance 3 of x (the candidate
    set dataset_maker.py:139 samples from) with similarity.py's measure of (H2(x), N(b))
    (similarity.py:48-58 orientation: H2 of the source, hop-1 set of the candidate) and keep
    the k best: score descending, then node id ascending. The reference has no top-k; this
    composes its scorers. Returns ([(b, score)], n_candidates)."""
    h2 = nodes_at_hop(adj, x, 2)
    cands = nodes_at_hop(adj, x, 3)
    rows = []
    for b in cands:
        nb = nodes_at_hop(adj, b, 1)
        if method == "common_neighbors":
            s = common_neighbors(h2, nb)
            key = s
        elif method == "jaccard":
            s = jaccard(h2, nb)
            key = s
        else:
            s = adamic_adar_exact(h2, nb, adj)
            key = s
        rows.append((-key, b, s))
    rows.sort()
    return [(b, s) for _, b, s in rows[:k]], len(cands)
