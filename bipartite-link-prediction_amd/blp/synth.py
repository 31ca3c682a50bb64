"""Synthetic review graphs and example batches; no data ships with the
reference (data/.gitignore:1-4) and the Yelp dump is absent, so every benchmark and
scale test runs on these seeded stand-ins of the reference's data shapes.

Graph: users ``0..U-1`` and businesses ``U..U+B-1`` (disjoint id space as in
dataset_maker.py:173-174), ``draws`` reviews with a uniform user and a business drawn with
popularity proportional to rank^-0.8, duplicates merged by the graph loader.
Examples: sampled users, their exact distance-3 candidates (dataset_maker.py:139) labelled
by a held-out second draw of new edges (:141-142), negatives kept at rate 0.01 (:143-144),
computed on the GPU by ``DeviceGraph.hop3_sample``.
"""
import numpy as np

CONFIGS = {
    # name: (users, businesses, draws)
    "yelp": (252_898, 42_153, 1_125_458),  # config 1 shape (writeups/proposal.tex:93)
    "c2": (1_000_000, 100_000, 10_000_000),  # configs 2 / 3
    "c4": (2_000_000, 200_000, 50_000_000),  # config 4
    "c5": (50_000_000, 2_000_000, 1_000_000_000),  # config 5
}


def popularity(n_bus, zipf=0.8):
    p = np.arange(1, n_bus + 1, dtype=np.float64) ** -zipf
    return p / p.sum()


def review_edges(users, businesses, draws, seed=0, zipf=0.8, chunk=50_000_000):
    """(user_id, business_id) int64 arrays of `draws` reviews (duplicates kept, like graph.txt)."""
    rng = np.random.default_rng(seed)
    cdf = np.cumsum(popularity(businesses, zipf))
    cdf[-1] = 1.0
    u = np.empty(draws, np.int64)
    b = np.empty(draws, np.int64)
    for s in range(0, draws, chunk):
        e = min(draws, s + chunk)
        u[s:e] = rng.integers(0, users, e - s)
        b[s:e] = np.searchsorted(cdf, rng.random(e - s), side="right") + users
    np.minimum(b, users + businesses - 1, out=b)
    return u, b


def heldout_edges(users, businesses, draws, seed=1, zipf=0.8):
    """The 'new edges' draw (dataset_maker.py:198-199 analogue): 1% more reviews, seed 1."""
    return review_edges(users, businesses, max(1, draws // 100), seed=seed, zipf=zipf)


def sample_users(G, n_users, seed=0):
    """Dense ids of `n_users` distinct users with degree >= 1 (dataset_maker.py:101,133)."""
    rng = np.random.default_rng(seed)
    cand = np.flatnonzero((G.node_ids < G.n_users_hint) & (G.hop1_size > 0)) if hasattr(G, "n_users_hint") else \
        np.flatnonzero(G.hop1_size > 0)
    return np.sort(rng.choice(cand, size=min(n_users, len(cand)), replace=False)).astype(np.int32)


def positives_csr(G, src, new_u, new_b):
    """Group held-out (user, business) edges by source position -> (pos_off, pos_y) dense."""
    du, okk = G.lookup(new_u)
    db, okb = G.lookup(new_b)
    ok = okk & okb
    du, db = du[ok], db[ok]
    rank = np.full(G.n, -1, np.int64)
    rank[src] = np.arange(len(src))
    r = rank[du]
    keep = r >= 0
    r, db = r[keep], db[keep]
    order = np.argsort(r, kind="stable")
    r, db = r[order], db[order]
    pos_off = np.zeros(len(src) + 1, np.int64)
    np.add.at(pos_off, r + 1, 1)
    return np.cumsum(pos_off).astype(np.int32), db.astype(np.int32)


def make_examples(G, users, businesses, draws, n_users=10_000, rate=0.01, seed=0, zipf=0.8):
    """Candidate (user, business, label) triples for `n_users` sampled users (dense ids)."""
    G.n_users_hint = users
    src = sample_users(G, n_users, seed=seed)
    nu, nb = heldout_edges(users, businesses, draws, seed=seed + 1, zipf=zipf)
    pos_off, pos_y = positives_csr(G, src, nu, nb)
    return G.hop3_sample(src, pos_off, pos_y, rate=rate, seed=seed)


def uniform_examples(G, src, rate=0.01, seed=0):
    """Candidate pairs for graphs too large for exact hop-3 enumeration per source (config 5:
    H3(u) is nearly every business): each business outside N(u) is kept with probability
    `rate`, uniformly -- the distribution dataset_maker.py:143 draws from when H3(u) covers
    the business set. Labels are not produced (no held-out draw at this scale)."""
    rng = np.random.default_rng(seed)
    n0 = G.n_col0
    nb = G.n - n0
    xs, ys = [], []
    for x in src:
        k = rng.binomial(nb, rate)
        cand = np.unique(rng.integers(0, nb, k)) + n0
        own = G.col_idx[G.row_ptr[x]:G.row_ptr[x + 1]]
        cand = cand[~np.isin(cand, own)]
        xs.append(np.full(len(cand), x, np.int32))
        ys.append(cand.astype(np.int32))
    return np.concatenate(xs), np.concatenate(ys)
