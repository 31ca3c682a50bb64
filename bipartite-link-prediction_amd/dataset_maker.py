"""Drop-in for the candidate generation of the reference's dataset_maker.py.

``make_examples(data_dir, n_users=5000, min_degree=1, negative_sample_rate=0.01,
min_active_time=None, new_edge_only=False)`` keeps dataset_maker.py:80-159:
* the candidate users: nodes with a review.json entry and degree >= min_degree, optionally
  only users with a new edge (new_edge_only) or a review after min_active_time (:95-115);
* ``random.seed(0); random.sample(users, n_users)`` (:133-134);
* for every sampled user u, EVERY node at exact distance 3 (GetNodesAtHop(G, u, 3), :139)
  is a candidate; a candidate that is a new edge (new_edges.txt) is labelled 1 (:141-142),
  the others are kept with probability negative_sample_rate and labelled 0 (:143-144);
* the result is written to data_dir + 'examples.json' as {user: {business: label}}.

The hop-3 enumeration, positive labelling and negative sampling run on the GPU
(``blp_hop3_sample``). The candidate SETS are exact. Two things are statistical parity
only, because the reference's order comes from SNAP's hash-table and BFS iteration:
* the 1% negative draw uses a counter-based hash of (seed, u, b);
* the user sample is taken over the graph's node order.
The make_dataset ETL over the raw Yelp dump (:162-201) is out of scope.
"""
import datetime
import random

import numpy as np

import blp
import util


def get_date(review):
    """dataset_maker.get_date: a review's 'date' field (YYYY-MM-DD) as a datetime.date."""
    return datetime.datetime.strptime(review["date"], "%Y-%m-%d").date()


def _read_edges(path):
    with open(path) as f:
        return {tuple(map(int, line.split())) for line in f if line.strip()}


def make_examples(data_dir, n_users=5000, min_degree=1, negative_sample_rate=0.01, min_active_time=None,
                  new_edge_only=False, device=0, seed=0):
    print("Loading data...")
    G = blp.load_edge_list(data_dir + "graph.txt", device=device)
    edges = _read_edges(data_dir + "new_edges.txt")
    new_edge_count = {}
    for (u, b) in edges:
        new_edge_count[u] = new_edge_count.get(u, 0) + 1
    review_data = util.load_json(data_dir + "review.json")

    print("Getting candidate set of users...")
    users = []
    for i, u in enumerate(G.node_ids.tolist()):  # G.Nodes() (:93)
        if new_edge_only and u not in new_edge_count:
            continue
        if str(u) not in review_data or G.degree[i] < min_degree:
            continue
        if min_active_time:
            recent = False
            for b in review_data[str(u)]:
                if (int(u), int(b)) in edges:
                    continue
                if any(get_date(r) > min_active_time for r in review_data[str(u)][b]):
                    recent = True
                    break
            if not recent:
                continue
        users.append(u)

    random.seed(0)
    users = random.sample(users, min(n_users, len(users)))

    print("Getting candidate set of edges...")
    src = G.dense(users)
    eu = np.array([e[0] for e in edges], np.int64)
    eb = np.array([e[1] for e in edges], np.int64)
    ru = np.full(len(eu), -1, np.int64)
    if len(eu):
        order = np.argsort(np.asarray(users, np.int64))
        su = np.asarray(users, np.int64)[order]
        pos = np.minimum(np.searchsorted(su, eu), max(len(su) - 1, 0))
        hit = len(su) > 0
        ru = np.where(hit & (su[pos] == eu), order[pos], -1) if hit else ru
    db, okb = G.lookup(eb)
    keep = (ru >= 0) & okb
    ru, db = ru[keep], db[keep]
    o = np.argsort(ru, kind="stable")
    ru, db = ru[o], db[o]
    pos_off = np.zeros(len(users) + 1, np.int64)
    np.add.at(pos_off, ru + 1, 1)
    pos_off = np.cumsum(pos_off).astype(np.int32)
    pos_y = db.astype(np.int32) if len(db) else np.zeros(1, np.int32)
    x, y, lab = G.hop3_sample(src, pos_off, pos_y, rate=negative_sample_rate, seed=seed)
    examples = {}
    for xi, yi, li in zip(G.node_ids[x].tolist(), G.node_ids[y].tolist(), lab.tolist()):
        examples.setdefault(str(xi), {})[str(yi)] = int(li)
    print("Writing examples...")
    util.write_json(examples, data_dir + "examples.json")
    return examples
