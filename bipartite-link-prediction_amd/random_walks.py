"""Drop-in for the reference's random_walks.py, walked on the GPU (blp.walk).

Same call surface and output (random_walks.py:9-53):
* ``run_random_walks(data_dir, weight_edges=False)`` -- like the reference it forces
  ``data_dir = 'train'`` and ``weight_edges = False`` (random_walks.py:11-12), builds the
  unweighted transition matrix T = D^-1 A over the nodes of graph.txt in FIRST-APPEARANCE
  order (nx.read_edgelist, :14,:26-29), walks 10 damped steps (jump_p = 0.2, restart
  commented out at :51) from row ``int(u)`` of every example user and writes
  ``p[int(b)]`` (:36-37) to ./data/train/random_walks.json. As in the reference, a node id
  is used directly as a matrix row, which is the node itself only when ids are dense and in
  first-appearance order (what dataset_maker writes); Python's negative-index wrap and the
  IndexError for ids >= n are kept.
* ``run_random_walk(transition_matrix, u, iterations, jump_p)`` -- returns p as a 1 x n
  sparse row like the reference's scipy product (:43-53).
On a bipartite graph an even number of steps from a user leaves all mass on users, so every
(user, business) score is exactly 0.0 -- the reference's own result (tests/golden/bip).
"""
import numpy as np
import scipy.sparse as sp

import blp
import util
from blp.walk import DeviceWalk


def transition_pull_csr(path):
    """graph.txt -> (order, W = T^T CSR) with T = D^-1 A over first-appearance order.

    A is the simple undirected graph (nx.Graph): duplicates merged, a self-loop a diagonal 1."""
    a, b = blp.parse_edge_list(path)
    seq = np.empty(2 * len(a), np.int64)
    seq[0::2] = a
    seq[1::2] = b
    uniq, first = np.unique(seq, return_index=True)
    order = uniq[np.argsort(first, kind="stable")]  # position -> node id
    pos = np.empty(len(order), np.int64)
    pos[np.argsort(order)] = np.arange(len(order))
    pa = pos[np.searchsorted(uniq, a)]
    pb = pos[np.searchsorted(uniq, b)]
    n = len(order)
    A = sp.coo_matrix((np.ones(2 * len(pa)), (np.r_[pa, pb], np.r_[pb, pa])), shape=(n, n)).tocsr()
    A.data[:] = 1.0  # merged duplicates and the doubled self-loop entry -> 1
    rs = np.asarray(A.sum(axis=1)).ravel()
    W = (A @ sp.diags(1.0 / rs)).tocsr()  # W[j, i] = A[j, i] / rs[i] = T[i, j]
    W.sort_indices()
    return order, (W.indptr, W.indices, W.data, n)


def _row(idx, n):
    """Python list indexing of a length-n vector (p[int(u)] = 1.0, random_walks.py:45)."""
    i = int(idx)
    if i < -n or i >= n:
        raise IndexError("list assignment index out of range")
    return i % n


def run_random_walks(data_dir, weight_edges=False, iterations=10, jump_p=0.2, device=0):
    print("Loading data and building transition matrix...")
    data_dir = "train"  # random_walks.py:11-12: the reference overrides both arguments
    weight_edges = False
    examples = util.load_json("./data/" + data_dir + "/examples.json")
    order, wt = transition_pull_csr("./data/" + data_dir + "/graph.txt")
    n = len(order)
    print("Running random walks...")
    starts, qs, qn = [], [], []
    for si, u in enumerate(examples):
        starts.append(_row(u, n))
        for bk in examples[u]:
            qs.append(si)
            qn.append(_row(bk, n))
    walk = DeviceWalk(wt_csr=wt, device=device)
    try:
        vals = walk.run(np.array(starts, np.int32), np.array(qs, np.int32), np.array(qn, np.int32),
                        iterations=iterations, scale=1.0 - jump_p).tolist()
    finally:
        walk.close()
    i = 0
    for u in examples:
        for bk in examples[u]:
            examples[u][bk] = vals[i]
            i += 1
    util.write_json(examples, "./data/" + data_dir
                    + ("/weighted_random_walks.json" if weight_edges else "/random_walks.json"))


def run_random_walk(transition_matrix, u, iterations, jump_p):
    """p = e_u; iterations x { p = p . T; p *= (1 - jump_p) }  (random_walks.py:43-53)."""
    walk = DeviceWalk(transition_matrix)
    try:
        p = walk.run_dense(_row(u, walk.n), iterations=iterations, scale=1.0 - jump_p)
    finally:
        walk.close()
    return sp.csr_matrix(p.reshape(1, -1))


if __name__ == "__main__":
    run_random_walks("train", False)
    run_random_walks("train", False)
    run_random_walks("test", False)
    run_random_walks("test", True)
