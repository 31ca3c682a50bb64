"""Drop-in for the reference's svd.py: truncated-SVD link scores, reconstructed on the GPU.

``svd_user_business(data_dir, k=50)`` (svd.py:7-31) keeps the reference's steps: rows and
columns in user.json / business.json key order (svd.py:9-14), the binary user x business
matrix from graph.txt (svd.py:16-21), the rank-k factorisation of svd.py:24-25 --
``blp.factor.svds`` on the GPU (block subspace iteration, agrees with ARPACK to ~1e-13 of
the score scale) for matrices with at least 256 rows and columns, the reference's own
``scipy.sparse.linalg.svds`` for smaller ones (a 128-column block does not fit them) -- and
every candidate pair's ``np.dot(us[row], vt[:, col])`` (svd.py:28-30) computed by libblp's
fp64 kernel; the scores are written to ./data/<dir>/svd.json.
``svd_topk`` is new: the full-candidate ranking (every business per user) on fp64 MFMA.
"""
import numpy as np
import scipy.sparse.linalg  # noqa: F401  (sparse.linalg.svds)
from scipy import sparse

import blp
import util
from blp.factor import DeviceSVD


def user_business_matrix(data_dir):
    """svd.py:9-21: (users, businesses, examples, csr matrix) in the reference's order."""
    users = list(util.load_json("./data/" + data_dir + "/user.json").keys())
    businesses = list(util.load_json("./data/" + data_dir + "/business.json").keys())
    examples = util.load_json("./data/" + data_dir + "/examples.json")
    user_to_row = dict(zip(users, range(len(users))))
    business_to_column = dict(zip(businesses, range(len(businesses))))
    rows, cols = [], []
    with open("./data/" + data_dir + "/graph.txt") as f:  # svd.py:17-20: string keys
        for line in f:
            u, b = line.split()
            rows.append(user_to_row[u])
            cols.append(business_to_column[b])
    M = sparse.csr_matrix((np.ones(len(rows)), (rows, cols)), shape=(len(users), len(businesses)))
    M.sum_duplicates()
    M.data[:] = 1.0  # lil_matrix assignment of 1 is idempotent on repeated reviews
    return users, businesses, examples, user_to_row, business_to_column, M


def factorize(M, k, factor="auto", device=0):
    """svd.py:24-25 -> (us = u * s, vt). factor: 'gpu' (blp.factor.svds), 'host' (scipy
    ARPACK, the reference's numeric) or 'auto' (gpu when M has >= 256 rows and columns and
    k < 128)."""
    from blp import factor as F

    auto = factor == "auto"
    if auto:
        factor = "gpu" if min(M.shape) >= 256 and k < F.block_width() else "host"
    if factor == "gpu":
        try:
            us, s, v = F.svds(M, k=k, device=device, return_us=True)
            return us, np.ascontiguousarray(v.T)
        except RuntimeError as e:  # Ritz values did not settle: 'auto' takes the reference's ARPACK
            if not auto or isinstance(e, (blp.BLPError, blp.BLPUnavailable)):
                raise
            print("GPU factorisation did not converge (%s); using scipy.sparse.linalg.svds" % e)
    u, s, vt = sparse.linalg.svds(M, k=k)
    return u * s, vt


def svd_user_business(data_dir, k=50, device=0, factor="auto"):
    print("Loading data and building user-business matrix...")
    users, businesses, examples, user_to_row, business_to_column, M = user_business_matrix(data_dir)
    print("Computing singular value decomposition...")
    us, vt = factorize(M, k, factor, device)
    print("Writing results...")
    scores = score_examples(examples, us, vt, user_to_row, business_to_column, device=device)
    i = 0
    for uk in examples:
        for bk in examples[uk]:
            examples[uk][bk] = scores[i]
            i += 1
    util.write_json(examples, "./data/" + data_dir + "/svd.json")
    return examples


def score_examples(examples, us, vt, user_to_row, business_to_column, device=0):
    """np.dot(us[row], vt[:, col]) for every pair of examples, in dict order, on the GPU."""
    rows, cols = [], []
    for uk, inner in examples.items():
        r = user_to_row[uk]
        for bk in inner:
            rows.append(r)
            cols.append(business_to_column[bk])
    dev = DeviceSVD(us, np.ascontiguousarray(vt.T), device=device)
    try:
        return dev.score_pairs(np.array(rows, np.int32), np.array(cols, np.int32)).tolist()
    finally:
        dev.close()


def svd_topk(us, vt, user_rows, topk=20, exclude=None, device=0):
    """Top-`topk` businesses per user over ALL businesses (score desc, column asc) on fp64
    MFMA; exclude: optional CSR (offsets, sorted columns) of columns to skip per user."""
    dev = DeviceSVD(us, np.ascontiguousarray(vt.T), device=device)
    try:
        return dev.topk(user_rows, topk=topk, exclude=exclude)
    finally:
        dev.close()


def svd(data_dir, k=50):
    """svd.py:34-48 (dead code in the reference): it indexes us[u, :] with the STRING key u
    (svd.py:47) and raises IndexError before writing anything; kept with that behaviour."""
    print("Loading data and building adjacency matrix...")
    examples = util.load_json("./data/" + data_dir + "/examples.json")
    for u in examples:
        for _ in examples[u]:
            raise IndexError("only integers, slices (`:`), ellipsis (`...`), numpy.newaxis (`None`) and integer "
                             "or boolean arrays are valid indices")
    util.write_json(examples, "./data/" + data_dir + "/svd.json")  # reached only with no pairs


if __name__ == "__main__":
    svd_user_business("train")
    svd_user_business("test")
