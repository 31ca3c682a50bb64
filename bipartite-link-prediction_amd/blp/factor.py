"""Device-resident truncated-SVD factors: reconstruction of svd.py:25-30 on the GPU."""
import ctypes
import time

import numpy as np

from . import _lib
from ._lib import check, lib, ptr

_P, _I64, _I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
_lib.register("blp_svd_create", [_P, _I64, _P, _I64, _I32, _I32, ctypes.POINTER(ctypes.c_void_p)])
_lib.register("blp_svd_destroy", [_P])
_lib.register("blp_svd_score_pairs", [_P, _P, _P, _I64, _P])
_lib.register("blp_svd_score_pairs_device", [_P, _P, _P, _I64, _P])
_lib.register("blp_svd_topk_device", [_P, _P, _I64, _P, _P, _I32, _P, _P])
_lib.register("blp_svd_topk", [_P, _P, _I64, _P, _P, _I32, _P, _P])
_lib.register("blp_svd_stats", [_P, _I32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)])
_lib.register("blp_svd_sync", [_P])
_lib.register("blp_svd_stream_join", [_P, _P, _I32])
_lib.register("blp_svd_set_prune", [_P, _I32])
_lib.register("blp_svd_tiles", [_P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)])


class DeviceSVD:
    """us = u * s (n_rows x k) and v = vt.T (n_cols x k) in HBM, fp64 (svd.py:24-25)."""

    def __init__(self, us, v, device=0):
        self.us = np.ascontiguousarray(us, dtype=np.float64)
        self.v = np.ascontiguousarray(v, dtype=np.float64)
        if self.us.ndim != 2 or self.v.ndim != 2 or self.us.shape[1] != self.v.shape[1]:
            raise ValueError("factors must be (n_rows, k) and (n_cols, k)")
        self.n_rows, self.k = self.us.shape
        self.n_cols = self.v.shape[0]
        self.device = device
        h = ctypes.c_void_p()
        check(lib().blp_svd_create(ptr(self.us), self.n_rows, ptr(self.v), self.n_cols, self.k, device,
                                   ctypes.byref(h)))
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            lib().blp_svd_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def score_pairs(self, rows, cols):
        """np.dot(us[row, :], vt[:, col]) per pair (svd.py:28-30)."""
        rows = _lib.as_i32(rows)
        cols = _lib.as_i32(cols)
        out = np.zeros(len(rows), np.float64)
        check(lib().blp_svd_score_pairs(self.handle, ptr(rows), ptr(cols), len(rows), ptr(out)))
        return out

    def topk(self, users, topk=20, exclude=None):
        """Best `topk` columns per selected row over all columns (score desc, column asc).

        exclude: optional list/tuple (offsets, cols) CSR over the selected rows, sorted cols."""
        users = _lib.as_i32(users)
        oc = np.zeros((len(users), topk), np.int32)
        os_ = np.zeros((len(users), topk), np.float64)
        eo = ec = None
        if exclude is not None:
            eo = np.ascontiguousarray(exclude[0], dtype=np.int64)
            ec = _lib.as_i32(exclude[1] if len(exclude[1]) else np.zeros(1, np.int32))
        check(lib().blp_svd_topk(self.handle, ptr(users), len(users), ptr(eo), ptr(ec), topk, ptr(oc), ptr(os_)))
        return oc, os_

    def topk_device(self, users, topk, out_cols, out_scores, exclude=None):
        """blp_svd_topk_device: every argument a device-resident torch tensor on this handle's
        device (users int32 [n]; exclude (int64 offsets [n+1], int32 cols) or None; out_cols
        int32 [n, topk], out_scores float64 [n, topk]), all contiguous.

        Stream contract: the handle's stream first waits for the work queued so far on torch's
        current stream (so inputs made by torch kernels are complete), and torch's current
        stream then waits for the top-k (so the outputs are complete before torch reads,
        reuses or frees them). Returns without a host sync (sync() waits)."""
        import torch

        dev = torch.device("cuda", self.device)
        n = users.numel()

        def want(t, name, dtype, shape):
            if not isinstance(t, torch.Tensor) or t.device != dev or t.dtype != dtype or not t.is_contiguous() \
                    or tuple(t.shape) != tuple(shape):
                raise ValueError("topk_device: %s must be a contiguous %s tensor of shape %s on %s (got %s)" % (
                    name, dtype, tuple(shape), dev, (getattr(t, "dtype", type(t)), tuple(getattr(t, "shape", ())),
                                                   getattr(t, "device", None))))

        if not 1 <= int(topk) <= 256:
            raise ValueError("topk_device: topk must be in [1, 256]")
        want(users, "users", torch.int32, (n,))
        want(out_cols, "out_cols", torch.int32, (n, topk))
        want(out_scores, "out_scores", torch.float64, (n, topk))
        eo = ec = None
        if exclude is not None:
            want(exclude[0], "exclude offsets", torch.int64, (n + 1,))
            want(exclude[1], "exclude cols", torch.int32, (exclude[1].numel(),))
            eo, ec = exclude[0].data_ptr(), exclude[1].data_ptr()
        cur = torch.cuda.current_stream(dev).cuda_stream
        check(lib().blp_svd_stream_join(self.handle, cur, 1))
        check(lib().blp_svd_topk_device(self.handle, users.data_ptr(), n, eo, ec, topk,
                                        out_cols.data_ptr(), out_scores.data_ptr()))
        check(lib().blp_svd_stream_join(self.handle, cur, 0))

    def sync(self):
        check(lib().blp_svd_sync(self.handle))

    def set_prune(self, on=True):
        """Top-k by norm pruning (the default; same lists) or the dense pass over every pair."""
        check(lib().blp_svd_set_prune(self.handle, 1 if on else 0))

    def tiles(self):
        """(MFMA tiles of 16 users x 16 businesses scored, tiles of the dense pass) over the top-k
        calls since the last tiles() call."""
        a, b = ctypes.c_int64(0), ctypes.c_int64(0)
        check(lib().blp_svd_tiles(self.handle, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def stats(self, which=0):
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        check(lib().blp_svd_stats(self.handle, which, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value


# ------------------------------------------------------------------ factorisation on the GPU
_lib.register("blp_fact_create", [_P, _P, _I64, _I64, _I32, ctypes.POINTER(ctypes.c_void_p)])
_lib.register("blp_fact_destroy", [_P])
_lib.register("blp_fact_block_width", [])
_lib.register("blp_fact_set_q", [_P, _P])
_lib.register("blp_fact_step", [_P, _P])
_lib.register("blp_fact_gram_w", [_P, _P])
_lib.register("blp_fact_apply_w", [_P, _P, _I32])
_lib.register("blp_fact_extract", [_P, _P, _I32, _P, _P])
_lib.register("blp_fact_stats", [_P, _I32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)])


def block_width():
    """Columns of the subspace block (k must be smaller)."""
    return lib().blp_fact_block_width()


class FactorStats:
    def __init__(self):
        self.iterations = 0
        self.converged_at = None
        self.spmm_ms = 0.0
        self.dense_ms = 0.0
        self.ritz = None
        self.create_s = 0.0


def _sym(S):
    return 0.5 * (S + S.T)


def svds(M, k=6, tol=1e-12, max_iter=400, seed=0, device=0, stats=None, return_us=False):
    """scipy.sparse.linalg.svds(M, k) for a BINARY sparse matrix (svd.py:24), on the GPU.

    Block subspace iteration on M^T M with a 128-column fp64 block and Rayleigh-Ritz
    (csrc/factor.hip). Stops once the top-k Ritz values change by < `tol` (relative) between
    iterations AND as many iterations again have run (the subspace error keeps falling ~5x
    per 3 iterations after the Ritz values settle: tests/test_gpu_factor.py).
    Returns (u, s, vt) like svds: s ascending, u[:, i] / vt[i] the matching vectors; or, with
    return_us, (us, s, v) with us = u * s and v = vt.T in descending order (what svd.py's
    reconstruction needs, without the divide/multiply round trip)."""
    from scipy import sparse

    M = sparse.csr_matrix(M)
    if M.nnz and not np.all(M.data == 1):
        raise ValueError("blp.factor.svds: the matrix must be binary (svd.py:20 assigns 1)")
    M.sort_indices()
    n_rows, n_cols = M.shape
    Pw = lib().blp_fact_block_width()
    if not 1 <= k < Pw // 1:
        raise ValueError("blp.factor.svds: k must be in [1, %d)" % Pw)
    if min(n_rows, n_cols) < Pw:
        raise ValueError("blp.factor.svds: the matrix must have at least %d rows and columns" % Pw)
    rp = np.ascontiguousarray(M.indptr, np.int64)
    ci = np.ascontiguousarray(M.indices, np.int32)
    h = ctypes.c_void_p()
    t_create = time.perf_counter()
    check(lib().blp_fact_create(ptr(rp), ptr(ci), n_rows, n_cols, device, ctypes.byref(h)))
    st = stats if stats is not None else FactorStats()
    try:
        # a Gaussian start block: the first step's W = M^T M Q0 is orthonormalised on the device
        # like every later one (only span(Q0) matters); its Ritz values are not used
        st.create_s = time.perf_counter() - t_create
        rng = np.random.default_rng(seed)
        q = rng.standard_normal((n_cols, Pw)) / np.sqrt(n_cols)
        check(lib().blp_fact_set_q(h, ptr(q)))
        S = np.empty((Pw, Pw))
        G = np.empty((Pw, Pw))
        prev = None
        for it in range(1, max_iter + 1):
            check(lib().blp_fact_step(h, ptr(S)))
            lam = np.sort(np.linalg.eigvalsh(_sym(S)))[::-1][:k]
            # relative change, with the denominator floored at eps * lam_1: a zero Ritz value
            # (rank(M) < k) must not turn the test into NaN and run all max_iter iterations
            den = np.maximum(np.abs(lam), np.finfo(np.float64).eps * max(abs(lam[0]), np.finfo(np.float64).tiny))
            if it > 1 and prev is not None and st.converged_at is None and np.max(np.abs(lam - prev) / den) < tol:
                st.converged_at = it
            prev = lam
            st.iterations = it
            if st.converged_at is not None and it >= 2 * st.converged_at:
                break
            # Q <- orth(W): shifted CholeskyQR then CholeskyQR (the shift keeps a nearly
            # rank-deficient block factorisable; the second pass restores orthogonality)
            for rep in range(2):
                check(lib().blp_fact_gram_w(h, ptr(G)))
                Gs = _sym(G)
                if rep == 0:
                    Gs = Gs + np.eye(Pw) * (1e-14 * np.trace(Gs))
                R = np.linalg.cholesky(Gs).T  # upper: G = R^T R
                Rinv = np.ascontiguousarray(np.linalg.inv(R))
                check(lib().blp_fact_apply_w(h, ptr(Rinv), 1 if rep == 1 else 0))
        if st.converged_at is None:
            raise RuntimeError("blp.factor.svds: the top-%d Ritz values did not settle to %g within %d iterations; "
                               "raise max_iter or use scipy.sparse.linalg.svds" % (k, tol, max_iter))
        lam_all, V = np.linalg.eigh(_sym(S))
        order = np.argsort(-lam_all)
        Vd = np.zeros((Pw, Pw))
        Vd[:, :k] = V[:, order[:k]]
        us = np.empty((n_rows, k))
        v = np.empty((n_cols, k))
        check(lib().blp_fact_extract(h, ptr(np.ascontiguousarray(Vd)), k, ptr(us), ptr(v)))
        sig = np.sqrt(np.maximum(lam_all[order[:k]], 0.0))
        st.ritz = lam_all[order[:k]]
        for which, attr in ((0, "spmm_ms"), (1, "dense_ms")):
            ms = ctypes.c_double(0)
            n = ctypes.c_int64(0)
            check(lib().blp_fact_stats(h, which, ctypes.byref(ms), ctypes.byref(n)))
            setattr(st, attr, ms.value)
    finally:
        lib().blp_fact_destroy(h)
    if return_us:
        return us, sig, v
    with np.errstate(divide="ignore", invalid="ignore"):
        u = np.where(sig > 0, us / sig, 0.0)
    return u[:, ::-1].copy(), sig[::-1].copy(), v[:, ::-1].T.copy()
