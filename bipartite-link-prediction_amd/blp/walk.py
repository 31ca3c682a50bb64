"""Device random walks (random_walks.py:9-53): dense fp64 SpMM walks over W = T^T."""
import ctypes

import numpy as np
import scipy.sparse as sp

from . import _lib
from ._lib import check, lib, ptr

_P, _I64, _I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
_lib.register("blp_walk_create", [_P, _P, _P, _I64, _I32, ctypes.POINTER(ctypes.c_void_p)])
_lib.register("blp_walk_destroy", [_P])
_lib.register("blp_walk_run", [_P, _P, _I64, _I32, ctypes.c_double, _P, _P, _I64, _P])
_lib.register("blp_walk_run_dense", [_P, _I32, _I32, ctypes.c_double, _P])
_lib.register("blp_walk_stats", [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)])


class DeviceWalk:
    """A transition matrix T (n x n, scipy sparse or CSR arrays of W = T^T) in HBM."""

    def __init__(self, T=None, *, wt_csr=None, device=0):
        if wt_csr is None:
            W = sp.csr_matrix(T).T.tocsr()  # pull form: row j holds T[:, j]
            W.sort_indices()
            wt_csr = (W.indptr, W.indices, W.data, W.shape[0])
        rp, ci, val, n = wt_csr
        self.rp = np.ascontiguousarray(rp, dtype=np.int64)
        self.ci = np.ascontiguousarray(ci, dtype=np.int32)
        self.val = np.ascontiguousarray(val, dtype=np.float64)
        self.n = int(n)
        h = ctypes.c_void_p()
        check(lib().blp_walk_create(ptr(self.rp), ptr(self.ci), ptr(self.val), self.n, device, ctypes.byref(h)))
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            lib().blp_walk_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, starts, q_start, q_node, iterations=10, scale=0.8):
        starts = _lib.as_i32(starts)
        q_start = _lib.as_i32(q_start)
        q_node = _lib.as_i32(q_node)
        out = np.zeros(len(q_start), np.float64)
        check(lib().blp_walk_run(self.handle, ptr(starts), len(starts), iterations, scale, ptr(q_start), ptr(q_node),
                                 len(q_start), ptr(out)))
        return out

    def run_dense(self, start, iterations=10, scale=0.8):
        out = np.zeros(self.n, np.float64)
        check(lib().blp_walk_run_dense(self.handle, int(start), iterations, scale, ptr(out)))
        return out

    def stats(self):
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        check(lib().blp_walk_stats(self.handle, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value
