"""Device-resident truncated-SVD factors: reconstruction of svd.py:25-30 on the GPU."""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib, ptr

_P, _I64, _I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
_lib.register("blp_svd_create", [_P, _I64, _P, _I64, _I32, _I32, ctypes.POINTER(ctypes.c_void_p)])
_lib.register("blp_svd_destroy", [_P])
_lib.register("blp_svd_score_pairs", [_P, _P, _P, _I64, _P])
_lib.register("blp_svd_score_pairs_device", [_P, _P, _P, _I64, _P])
_lib.register("blp_svd_topk", [_P, _P, _I64, _P, _P, _I32, _P, _P])
_lib.register("blp_svd_stats", [_P, _I32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)])
_lib.register("blp_svd_sync", [_P])


class DeviceSVD:
    """us = u * s (n_rows x k) and v = vt.T (n_cols x k) in HBM, fp64 (svd.py:24-25)."""

    def __init__(self, us, v, device=0):
        self.us = np.ascontiguousarray(us, dtype=np.float64)
        self.v = np.ascontiguousarray(v, dtype=np.float64)
        if self.us.ndim != 2 or self.v.ndim != 2 or self.us.shape[1] != self.v.shape[1]:
            raise ValueError("factors must be (n_rows, k) and (n_cols, k)")
        self.n_rows, self.k = self.us.shape
        self.n_cols = self.v.shape[0]
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

    def stats(self, which=0):
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        check(lib().blp_svd_stats(self.handle, which, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value
