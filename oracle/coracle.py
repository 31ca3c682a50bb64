"""ctypes wrapper for oracle/liboracle.so — TEST INFRASTRUCTURE ONLY (see oracle.c)."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        L.og_create.restype = P
        L.og_create.argtypes = [ctypes.c_int64, ctypes.c_int64, P, P]
        L.og_destroy.argtypes = [P]
        L.og_n.restype = ctypes.c_int64
        L.og_n.argtypes = [P]
        L.og_nnz.restype = ctypes.c_int64
        L.og_nnz.argtypes = [P]
        L.og_score_pairs.restype = ctypes.c_int
        L.og_score_pairs.argtypes = [P, ctypes.c_int64, P, P, ctypes.c_uint32, P, P, P, P, ctypes.c_int]
        L.og_csr.argtypes = [P, P, P]
        L.og_hop3.restype = ctypes.c_int64
        L.og_hop3.argtypes = [P, ctypes.c_int64, P, P, P, ctypes.c_int64]
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleGraph:
    """Dense-id undirected graph (ids 0..n-1) built from an edge list, SNAP semantics."""

    def __init__(self, n, a, b):
        self.a = np.ascontiguousarray(a, dtype=np.int32)
        self.b = np.ascontiguousarray(b, dtype=np.int32)
        self.n = int(n)
        self.h = lib().og_create(self.n, len(self.a), _p(self.a), _p(self.b))

    def __del__(self):
        if getattr(self, "h", None):
            lib().og_destroy(self.h)
            self.h = None

    def csr(self):
        """(row_ptr int64[n + 1], col_idx int32[nnz]): read-only views of the oracle's own CSR,
        valid while this graph lives."""
        L = lib()
        rp = ctypes.POINTER(ctypes.c_int64)()
        ci = ctypes.POINTER(ctypes.c_int32)()
        L.og_csr(self.h, ctypes.byref(rp), ctypes.byref(ci))
        nnz = int(L.og_nnz(self.h))
        r = np.ctypeslib.as_array(rp, (self.n + 1,))
        c = np.ctypeslib.as_array(ci, (max(nnz, 1),))[:nnz]
        r.flags.writeable = False
        c.flags.writeable = False
        return r, c

    def score_pairs(self, x, y, mask=7, nthreads=1):
        """-> (cn uint32, jaccard f64, adamic f64, |H2(x)| uint32) per pair."""
        x = np.ascontiguousarray(x, dtype=np.int32)
        y = np.ascontiguousarray(y, dtype=np.int32)
        n = len(x)
        cn = np.zeros(n, np.uint32)
        jac = np.zeros(n, np.float64)
        aa = np.zeros(n, np.float64)
        h2 = np.zeros(n, np.uint32)
        rc = lib().og_score_pairs(self.h, n, _p(x), _p(y), mask, _p(cn), _p(jac), _p(aa), _p(h2), nthreads)
        if rc:
            raise ZeroDivisionError("float division by zero")
        return cn, jac, aa, h2

    def hop3(self, users, with_members=True):
        users = np.ascontiguousarray(users, dtype=np.int32)
        counts = np.zeros(len(users), np.int64)
        total = lib().og_hop3(self.h, len(users), _p(users), _p(counts), None, 0)
        if not with_members:
            return counts, None
        out = np.zeros(max(total, 1), np.int32)
        lib().og_hop3(self.h, len(users), _p(users), _p(counts), _p(out), total)
        return counts, out[:total]
