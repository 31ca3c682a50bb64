"""Full-candidate top-k on the device (BASELINE.json configs[2]; blp_topk_* in blp.h).

For each source (user) every business at exact distance 3 -- the whole candidate set that
dataset_maker.py:139 samples from -- is scored with similarity.py's measures (:108-126)
and the k best per method are kept (score descending, then dense id ascending).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib, ptr

_P, _I64, _I32, _U32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_uint32
_PI64 = ctypes.POINTER(ctypes.c_int64)
_lib.register("blp_topk_create", [_P, _I64, _I64, _I64, _I64, ctypes.POINTER(ctypes.c_void_p)])
_lib.register("blp_topk_destroy", [_P])
_lib.register("blp_topk_info", [_P, _PI64, _PI64, _PI64, _PI64])
_lib.register("blp_topk_set_sources", [_P, _P, _I64])
_lib.register("blp_topk_run", [_P, _I32, _U32])
_lib.register("blp_topk_fetch", [_P, _U32, _P, _P, _P])
_lib.register("blp_topk_stats", [_P, _I32, ctypes.POINTER(ctypes.c_double), _PI64])
_lib.register("blp_topk_stats_reset", [_P])

METHOD_BITS = {"common_neighbors": _lib.CN, "jaccard": _lib.JACCARD, "adamic_adar": _lib.ADAMIC}


class TopK:
    """Top-k engine over a :class:`blp.DeviceGraph` whose file is a user->business edge list.

    side "user": sources are the column-0 nodes (users), targets the column-1-only nodes
    (businesses) -- the user-side orientation of similarity.users (similarity.py:20-61).
    side "business" swaps the roles (similarity.business's orientation, :63-106)."""

    def __init__(self, graph, side="user"):
        self.graph = graph
        n0 = graph.n_col0
        users, bus = (0, n0), (n0, graph.n)
        src, tgt = (users, bus) if side == "user" else (bus, users)
        h = ctypes.c_void_p()
        check(lib().blp_topk_create(graph.handle, src[0], src[1], tgt[0], tgt[1], ctypes.byref(h)))
        self.handle = h
        graph._adopt(self)
        self.src_range, self.tgt_range = src, tgt
        self.n_src = 0
        self.k = None
        self.mask = 0

    def info(self):
        a, b, c, d = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(lib().blp_topk_info(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c), ctypes.byref(d)))
        return {"chunks": a.value, "tier32": b.value, "tier16": c.value, "wedge_entries": d.value}

    def set_sources(self, src):
        self.src = _lib.as_i32(src)
        self.n_src = len(self.src)
        check(lib().blp_topk_set_sources(self.handle, ptr(self.src), self.n_src))

    def run(self, k=20, mask=_lib.JACCARD | _lib.ADAMIC):
        """Asynchronous on the graph's stream; fetch() waits."""
        check(lib().blp_topk_run(self.handle, int(k), int(mask)))
        self.k, self.mask = int(k), int(mask)

    def fetch(self, method):
        """-> (cols [n_src, k] dense ids (-1 past the end), scores [n_src, k], n_cand [n_src])."""
        bit = METHOD_BITS.get(method, method)
        cols = np.empty((self.n_src, self.k), np.int32)
        scores = np.empty((self.n_src, self.k), np.float64)
        ncand = np.empty(self.n_src, np.int64)
        check(lib().blp_topk_fetch(self.handle, int(bit), ptr(cols), ptr(scores), ptr(ncand)))
        return cols, scores, ncand

    def __call__(self, src, k=20, mask=_lib.JACCARD | _lib.ADAMIC):
        self.set_sources(src)
        self.run(k, mask)
        return {m: self.fetch(b) for m, b in METHOD_BITS.items() if mask & b}

    def stats(self, which=0):
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        check(lib().blp_topk_stats(self.handle, which, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def stats_reset(self):
        check(lib().blp_topk_stats_reset(self.handle))

    def close(self):
        if getattr(self, "handle", None):
            lib().blp_topk_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
