"""Device-resident graph handle: the engine's replacement for SNAP's PUNGraph.

``load_edge_list(path)`` replaces ``snap.LoadEdgeList(snap.PUNGraph, path, 0, 1)``
(similarity.py:16). The graph is the undirected simple graph of the edge list:

* node ids are the integers of graph.txt (SNAP TInt); they are remapped to dense ids
  ``0..n-1`` -- nodes seen in column 0 first (ascending), then the column-1-only nodes --
  so a reference bipartite file puts users in one contiguous range and businesses in
  another (``dataset_maker.py:197`` writes "user business");
* duplicate / reversed edges are merged; a self-loop is not stored in the CSR (it never
  changes a BFS hop set) but adds 1 to the node's SNAP degree (TUNGraph stores it once);
* the CSR (both directions, sorted rows) and the per-node Adamic-Adar weight
  ``(log deg)^-1`` (0 for deg <= 1, similarity.py:121-125) live in HBM. The weights are
  computed here with Python's ``math.log`` -- the reference's own arithmetic -- once per
  distinct degree.
"""
import ctypes
import math
import os
import weakref

import numpy as np

from . import _lib
from ._lib import check, lib, ptr

_I64P = ctypes.POINTER(ctypes.c_int64)
_lib.register("blp_edges_load", [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)])
_lib.register("blp_edges_info", [ctypes.c_void_p, _I64P, _I64P, _I64P, _I64P, _I64P])
_lib.register("blp_edges_fetch", [ctypes.c_void_p] * 7)
_lib.register("blp_edges_destroy", [ctypes.c_void_p])
_lib.register("blp_edges_load_device", [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_void_p)])
_lib.register("blp_edges_device", [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)])
_lib.register("blp_edges_csr", [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)])
_lib.register("blp_ids_lookup", [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                 ctypes.c_void_p])


def parse_edge_list(path, c0=0, c1=1):
    """graph.txt -> (a, b) int64 arrays (SNAP LoadEdgeList text semantics)."""
    L = lib()
    m = ctypes.c_int64(0)
    bpath = path.encode() if isinstance(path, str) else path
    check(L.blp_edges_parse(bpath, c0, c1, None, None, ctypes.byref(m)))
    a = np.empty(m.value, np.int64)
    b = np.empty(m.value, np.int64)
    check(L.blp_edges_parse(bpath, c0, c1, ptr(a), ptr(b), ctypes.byref(m)))
    return a[: m.value], b[: m.value]


def aa_weights_from_degree(deg):
    """Per-node Adamic-Adar term with the reference's arithmetic (similarity.py:121-125)."""
    deg = np.asarray(deg)
    out = np.zeros(len(deg), np.float64)
    if len(deg) == 0:
        return out
    dmax = int(deg.max())
    if int(deg.min()) >= 0 and dmax <= max(4 * len(deg), 1 << 20):  # one table over 0..max degree
        table = np.zeros(dmax + 1, np.float64)
        for d in np.flatnonzero(np.bincount(deg)):
            table[d] = (math.log(int(d)) ** -1) if d > 1 else 0.0
        return table[deg]
    uniq, inv = np.unique(deg, return_inverse=True)
    table = np.array([(math.log(int(d)) ** -1) if d > 1 else 0.0 for d in uniq], np.float64)
    return table[inv]


def _unique(x):
    """np.unique(x) for an int64 array; one presence table instead of a sort when the id span
    is compact (graph.txt ids usually are)."""
    if len(x) == 0:
        return np.unique(x)
    lo, hi = int(x.min()), int(x.max())
    if hi - lo + 1 > max(4 * len(x), 1 << 20):
        return np.unique(x)
    seen = np.zeros(hi - lo + 1, bool)
    seen[x - lo] = True
    return np.flatnonzero(seen).astype(np.int64) + lo


class HostGraph:
    """Host half of the graph: id map, CSR, SNAP degrees, Adamic-Adar weights.

    Needs libblp.so's host helpers only (no GPU), so the id/CSR logic is testable on a
    CPU-only machine. :class:`DeviceGraph` adds the HBM copy and the kernels.
    """

    def __init__(self, a_ids, b_ids, aa=True):
        a_ids = np.asarray(a_ids, dtype=np.int64)
        b_ids = np.asarray(b_ids, dtype=np.int64)
        if len(a_ids) != len(b_ids):
            raise ValueError("edge endpoint arrays differ in length")
        da, db = self._ids(a_ids, b_ids)
        self._host_csr(da, db, aa)

    def _host_csr(self, da, db, aa):
        """The CSR of the dense edge list on the host (blp_csr_from_edges)."""
        rp = np.zeros(self.n + 1, np.int64)
        ci = np.empty(max(2 * len(da), 1), np.int32)
        sl = np.zeros(max(self.n, 1), np.uint8)
        nnz = ctypes.c_int64(0)
        check(lib().blp_csr_from_edges(self.n, len(da), ptr(da), ptr(db), ptr(rp), ptr(ci), ptr(sl),
                                       ctypes.byref(nnz)))
        self._set_csr(rp, ci[: nnz.value].copy(), sl[: self.n], aa)

    def _set_ids(self, node_ids, n_col0, id_lo, id_map, n_edges_in):
        """The id map as blp_edges_load built it natively (same order as _ids): a dense table
        id_map[id - id_lo] answers every lookup."""
        self.node_ids = node_ids
        self.n_col0 = int(n_col0)
        self.n = len(node_ids)
        self._id_lo = int(id_lo)
        self._id_map = id_map
        self.n_edges_in = n_edges_in

    @property
    def _sort(self):  # dense ids in original-id order (the searchsorted lookup of sparse id spaces)
        if getattr(self, "_sort_", None) is None:
            self._sort_ = np.argsort(self.node_ids, kind="stable")
        return self._sort_

    @_sort.setter
    def _sort(self, v):
        self._sort_ = v

    @property
    def _sorted_ids(self):
        if getattr(self, "_sorted_ids_", None) is None:
            self._sorted_ids_ = self.node_ids[self._sort]
        return self._sorted_ids_

    @_sorted_ids.setter
    def _sorted_ids(self, v):
        self._sorted_ids_ = v

    def _ids(self, a_ids, b_ids):
        """The id map (dense ids: column-0 ids ascending, then the other ids ascending) and the
        edge list over dense ids."""
        u0 = _unique(a_ids)
        u1 = np.setdiff1d(_unique(b_ids), u0, assume_unique=True)
        self.node_ids = np.concatenate([u0, u1])  # dense id -> original id
        self.n_col0 = len(u0)  # dense ids [0, n_col0) appear in column 0 (users of a graph.txt)
        self.n = len(self.node_ids)
        if self.n >= 2**31 - 1:
            raise ValueError("too many nodes for int32 dense ids")
        self._sort = np.argsort(self.node_ids, kind="stable")
        self._sorted_ids = self.node_ids[self._sort]
        self.n_edges_in = len(a_ids)
        return self.dense(a_ids), self.dense(b_ids)

    def _set_csr(self, rp, ci, sl, aa):
        self.row_ptr = rp
        self.col_idx = ci
        self.self_loop = sl
        self.hop1_size = np.diff(rp)  # |GetNodesAtHop(v, 1)|
        self.degree = self.hop1_size + self.self_loop  # SNAP GetDeg
        self.aa_weight = aa_weights_from_degree(self.degree) if aa else None

    @classmethod
    def from_csr(cls, row_ptr, col_idx, self_loop, n_col0, aa=True):
        """A graph whose node ids are already dense (id i = dense id i): the CSR of
        blp_csr_from_edges(_device), e.g. built on the GPU after the multi-GPU exchange."""
        g = cls.__new__(cls)
        g.n = len(row_ptr) - 1
        g.node_ids = np.arange(g.n, dtype=np.int64)
        g.n_col0 = int(n_col0)
        g._sort = g.node_ids
        g._sorted_ids = g.node_ids
        g.n_edges_in = None
        g._set_csr(np.asarray(row_ptr, np.int64), np.asarray(col_idx, np.int32), np.asarray(self_loop, np.uint8), aa)
        return g

    @property
    def nnz(self):
        return int(self.row_ptr[-1])

    @property
    def col_idx(self):
        """Column ids of the CSR (int32, nnz). A graph adopted from a device CSR fetches them on
        first access (similarity.main never does: its scoring plans on the device)."""
        ci = self.__dict__.get("_col_idx")
        if ci is None:
            ci = self._col_idx = self._fetch_col_idx()
        return ci

    @col_idx.setter
    def col_idx(self, v):
        self._col_idx = v

    def _fetch_col_idx(self):
        raise AttributeError("col_idx")

    # ------------------------------------------------------------------ ids
    def lookup(self, ids):
        """original ids -> (dense ids, present mask); absent ids map to -1."""
        ids = np.asarray(ids, dtype=np.int64)
        if self.n == 0:
            return np.full(len(ids), -1, np.int32), np.zeros(len(ids), bool)
        if getattr(self, "_id_map", None) is not None:  # native table lookup (multi-threaded)
            ids = np.ascontiguousarray(ids)
            dense = np.empty(len(ids), np.int32)
            check(lib().blp_ids_lookup(ptr(self._id_map), self._id_lo, len(self._id_map), ptr(ids), len(ids),
                                       ptr(dense)))
            return dense, dense >= 0
        lo, span = int(self._sorted_ids[0]), int(self._sorted_ids[-1]) - int(self._sorted_ids[0]) + 1
        if span <= max(4 * self.n, 1 << 20):  # compact id space: one direct table gather
            tab = getattr(self, "_direct", None)
            if tab is None:
                tab = self._direct = np.full(span, -1, np.int32)
                tab[self._sorted_ids - lo] = self._sort
            off = ids - lo
            ok = (off >= 0) & (off < span)
            dense = np.where(ok, tab[np.where(ok, off, 0)], -1).astype(np.int32)
            return dense, dense >= 0
        pos = np.searchsorted(self._sorted_ids, ids)
        pos = np.minimum(pos, self.n - 1)
        present = self._sorted_ids[pos] == ids
        dense = np.where(present, self._sort[pos], -1).astype(np.int32)
        return dense, present

    def dense(self, ids):
        d, ok = self.lookup(ids)
        if not ok.all():
            raise KeyError("node id not in graph")
        return d

    def __contains__(self, node_id):
        return bool(self.lookup([int(node_id)])[1][0])

    def GetNodes(self):  # SNAP-style accessors used by the reference's drivers
        return self.n

    def GetEdges(self):
        return int(self.nnz // 2 + self.self_loop.sum())

    def GetDeg(self, node_id):
        return int(self.degree[self.dense([int(node_id)])[0]])


class DeviceGraph(HostGraph):
    """Undirected simple graph in HBM (CSR over dense ids) + the id map on the host.

    Mirrors the pieces of SNAP's PUNGraph the reference uses: node membership
    (``int(u) in nodes``, similarity.py:22,26,38,52), degree (``GetNI(i).GetDeg()``,
    :121) and the hop sets (:29,:41,:74,:85), which the kernels compute on the device.
    """

    def __init__(self, a_ids, b_ids, device=0, aa=True):
        a_ids = np.asarray(a_ids, dtype=np.int64)
        b_ids = np.asarray(b_ids, dtype=np.int64)
        if len(a_ids) != len(b_ids):
            raise ValueError("edge endpoint arrays differ in length")
        import time

        t0 = time.perf_counter()
        da, db = self._ids(a_ids, b_ids)
        self._build(da, db, device, aa)
        self.build_times["id_map_s"] = time.perf_counter() - t0 - self.build_times.get("total_s", 0.0)

    def _build(self, da, db, device, aa):
        """CSR + graph handle from dense endpoints (the id map is set)."""
        import time

        t0 = time.perf_counter()
        if len(da) == 0 or len(da) < int(os.environ.get("BLP_DEVICE_CSR_MIN", 1 << 16)):
            self._host_csr(da, db, aa)
            self._upload(device, aa)
            self.build_times = {"total_s": time.perf_counter() - t0}
            return
        # large edge lists: the CSR is built on the device (blp_csr_build_host: upload, radix
        # sort of the directed (row, col) keys, unique) and the host mirror fetched back --
        # the same CSR as blp_csr_from_edges (tests/test_gpu_ingest.py)
        c = ctypes.c_void_p()
        check(lib().blp_csr_build_host(device, ptr(da), ptr(db), len(da), self.n, ctypes.byref(c)))
        t1 = time.perf_counter()
        self._adopt_csr(c, device, aa)
        self.build_times.update({"device_csr_s": t1 - t0, "total_s": time.perf_counter() - t0})

    @classmethod
    def from_dense(cls, da, db, node_ids, n_col0, id_lo, id_map, device=0, aa=True):
        """A graph from dense endpoints plus the id map blp_edges_load built natively."""
        g = cls.__new__(cls)
        g._set_ids(node_ids, n_col0, id_lo, id_map, len(da))
        g._build(da, db, device, aa)
        return g

    @classmethod
    def from_edges_handle(cls, h, node_ids, n_col0, id_lo, id_map, m, device=0, aa=True):
        """A graph from a blp_edges handle whose dense endpoints are already in HBM
        (blp_edges_load_device): blp_edges_csr builds the CSR from them, no upload."""
        import time

        g = cls.__new__(cls)
        g._set_ids(node_ids, n_col0, id_lo, id_map, m)
        t0 = time.perf_counter()
        c = ctypes.c_void_p()
        check(lib().blp_edges_csr(h, device, ctypes.byref(c)))
        t1 = time.perf_counter()
        g._adopt_csr(c, device, aa)
        g.build_times.update({"device_csr_s": t1 - t0, "total_s": time.perf_counter() - t0})
        return g

    @classmethod
    def from_csr(cls, row_ptr, col_idx, self_loop, n_col0, device=0, aa=True):
        g = HostGraph.from_csr.__func__(cls, row_ptr, col_idx, self_loop, n_col0, aa)
        g._upload(device, aa)
        return g

    @classmethod
    def from_device_edges(cls, a_ptr, b_ptr, m, n, n_col0, device=0, aa=True):
        """The multi-GPU ingest path (blp.dist.allgather_edges): build the CSR on `device` from
        device-resident int32 endpoints (m edges, dense ids in [0, n)) and keep it there
        (blp_csr_build_device -> blp_graph_create_from_csr: no host-to-device upload). The host
        half (id map, degrees, Adamic-Adar weights with the reference's math.log) comes from
        one device-to-host copy of the CSR, which the handle borrows as its planning mirror.
        ``build_times`` records the phases."""
        import time

        t0 = time.perf_counter()
        c = ctypes.c_void_p()
        check(lib().blp_csr_build_device(device, ctypes.c_void_p(a_ptr), ctypes.c_void_p(b_ptr), m, n,
                                         ctypes.byref(c)))
        t_csr = time.perf_counter() - t0
        g = cls.from_csr_handle(c, n, n_col0, device, aa)
        g.build_times["device_csr_s"] = t_csr
        return g

    @classmethod
    def from_csr_handle(cls, c, n, n_col0, device=0, aa=True):
        """A graph over a device CSR handle (blp_csr_build_device / blp_multi_gather_csr output,
        dense ids in [0, n)); the handle is consumed."""
        g = cls.__new__(cls)
        g.node_ids = np.arange(n, dtype=np.int64)  # ids already dense
        g.n_col0 = int(n_col0)
        g._sort = g.node_ids
        g._sorted_ids = g.node_ids
        g.n_edges_in = None
        g._adopt_csr(c, device, aa)
        return g

    def _adopt_csr(self, c, device, aa):
        """Host half from one device-to-host copy of the device CSR `c`, then the graph handle
        over it (blp_graph_create_from_csr, which consumes `c` and borrows the host mirror)."""
        import time

        L = lib()
        t = {}
        try:
            nn, nnz = ctypes.c_int64(), ctypes.c_int64()
            check(L.blp_csr_info(c, ctypes.byref(nn), ctypes.byref(nnz)))
            n = nn.value
            t0 = time.perf_counter()
            # row offsets and self-loop flags only: the column ids stay in HBM (col_idx fetches
            # them on first access; the handle's own planning runs on the device)
            rp = np.empty(n + 1, np.int64)
            sl = np.empty(max(n, 1), np.uint8)
            check(L.blp_csr_fetch(c, ptr(rp), None, ptr(sl)))
            t["fetch_s"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            self.n = n
            self._set_csr(rp, None, sl[:n], aa)
            t["host_half_s"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            h = ctypes.c_void_p()
            check(L.blp_graph_create_from_csr(c, ptr(self.row_ptr), None, ptr(self.aa_weight) if aa else None,
                                              ctypes.byref(h)))
            c = None  # consumed
            t["graph_create_s"] = time.perf_counter() - t0
        finally:
            if c is not None:
                L.blp_csr_destroy(c)
        self.device = device
        self.handle = h
        self.build_times = t

    def _fetch_col_idx(self):
        ci = np.empty(max(self.nnz, 1), np.int32)
        check(lib().blp_graph_col_idx(self.handle, ptr(ci)))
        return ci[: self.nnz]

    def _upload(self, device, aa):
        self.device = device
        h = ctypes.c_void_p()
        check(lib().blp_graph_create(ptr(self.row_ptr), ptr(self.col_idx), self.n,
                                     ptr(self.aa_weight) if aa else None, device, ctypes.byref(h)))
        self.handle = h

    @property
    def aa_shift(self):
        """Fixed-point scale (2^-shift) of the Adamic-Adar sums (blp_graph_aa_shift)."""
        v = ctypes.c_int(0)
        check(lib().blp_graph_aa_shift(self.handle, ctypes.byref(v)))
        return v.value

    # ------------------------------------------------------------------ lifecycle
    def _adopt(self, child):
        """Register a handle built on this graph (a pair batch, a top-k engine): it is closed
        before the graph's own handle, whatever order Python collects them in."""
        kids = self.__dict__.setdefault("_children", weakref.WeakSet())
        kids.add(child)

    def close(self):
        for child in list(self.__dict__.get("_children", ())):
            child.close()
        if getattr(self, "handle", None):
            lib().blp_graph_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ scoring
    def score_pairs(self, x, y, mask=7):
        """Pairs (x, y) of dense ids -> dict(cn, jaccard, adamic) arrays (caller order).

        x is the node whose exact 2-hop set is built (user side: user; business side:
        business), y the node whose 1-hop set is intersected with it."""
        x = _lib.as_i32(x)
        y = _lib.as_i32(y)
        n = len(x)
        cn = np.zeros(n, np.uint32)
        jac = np.zeros(n, np.float64) if mask & _lib.JACCARD else None
        aa = np.zeros(n, np.float64) if mask & _lib.ADAMIC else None
        if n:
            check(lib().blp_score_pairs(self.handle, 0, mask | _lib.CN, ptr(x), ptr(y), n, ptr(cn), ptr(jac),
                                        ptr(aa)))
        return {"cn": cn, "jaccard": jac, "adamic": aa}

    def batch(self, x, y):
        return PairBatch(self, x, y)

    def batch_pair(self, x, y):
        """(PairBatch(x, y), PairBatch(y, x)): similarity.main's two passes over one pair list
        with ONE upload of the pairs (blp_batch_create_pair)."""
        return PairBatch.pair(self, x, y)

    def score_batches(self, items):
        """Enqueue several batches of this graph as one concurrent step (blp_batches_score).
        items: [(PairBatch, mask), ...]; returns at once, fetch() waits."""
        n = len(items)
        hs = (ctypes.c_void_p * max(n, 1))(*[b.handle for b, _ in items])
        ms = (ctypes.c_uint32 * max(n, 1))(*[int(m) for _, m in items])
        check(lib().blp_batches_score(self.handle, n, hs, ms))

    def hop3_sample(self, src, pos_off=None, pos_y=None, rate=0.01, seed=0):
        """Exact-distance-3 candidates of each source, sampled (dataset_maker.py:137-144).

        src: dense source ids; pos_off/pos_y: CSR of each source's held-out positives
        (dense ids). Returns (x, y, label) arrays, grouped by source in `src` order;
        within a source: positives first, then kept negatives by ascending dense id."""
        src = _lib.as_i32(src)
        ns = len(src)
        if pos_off is None:
            pos_off = np.zeros(ns + 1, np.int32)
            pos_y = np.zeros(1, np.int32)
        pos_off = _lib.as_i32(pos_off)
        pos_y = _lib.as_i32(pos_y if len(pos_y) else np.zeros(1, np.int32))
        cap = max(1024, int(ns * 64))
        while True:
            ox = np.empty(cap, np.int32)
            oy = np.empty(cap, np.int32)
            ol = np.empty(cap, np.uint8)
            n_out = ctypes.c_int64(0)
            check(lib().blp_hop3_sample(self.handle, ptr(src), ns, ptr(pos_off), ptr(pos_y), float(rate),
                                        int(seed) & (2**64 - 1), ptr(ox), ptr(oy), ptr(ol), cap,
                                        ctypes.byref(n_out)))
            if n_out.value <= cap:
                break
            cap = int(n_out.value)
        n = n_out.value
        ox, oy, ol = ox[:n], oy[:n], ol[:n]
        # deterministic order: by source position, keeping each source's emission order
        rank = np.empty(self.n, np.int64)
        rank[src] = np.arange(ns)
        order = np.argsort(rank[ox], kind="stable")
        return ox[order], oy[order], ol[order]

    def stats(self, kernel):
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        check(lib().blp_stats_get(self.handle, kernel, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def stats_reset(self):
        check(lib().blp_stats_reset(self.handle))

    def sync(self):
        check(lib().blp_graph_sync(self.handle))


class PairBatch:
    """Pairs resident in HBM for repeated scoring (bench); see blp_batch_* in blp.h."""

    def __init__(self, graph, x, y):
        self.graph = graph
        self.x = _lib.as_i32(x)
        self.y = _lib.as_i32(y)
        self.n = len(self.x)
        h = ctypes.c_void_p()
        check(lib().blp_batch_create(graph.handle, ptr(self.x), ptr(self.y), self.n, ctypes.byref(h)))
        self.handle = h
        graph._adopt(self)

    @classmethod
    def pair(cls, graph, x, y):
        xs, ys = _lib.as_i32(x), _lib.as_i32(y)
        if len(xs) != len(ys):
            raise ValueError("pair arrays differ in length")
        h1, h2 = ctypes.c_void_p(), ctypes.c_void_p()
        check(lib().blp_batch_create_pair(graph.handle, ptr(xs), ptr(ys), len(xs), ctypes.byref(h1), ctypes.byref(h2)))
        out = []
        for h, (a, b) in ((h1, (xs, ys)), (h2, (ys, xs))):
            bt = cls.__new__(cls)
            bt.graph, bt.x, bt.y, bt.n, bt.handle = graph, a, b, len(a), h
            graph._adopt(bt)
            out.append(bt)
        return tuple(out)

    def plan(self):
        lo, hi = ctypes.c_int64(), ctypes.c_int64()
        ch, blk, hv = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().blp_batch_plan(self.handle, ctypes.byref(lo), ctypes.byref(hi), ctypes.byref(ch),
                                   ctypes.byref(blk), ctypes.byref(hv)))
        ns, nh, runs, wbm = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int(), ctypes.c_int()
        check(lib().blp_batch_routes(self.handle, ctypes.byref(ns), ctypes.byref(nh), ctypes.byref(runs),
                                     ctypes.byref(wbm)))
        return {"lo": lo.value, "hi": hi.value, "chunks": ch.value, "block": blk.value, "heavy": hv.value,
                "sources": ns.value, "hash_sources": nh.value, "runs": bool(runs.value),
                "wedge_bitmaps": bool(wbm.value)}

    def score(self, mask=7):
        check(lib().blp_batch_score(self.graph.handle, self.handle, mask))

    def kernel(self, mask=7):
        """The scorer kernel's template instance, as rocprofv3 names it (blp_batch_kernel)."""
        buf = ctypes.create_string_buffer(128)
        check(lib().blp_batch_kernel(self.handle, mask, buf, len(buf)))
        return buf.value.decode()

    def stats(self, which=0):
        """(total ms, launches) of this batch's scorer (0) or grouping (1) kernels."""
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        check(lib().blp_batch_stats(self.handle, which, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def stats_reset(self):
        check(lib().blp_batch_stats_reset(self.handle))

    def fetch(self, mask=7):
        # every entry is written by the copy (huge-page host memory: _lib.host_empty)
        cn = _lib.host_empty(self.n, np.uint32)
        jac = _lib.host_empty(self.n, np.float64) if mask & _lib.JACCARD else None
        aa = _lib.host_empty(self.n, np.float64) if mask & _lib.ADAMIC else None
        check(lib().blp_batch_fetch(self.graph.handle, self.handle, ptr(cn), ptr(jac), ptr(aa)))
        return {"cn": cn, "jaccard": jac, "adamic": aa}

    def fetch_repr(self, which, zero_int=False):
        """The Jaccard (which = JACCARD) or Adamic-Adar (ADAMIC) scores as json.dumps text,
        formatted on the device: uint8[n, 24], NUL-padded slots (blp_batch_fetch_repr)."""
        out = _lib.host_empty((self.n, 24), np.uint8)
        check(lib().blp_batch_fetch_repr(self.graph.handle, self.handle, which, int(bool(zero_int)), ptr(out)))
        return out

    def close(self):
        if getattr(self, "handle", None):
            lib().blp_batch_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load_edge_list(path, c0=0, c1=1, device=0):
    """snap.LoadEdgeList(snap.PUNGraph, path, c0, c1) -> DeviceGraph (similarity.py:16).

    The file is parsed once and, for a compact id space, mapped to dense ids natively: on the
    device when it has the reference's own line shape (blp_edges_load_device, the dense
    endpoints stay in HBM for the CSR build), else on the host (multi-threaded); a sparse id
    space goes through HostGraph._ids."""
    import time

    t0 = time.perf_counter()
    L = lib()
    h = ctypes.c_void_p()
    bpath = path.encode() if isinstance(path, str) else path
    check(L.blp_edges_load_device(bpath, c0, c1, device, ctypes.byref(h)))
    try:
        m, n, n0, lo, span = (ctypes.c_int64() for _ in range(5))
        check(L.blp_edges_info(h, *(ctypes.byref(v) for v in (m, n, n0, lo, span))))
        on = ctypes.c_int(-1)
        check(L.blp_edges_device(h, ctypes.byref(on)))
        if span.value > 0 and on.value >= 0:
            node_ids = np.empty(n.value, np.int64)
            id_map = np.empty(span.value, np.int32)
            check(L.blp_edges_fetch(h, None, None, None, None, ptr(node_ids), ptr(id_map)))
            t1 = time.perf_counter()
            G = DeviceGraph.from_edges_handle(h, node_ids, n0.value, lo.value, id_map, m.value, device=device)
        elif span.value > 0:
            da = np.empty(m.value, np.int32)
            db = np.empty(m.value, np.int32)
            node_ids = np.empty(n.value, np.int64)
            id_map = np.empty(span.value, np.int32)
            check(L.blp_edges_fetch(h, None, None, ptr(da), ptr(db), ptr(node_ids), ptr(id_map)))
            t1 = time.perf_counter()
            G = DeviceGraph.from_dense(da, db, node_ids, n0.value, lo.value, id_map, device=device)
        else:
            a = np.empty(m.value, np.int64)
            b = np.empty(m.value, np.int64)
            check(L.blp_edges_fetch(h, ptr(a), ptr(b), None, None, None, None))
            t1 = time.perf_counter()
            G = DeviceGraph(a, b, device=device)
    finally:
        L.blp_edges_destroy(h)
    G.build_times["parse_and_id_map_s"] = t1 - t0
    return G


LoadEdgeList = load_edge_list
