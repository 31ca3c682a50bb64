"""The engine's own multi-GPU exchange (csrc/multi.hip, blp_multi_*): config 5's row-block
sharded ingest through libblp's RCCL communicator instead of
torch.distributed (blp/dist.py). One process per GPU; rank 0 makes the id
(``Multi.unique_id()``) and ships its bytes to the other ranks over any channel.

    m = Multi(uid, world, rank, device)
    G = m.gather_graph(a_local, b_local, n, n_col0)   # ONE RCCL all-gather, CSR built in HBM
    t_max = m.allreduce(t_local, "max")
"""
import ctypes
import time

import numpy as np

from ._lib import check, lib

ID_BYTES = 128
_OPS = {"sum": 0, "max": 1}


class Multi:
    def __init__(self, uid, world, rank, device=0):
        uid = bytes(uid)
        if len(uid) != ID_BYTES:
            raise ValueError("communicator id must be %d bytes" % ID_BYTES)
        self.world, self.rank, self.device = int(world), int(rank), int(device)
        self._id = (ctypes.c_uint8 * ID_BYTES).from_buffer_copy(uid)
        self._h = ctypes.c_void_p()
        check(lib().blp_multi_init(self._id, self.world, self.rank, self.device, ctypes.byref(self._h)))
        self.bytes_in = 0
        self.seconds = None

    @staticmethod
    def unique_id():
        buf = (ctypes.c_uint8 * ID_BYTES)()
        check(lib().blp_multi_unique_id(buf))
        return bytes(buf)

    def gather_csr(self, a, b, n, m=None):
        """The exchange: this rank's edge partial -- int32 numpy arrays, or device pointers with
        the edge count m -- all-gathered over RCCL; returns the union's device CSR handle."""
        if m is None:
            a = np.ascontiguousarray(a, np.int32)
            b = np.ascontiguousarray(b, np.int32)
            if len(a) != len(b):
                raise ValueError("endpoint arrays differ in length")
            m, pa, pb = len(a), a.ctypes.data, b.ctypes.data
        else:
            pa, pb = int(a), int(b)
        c = ctypes.c_void_p()
        got = ctypes.c_int64()
        t0 = time.perf_counter()
        check(lib().blp_multi_gather_csr(self._h, ctypes.c_void_p(pa), ctypes.c_void_p(pb), int(m), int(n),
                                         ctypes.byref(c), ctypes.byref(got)))
        self.seconds = time.perf_counter() - t0
        self.bytes_in = got.value
        return c

    @staticmethod
    def compact_csr(recv, counts, n, device=0):
        """The post-gather half of the exchange (blp_multi_compact_csr): recv is an all-gather
        receive buffer -- an int32 numpy array, or a device pointer -- of len(counts) slots
        [a | b], each half padded to max(counts); returns (device CSR handle, bytes_in)."""
        cnt = np.ascontiguousarray(counts, np.int64)
        if isinstance(recv, np.ndarray):
            recv = np.ascontiguousarray(recv, np.int32)
            if recv.size < 2 * int(cnt.max(initial=0)) * len(cnt):
                raise ValueError("receive buffer smaller than the counts imply")
            p = recv.ctypes.data
        else:
            p = int(recv)
        c = ctypes.c_void_p()
        got = ctypes.c_int64()
        check(lib().blp_multi_compact_csr(int(device), ctypes.c_void_p(p), cnt.ctypes.data_as(ctypes.c_void_p),
                                          len(cnt), int(n), ctypes.byref(c), ctypes.byref(got)))
        return c, got.value

    @staticmethod
    def fetch_csr(c, destroy=True):
        """(row_ptr int64, col_idx int32) of a device CSR handle (blp_csr_fetch); the handle
        is destroyed afterwards unless destroy=False."""
        L = lib()
        try:
            nn, nnz = ctypes.c_int64(), ctypes.c_int64()
            check(L.blp_csr_info(c, ctypes.byref(nn), ctypes.byref(nnz)))
            rp = np.empty(nn.value + 1, np.int64)
            ci = np.empty(max(nnz.value, 1), np.int32)
            check(L.blp_csr_fetch(c, rp.ctypes.data_as(ctypes.c_void_p), ci.ctypes.data_as(ctypes.c_void_p), None))
            return rp, ci[: nnz.value]
        finally:
            if destroy:
                L.blp_csr_destroy(c)

    def gather_graph(self, a, b, n, n_col0, m=None, aa=True):
        """gather_csr, then the graph handle over it (DeviceGraph.from_csr_handle)."""
        from .graph import DeviceGraph

        return DeviceGraph.from_csr_handle(self.gather_csr(a, b, n, m), n, n_col0, self.device, aa)

    def allreduce(self, v, op="max"):
        x = ctypes.c_double(float(v))
        check(lib().blp_multi_allreduce(self._h, ctypes.byref(x), _OPS[op]))
        return x.value

    def close(self):
        if self._h:
            lib().blp_multi_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
