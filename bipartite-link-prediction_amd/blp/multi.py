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
