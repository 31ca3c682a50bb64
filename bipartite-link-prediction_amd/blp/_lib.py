"""ctypes binding of libblp.so (include/blp.h). No torch, no fallback.

The library is built in-tree (``csrc/Makefile`` -> ``blp/libblp.so``, see
``__graft_entry__.build``). If it is missing or fails to load, every entry point of the
engine raises :class:`BLPUnavailable` -- there is deliberately no CPU path behind it.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BLP_LIB", os.path.join(_HERE, "libblp.so"))

CN, JACCARD, ADAMIC = 1, 2, 4
E_ZERODIV = -5

K_SCORE, K_GROUP, K_SVD_PAIRS, K_SVD_TOPK, K_WALK, K_HOP3 = range(6)


class BLPUnavailable(RuntimeError):
    """libblp.so (the HIP engine) is not built or cannot be loaded."""


class BLPError(RuntimeError):
    """A libblp call returned an error code."""

    def __init__(self, code, msg):
        super().__init__("%s (code %d)" % (msg, code))
        self.code = code


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int
_U32 = ctypes.c_uint32
_DP = ctypes.POINTER(ctypes.c_double)
_PP = ctypes.POINTER(ctypes.c_void_p)

# name -> argtypes (all return int unless listed in _RESTYPE)
SIGNATURES = {
    "blp_last_error": [],
    "blp_version": [],
    "blp_device_count": [ctypes.POINTER(ctypes.c_int)],
    "blp_device_sync": [_I32],
    "blp_stream_prewarm": [_I32, _I32],
    "blp_host_alloc": [ctypes.c_size_t, _PP],
    "blp_host_free": [_P, ctypes.c_size_t],
    "blp_edges_parse": [ctypes.c_char_p, _I32, _I32, _P, _P, ctypes.POINTER(ctypes.c_int64)],
    "blp_csr_from_edges": [_I64, _I64, _P, _P, _P, _P, _P, ctypes.POINTER(ctypes.c_int64)],
    "blp_csr_from_edges_device": [_I32, _P, _P, _I64, _I64, _P, _P, _P, ctypes.POINTER(ctypes.c_int64)],
    "blp_graph_create": [_P, _P, _I64, _P, _I32, _PP],
    "blp_csr_build_device": [_I32, _P, _P, _I64, _I64, _PP],
    "blp_csr_build_host": [_I32, _P, _P, _I64, _I64, _PP],
    "blp_csr_info": [_P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)],
    "blp_csr_fetch": [_P, _P, _P, _P],
    "blp_csr_destroy": [_P],
    "blp_graph_create_from_csr": [_P, _P, _P, _P, _PP],
    "blp_graph_destroy": [_P],
    "blp_multi_unique_id": [_P],
    "blp_multi_init": [_P, _I32, _I32, _I32, _PP],
    "blp_multi_info": [_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)],
    "blp_multi_gather_csr": [_P, _P, _P, _I64, _I64, _PP, ctypes.POINTER(ctypes.c_int64)],
    "blp_multi_allreduce": [_P, _DP, _I32],
    "blp_multi_destroy": [_P],
    "blp_multi_compact_csr": [_I32, _P, _P, _I32, _I64, _PP, ctypes.POINTER(ctypes.c_int64)],
    "blp_graph_wedge": [_P, ctypes.POINTER(ctypes.c_int64), _P, _P],
    "blp_graph_col_idx": [_P, _P],
    "blp_graph_info": [_P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                       ctypes.POINTER(ctypes.c_int)],
    "blp_graph_sync": [_P],
    "blp_graph_aa_shift": [_P, ctypes.POINTER(ctypes.c_int)],
    "blp_score_pairs": [_P, _I32, _U32, _P, _P, _I64, _P, _P, _P],
    "blp_batch_create": [_P, _P, _P, _I64, _PP],
    "blp_batch_create_pair": [_P, _P, _P, _I64, _PP, _PP],
    "blp_batch_score": [_P, _P, _U32],
    "blp_batches_score": [_P, _I32, _P, _P],
    "blp_batch_fetch": [_P, _P, _P, _P, _P],
    "blp_batch_fetch_repr": [_P, _P, _I32, _I32, _P],
    "blp_batch_kernel": [_P, _U32, _P, _I32],
    "blp_repr_format": [_P, _I64, _I32, _P],
    "blp_repr_format_device": [_I32, _P, _I64, _I32, _P],
    "blp_batch_destroy": [_P],
    "blp_batch_plan": [_P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                       ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                       ctypes.POINTER(ctypes.c_int)],
    "blp_batch_routes": [_P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int),
                         ctypes.POINTER(ctypes.c_int)],
    "blp_batch_stats": [_P, _I32, _DP, ctypes.POINTER(ctypes.c_int64)],
    "blp_batch_stats_reset": [_P],
    "blp_hop3_sample": [_P, _P, _I64, _P, _P, ctypes.c_double, ctypes.c_uint64, _P, _P, _P, _I64,
                        ctypes.POINTER(ctypes.c_int64)],
    "blp_stats_reset": [_P],
    "blp_stats_get": [_P, _I32, _DP, ctypes.POINTER(ctypes.c_int64)],
}
_RESTYPE = {"blp_last_error": ctypes.c_char_p, "blp_version": ctypes.c_char_p}

_lib = None


def lib():
    """Load libblp.so once; raise BLPUnavailable (loudly) if it cannot be loaded."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BLPUnavailable(
            "libblp.so not found at %s: build the HIP engine first "
            "(python -c 'import __graft_entry__ as g; g.build()')" % LIB_PATH)
    try:
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - depends on the box
        raise BLPUnavailable("cannot load %s: %s" % (LIB_PATH, e))
    for name, args in SIGNATURES.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = _RESTYPE.get(name, ctypes.c_int)
    _lib = L
    return L


def register(name, argtypes, restype=ctypes.c_int):
    """Add a signature for entry points defined by later translation units."""
    SIGNATURES[name] = argtypes
    if restype is not ctypes.c_int:
        _RESTYPE[name] = restype
    if _lib is not None:
        fn = getattr(_lib, name)
        fn.argtypes = argtypes
        fn.restype = restype


def check(rc):
    if rc != 0:
        msg = lib().blp_last_error().decode(errors="replace")
        if rc == E_ZERODIV:
            raise ZeroDivisionError("float division by zero")
        raise BLPError(rc, msg)
    return rc


def ptr(a):
    """Raw data pointer of a C-contiguous numpy array (None passes NULL)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return ctypes.c_void_p(a.ctypes.data)


def device_count():
    n = ctypes.c_int(0)
    check(lib().blp_device_count(ctypes.byref(n)))
    return n.value


def device_sync(device=0):
    check(lib().blp_device_sync(device))


def prewarm(device=0, streams=4):
    """Start the HIP runtime on `device` and fill the library's stream pool (blp_stream_prewarm):
    run on a spare thread while inputs load, so neither lands on the critical path."""
    check(lib().blp_device_sync(device))
    check(lib().blp_stream_prewarm(device, streams))


def host_empty(shape, dtype):
    """numpy.empty over blp_host_alloc: from 4 MiB on the memory is advised as transparent huge
    pages, so filling a fresh result array (a device-to-host fetch) and releasing it take a fault
    and an unmap per 2 MiB instead of per 4 KiB. Released with the last view of the array."""
    import weakref

    dt = np.dtype(dtype)
    shape = (int(shape),) if np.isscalar(shape) else tuple(int(s) for s in shape)
    nbytes = max(int(np.prod(shape, dtype=np.int64)) * dt.itemsize, 1)
    p = ctypes.c_void_p()
    check(lib().blp_host_alloc(nbytes, ctypes.byref(p)))
    buf = (ctypes.c_uint8 * nbytes).from_address(p.value)
    weakref.finalize(buf, lib().blp_host_free, ctypes.c_void_p(p.value), nbytes)
    n = int(np.prod(shape, dtype=np.int64))
    return np.frombuffer(buf, dtype=dt, count=n).reshape(shape)


def version():
    return lib().blp_version().decode()


def as_i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)
