"""Native score-file I/O for similarity.main (csrc/scorefile.hip; include/blp.h).

``Examples.load(path)`` parses examples.json into flat per-pair id arrays (or returns None
when the file is not of the reference's simple shape -- the caller then uses json.loads);
``Examples.write(path, kind, present, values)`` writes one score file with exactly the text
``json.dumps`` gives for the same nested dict (util.py:18-21)."""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, host_empty, lib, ptr

_P = ctypes.c_void_p
_I64P = ctypes.POINTER(ctypes.c_int64)
_lib.register("blp_examples_parse", [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)])
_lib.register("blp_examples_info", [_P, _I64P, _I64P])
_lib.register("blp_examples_ids", [_P, _P, _P, _P])
_lib.register("blp_examples_destroy", [_P])
_lib.register("blp_scores_write", [_P, ctypes.c_char_p, ctypes.c_int, _P, _P, ctypes.c_int64])

U32, F64, F64_INT0, NONE, REPR24 = 0, 1, 2, 3, 4  # BLP_SCORE_* (blp.h)
E_UNSUP = -4


class Examples:
    """examples.json as flat arrays: pair_user / pair_business (int of the keys, file order)
    and user_off (pair offsets per user)."""

    def __init__(self, handle):
        self.handle = handle
        nu, npairs = ctypes.c_int64(0), ctypes.c_int64(0)
        check(lib().blp_examples_info(handle, ctypes.byref(nu), ctypes.byref(npairs)))
        self.n_users, self.n_pairs = nu.value, npairs.value
        self.pair_user = host_empty(self.n_pairs, np.int64)
        self.pair_business = host_empty(self.n_pairs, np.int64)
        self.user_off = np.empty(self.n_users + 1, np.int64)
        check(lib().blp_examples_ids(handle, ptr(self.pair_user), ptr(self.pair_business), ptr(self.user_off)))

    @classmethod
    def load(cls, path):
        h = ctypes.c_void_p()
        rc = lib().blp_examples_parse(str(path).encode(), ctypes.byref(h))
        if rc == E_UNSUP:
            return None
        check(rc)
        return cls(h)

    def write(self, path, kind, present=None, values=None):
        """One score file; values hold one entry per present pair (uint32 for U32, a row of the
        uint8[n, 24] slots of PairBatch.fetch_repr for REPR24, float64 else)."""
        pres = None if present is None else np.ascontiguousarray(present, np.uint8)
        if kind == NONE:
            vals, n = None, 0
        elif kind == REPR24:
            vals = np.ascontiguousarray(values, np.uint8)
            if vals.ndim != 2 or vals.shape[1] != 24:
                raise ValueError("REPR24 values must be uint8[n, 24] slots")
            n = len(vals)
        else:
            vals = np.ascontiguousarray(values, np.uint32 if kind == U32 else np.float64)
            n = len(vals)
        check(lib().blp_scores_write(self.handle, str(path).encode(), kind, ptr(pres), ptr(vals), n))

    def close(self):
        if self.handle:
            lib().blp_examples_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def format_repr(values, zero_int=False):
    """repr(v) of each double as uint8[n, 24] slots, formatted on the host by the same code the
    device runs (blp_repr_format; csrc/repr.h)."""
    v = np.ascontiguousarray(values, np.float64)
    out = np.zeros((len(v), 24), np.uint8)
    check(lib().blp_repr_format(ptr(v), len(v), int(bool(zero_int)), ptr(out)))
    return out


def slot_strings(slots):
    """The text of each 24-byte slot (tests)."""
    return [bytes(r).rstrip(b"\0").decode() for r in np.asarray(slots, np.uint8)]
