"""Python's repr(float) restated for the device (csrc/repr.h, the digits of json.dumps for a
score, util.py:18-21): the host build of the same function (blp_repr_format) against CPython's
repr on edge cases and random doubles; the GPU build against the host build. Host tests run
without a GPU."""
import json

import numpy as np
import pytest

import blp  # noqa: F401  (loads libblp.so)
from blp import scorefile


def _edge_values():
    v = [0.0, -0.0, 1.0, -1.0, 0.5, 0.1, 0.2, 0.3, 1 / 3, 2 / 3, 2.5, 1e-5, 1e-4, 0.0001234, 9.999999999999999e-05,
         1e15, 1e16, 1e17, 9999999999999998.0, 1e22, 1e23, 123456789012345678.0, 9007199254740992.0,
         5e-324, 1e-323, 2.2250738585072009e-308, 2.2250738585072014e-308, 1.7976931348623157e308, 1e100, 1.5e-100]
    v += [2.0 ** k for k in range(-1074, 1024)]
    v += [m * 2.0 ** -k for m in range(1, 64) for k in range(0, 64)]
    v += [float(i) for i in range(0, 20000, 3)]
    v += [c / u for u in range(1, 200) for c in range(0, u + 1)]  # Jaccard-like quotients
    v += [1.0 / np.log(d) for d in range(2, 5000)]  # Adamic-Adar terms
    return np.array(v, np.float64)


def _random_values(seed, n):
    rng = np.random.default_rng(seed)
    bits = np.frombuffer(rng.integers(0, 2 ** 64 - 1, n, dtype=np.uint64).tobytes(), np.float64)
    bits = bits[np.isfinite(bits)]
    short = rng.integers(1, 10 ** 6, n) / 10.0 ** rng.integers(0, 12, n)  # few digits: exact ties
    return np.concatenate([bits, short, rng.random(n), rng.random(n) * 10.0 ** rng.integers(-30, 30, n)])


@pytest.mark.parametrize("values", ["edge", "random"])
def test_host_repr_equals_cpython(values):
    v = _edge_values() if values == "edge" else _random_values(11, 100_000)
    got = scorefile.slot_strings(scorefile.format_repr(v))
    want = [repr(x) for x in v.tolist()]
    bad = [(x, a, b) for x, a, b in zip(v.tolist(), got, want) if a != b]
    assert not bad, bad[:5]


def test_repr_specials_and_zero_int():
    v = np.array([0.0, -0.0, 1.5, float("nan"), float("inf"), -float("inf")])
    assert scorefile.slot_strings(scorefile.format_repr(v)) == ["0.0", "-0.0", "1.5", "NaN", "Infinity", "-Infinity"]
    assert json.dumps(v.tolist())[1:-1].split(", ") == ["0.0", "-0.0", "1.5", "NaN", "Infinity", "-Infinity"]
    # adamic_adar's "nothing added" (similarity.py:118): 0.0 is the int 0
    assert scorefile.slot_strings(scorefile.format_repr(v[:3], zero_int=True)) == ["0", "0", "1.5"]


@pytest.mark.gpu
def test_device_repr_equals_host(gpu):
    import ctypes

    import torch

    from blp._lib import check, lib

    v = np.concatenate([_edge_values(), _random_values(12, 200_000)])
    for zero_int in (0, 1):
        dv = torch.from_numpy(v).cuda(gpu)
        dout = torch.zeros(len(v) * 24, dtype=torch.uint8, device=f"cuda:{gpu}")
        check(lib().blp_repr_format_device(gpu, ctypes.c_void_p(dv.data_ptr()), len(v), zero_int,
                                           ctypes.c_void_p(dout.data_ptr())))
        got = dout.cpu().numpy().reshape(-1, 24)
        want = scorefile.format_repr(v, zero_int=bool(zero_int))
        assert np.array_equal(got, want)
        if not zero_int:
            assert scorefile.slot_strings(got[:1000]) == [repr(x) for x in v[:1000].tolist()]
