"""Native score-file I/O (csrc/scorefile.hip) against json.loads / json.dumps: the parsed
examples equal the dict walk of similarity.py:22-32, and every written file is the exact text
util.write_json (util.py:18-21) produces for the same values -- floats in Python repr
(fixed/exponent switch, shortest digits), ints, the int 0 of similarity.py:118 and the
missing-node zeros of similarity.py:59-60 / 104-105. Host code only: runs without a GPU."""
import json
import math
import os
import struct

import numpy as np
import pytest

import blp  # noqa: F401  (loads libblp.so)
import similarity
from blp import scorefile


def _examples(rng, n_users=60, weird=True):
    ex = {}
    for i in range(n_users):
        u = str(int(rng.integers(0, 10**7)))
        if weird and i % 17 == 3:
            u = "0" + u  # int() accepts it; the key is kept byte for byte
        if u in ex:
            continue
        inner = {}
        for _ in range(int(rng.integers(0, 40))):
            b = str(int(rng.integers(10**7, 10**7 + 5000)))
            if weird and rng.random() < 0.02:
                b = "+" + b
            inner[b] = int(rng.random() < 0.1)
        ex[u] = inner
    return ex


def _write(tmp_path, ex):
    p = str(tmp_path / "examples.json")
    with open(p, "w") as f:
        f.write(json.dumps(ex))
    return p


def _odd_doubles(rng, n):
    """Doubles of every magnitude the score files can hold, plus the repr switch points."""
    v = [0.0, 1.0, 0.5, 0.1, 1 / 3, 1e-4, 9.999e-5, 1e-5, 1.5e-5, 0.00012345, 1e15, 1e16, 9999999999999998.0,
         1e16 + 2, 1e17, 123456789012345678.0, 2.0 ** -1074, 5e-324, 1.7976931348623157e308, 2.5, 100.0,
         0.30000000000000004, 1e-7, 123.456, 6.02e23]
    bits = rng.integers(0, 2**63 - 2**52, n // 2, dtype=np.int64)  # finite positive doubles
    v += [struct.unpack("<d", struct.pack("<q", int(b)))[0] for b in bits]
    c = rng.integers(0, 400, n - len(v) if n > len(v) else 1)
    u = c + rng.integers(1, 10**6, len(c))
    v += (c / u).tolist()  # Jaccard-like ratios
    return np.array(v[:n] if len(v) >= n else v, np.float64)


def test_parse_matches_json_loads(tmp_path):
    rng = np.random.default_rng(1)
    ex = _examples(rng)
    ex_native = scorefile.Examples.load(_write(tmp_path, ex))
    assert ex_native is not None
    _, _, u_ids, v_ids = similarity.flatten_examples(json.loads(open(tmp_path / "examples.json").read()))
    np.testing.assert_array_equal(ex_native.pair_user, u_ids)
    np.testing.assert_array_equal(ex_native.pair_business, v_ids)
    assert ex_native.n_users == len(ex)


@pytest.mark.parametrize("text", [
    '{"1": {"\\u0032": 1}}',        # escaped key: json.dumps would re-encode it
    '{"a": {"2": 1}}',              # not an integer key
    '{"1": {"2": [1]}}',            # nested value
    '{"1": {"2": 1, "2": 0}}',      # duplicate inner key (json.loads: first position, last value)
    '{"1": {"2": 1}, "1": {"3": 0}}',  # duplicate outer key
    '{"1": {"5": 1, "05": 0, "5": 0}}',  # duplicate key of one id interleaved with another spelling
    '{"1": {"2": abc}}',            # not a JSON value (json.loads raises)
    '{"1": {"2": 1.2.3}}',
    '{"1": {"2": tru}}',
    '{"1": {"2": 01}}',             # leading zero: not JSON
    '[1, 2]',
    '{"1": {"2": 1}} x',
])
def test_parse_refuses_other_shapes(tmp_path, text):
    p = tmp_path / "e.json"
    p.write_text(text)
    assert scorefile.Examples.load(str(p)) is None


@pytest.mark.parametrize("label", ["1", "0", "-1", "0.5", "1e3", "-2.5E-7", "true", "false", "null", "NaN", "Infinity",
                                   "-Infinity"])
def test_parse_accepts_json_scalars(tmp_path, label):
    """Every label json.loads accepts (numbers, literals, Python's NaN / Infinity) parses natively."""
    p = tmp_path / "e.json"
    p.write_text('{"1": {"2": %s, "3": 0}}' % label)
    ex = scorefile.Examples.load(str(p))
    assert ex is not None and ex.n_pairs == 2


@pytest.mark.parametrize("kind", ["cn", "jaccard", "adamic", "none", "jaccard_repr", "adamic_repr"])
@pytest.mark.parametrize("absent_rate", [0.0, 0.07])
def test_written_text_equals_json_dumps(tmp_path, kind, absent_rate):
    rng = np.random.default_rng(7)
    ex = _examples(rng, 120)
    exn = scorefile.Examples.load(_write(tmp_path, ex))
    n = exn.n_pairs
    present = rng.random(n) >= absent_rate
    k = int(present.sum())
    if kind == "cn":
        scores = {"cn": rng.integers(0, 5000, k).astype(np.uint32)}
        bit, code = similarity.blp.CN, scorefile.U32
        vals = scores["cn"]
    elif kind == "jaccard":
        scores = {"jaccard": _odd_doubles(rng, k)}
        bit, code = similarity.blp.JACCARD, scorefile.F64
        vals = scores["jaccard"]
    elif kind == "adamic":
        a = _odd_doubles(rng, k)
        a[rng.random(k) < 0.2] = 0.0  # nothing added: the int 0
        scores = {"adamic": a}
        bit, code = similarity.blp.ADAMIC, scorefile.F64_INT0
        vals = a
    elif kind == "jaccard_repr":  # pre-formatted slots (similarity.main: formatted on the device)
        scores = {"jaccard": _odd_doubles(rng, k)}
        bit, code = similarity.blp.JACCARD, scorefile.REPR24
        vals = scorefile.format_repr(scores["jaccard"])
    elif kind == "adamic_repr":
        a = _odd_doubles(rng, k)
        a[rng.random(k) < 0.2] = 0.0
        scores = {"adamic": a}
        bit, code = similarity.blp.ADAMIC, scorefile.REPR24
        vals = scorefile.format_repr(a, zero_int=True)
    else:
        scores, bit, code, vals = {}, 0, scorefile.NONE, None
    out = str(tmp_path / "out.json")
    exn.write(out, code, None if present.all() else present, vals)
    want = json.dumps(similarity.assemble(ex, similarity._values(bit, present, scores)))
    assert open(out).read() == want


def test_float_repr_many_values(tmp_path):
    rng = np.random.default_rng(3)
    v = _odd_doubles(rng, 200000)
    ex = {"1": {str(10**6 + i): 0 for i in range(len(v))}}
    exn = scorefile.Examples.load(_write(tmp_path, ex))
    out = str(tmp_path / "o.json")
    exn.write(out, scorefile.F64, None, v)
    got = json.loads(open(out).read())["1"]
    text = open(out).read()
    assert text == json.dumps({"1": {str(10**6 + i): float(x) for i, x in enumerate(v)}})
    assert all(math.isfinite(x) for x in got.values())


def test_empty_examples(tmp_path):
    for obj in ({}, {"5": {}}):
        exn = scorefile.Examples.load(_write(tmp_path, obj))
        assert exn is not None and exn.n_pairs == 0
        out = str(tmp_path / "o.json")
        exn.write(out, scorefile.U32, None, np.zeros(0, np.uint32))
        assert open(out).read() == "{}"
        os.unlink(out)
