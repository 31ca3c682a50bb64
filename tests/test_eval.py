"""The drop-in eval.py (bipartite-link-prediction_amd/eval.py) against the reference's own
recorded output (tests/golden/bip/eval.json, produced by running /root/reference/eval.py on
the golden test split; tests/golden/make_golden.py). Reference: eval.py:10-32."""
import contextlib
import io
import json
import math
import os
import shutil

import numpy as np
import pytest

import eval as E
import util
from helpers import GOLDEN, load

SPLIT = os.path.join(GOLDEN, "bip", "test")
RECORDED = load(os.path.join(GOLDEN, "bip", "eval.json"))


def _run(methods, data_dir):
    ex = load(os.path.join(SPLIT, "examples.json"))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        res = E.run_evaluation(ex, methods, 20, data_dir=data_dir)
    return res, buf.getvalue().splitlines()


@pytest.mark.parametrize("method", sorted(m for m in RECORDED if "raises" not in RECORDED[m]))
def test_run_evaluation_prints_the_reference_lines(method):
    res, lines = _run([method], SPLIT + "/")
    rec = RECORDED[method]
    # eval.py:29-31 prints "Method: m", then the two metric lines (indented here as there)
    assert lines[0] == "Method: " + method
    assert lines[1].strip() == rec["precision_line"]
    assert lines[2].strip() == rec["auc_line"]
    assert math.isclose(res[method]["auc"], rec["auc"], rel_tol=0, abs_tol=1e-15)


def test_b_adamic_raises_like_sklearn():
    # the reference's b_adamic file holds only missing-node zeros, all of one label:
    # sklearn.roc_auc_score raises ValueError (eval.py:26), and so must the drop-in
    assert RECORDED["b_adamic"]["raises"] == "ValueError"
    with pytest.raises(ValueError):
        _run(["b_adamic"], SPLIT + "/")


def test_roc_auc_equals_mann_whitney_with_ties():
    rng = np.random.default_rng(3)
    for n in (2, 7, 100, 5000):
        ys = rng.integers(0, 2, n)
        ys[0], ys[-1] = 0, 1
        ps = rng.integers(0, 6, n).astype(np.float64)  # heavy ties
        pos, neg = ps[ys == 1], ps[ys == 0]
        want = ((pos[:, None] > neg[None, :]).sum() + 0.5 * (pos[:, None] == neg[None, :]).sum()) / (
            len(pos) * len(neg))
        assert math.isclose(E.roc_auc(ys, ps), want, rel_tol=1e-12)


def test_grouped_precision_equals_dict_precision():
    ex = load(os.path.join(SPLIT, "examples.json"))
    pred = load(os.path.join(SPLIT, "u_cn.json"))
    labels, scores, starts = [], [], []
    for u in pred:
        starts.append(len(labels))
        for b in pred[u]:
            labels.append(ex[u][b])
            scores.append(pred[u][b])
    assert E.grouped_precision_at_k(labels, scores, starts, len(ex), 20) == E.precision_at_k(ex, pred, 20)


def test_stale_sidecar_is_ignored(tmp_path):
    """A .npz sidecar is used only while it describes the JSON beside it: after the JSON
    is rewritten by anything that does not refresh the sidecar, load_scores reads JSON."""
    f = str(tmp_path / "u_cn.json")
    d1 = {"1": {"10": 3, "11": 0}}
    util.write_json(d1, f)
    util.write_sidecar(d1, f)
    assert util.load_scores(f) == d1
    d2 = {"1": {"10": 7, "11": 1}, "2": {"10": 0}}
    with open(f, "w") as fh:  # the reference's util.write_json: no sidecar handling
        fh.write(json.dumps(d2))
    assert util.load_scores(f) == d2
    # util.write_json itself drops a sidecar it would make stale
    util.write_sidecar(d2, f)
    util.write_json(d1, f)
    assert not os.path.exists(f + ".npz")
    assert util.load_scores(f) == d1


def test_eval_reads_sidecar_when_fresh(tmp_path):
    d = str(tmp_path) + "/"
    for name in ("u_jaccard",):
        shutil.copy(os.path.join(SPLIT, name + ".json"), d + name + ".json")
        util.write_sidecar(load(d + name + ".json"), d + name + ".json")
    res, lines = _run(["u_jaccard"], d)
    assert lines[2].strip() == RECORDED["u_jaccard"]["auc_line"]
