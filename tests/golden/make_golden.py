"""Generate the committed golden fixtures under tests/golden/<case>/ (build container only).

Run:  python tests/golden/make_golden.py        (needs /root/reference; ~1 min)

Inputs are synthetic graphs made here with numpy (seeded). Every *expected output*
is produced by the reference's own code (``refload.load()``: lib2to3-translated
``similarity.py``, ``svd.py``, ``eval.py``, ``random_walks.py``, ``dataset_maker.py``),
run in a scratch directory laid out the way the reference expects (``./data/train``,
``./data/test``). Fixtures are data only: graph/example inputs and score outputs.

Cases
  bip     bipartite review graph, train+test splits; examples from the reference's
          ``make_examples`` (dataset_maker.py:80-159, rate 0.3); all six similarity
          outputs (similarity.py:128-142), svd.json + the exact factors used
          (svd.py:24-30), random_walks.json (random_walks.py:9-41), eval results
          (eval.py:10-46) for every method file.
  hop3    same train graph, ``make_examples`` with negative_sample_rate=1.0 and every
          eligible user: the exact hop-3 candidate set (dataset_maker.py:137-144).
  edge    hand-made edge cases: '#' comment, duplicate + reversed edges, a self-loop,
          missing user / business keys, degree-1 intersectors, empty intersections.
  general non-bipartite graph (user-user and business-business edges, triangles):
          exercises *exact*-distance hop sets and random walks with nonzero scores.
"""
import contextlib
import io
import json
import os
import random
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refload  # noqa: E402


def _write_graph(d, edges, extra_lines=()):
    with open(os.path.join(d, "graph.txt"), "w") as f:
        for line in extra_lines:
            f.write(line)
        for a, b in edges:
            f.write("%d %d\n" % (a, b))


def _bip_reviews(rng, n_users, n_bus, n_draws, zipf=0.8):
    """Reviews (user_key, business_key) with Zipf business popularity."""
    p = np.arange(1, n_bus + 1, dtype=np.float64) ** -zipf
    p /= p.sum()
    us = rng.integers(0, n_users, n_draws)
    bs = rng.choice(n_bus, size=n_draws, p=p)
    return list(zip(us.tolist(), bs.tolist()))


def _assign_ids(reviews):
    """dataset_maker.KeyToInt (dataset_maker.py:9-18): first-appearance ids, shared space."""
    ids = {}

    def key(k):
        if k not in ids:
            ids[k] = len(ids)
        return ids[k]

    out = [(key("u%d" % u), key("b%d" % b)) for u, b in reviews]
    users = sorted({ids[k] for k in ids if k[0] == "u"})
    buses = sorted({ids[k] for k in ids if k[0] == "b"})
    return out, users, buses


def _run_quiet(fn, *a, **k):
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        r = fn(*a, **k)
    return r, buf.getvalue()


def _similarity(ref, d):
    sim = ref["similarity"]
    names = ["common_neighbors", "jaccard", "adamic_adar"]
    _run_quiet(
        sim.main,
        os.path.join(d, "examples.json"),
        os.path.join(d, "graph.txt"),
        names,
        [os.path.join(d, f) for f in ("u_cn.json", "u_jaccard.json", "u_adamic.json")],
        names,
        [os.path.join(d, f) for f in ("b_cn.json", "b_jaccard.json", "b_adamic.json")],
    )


def _svd(ref, root, split, k):
    """svd.svd_user_business with the factors it used recorded (svd.py:24-25)."""
    import scipy.sparse.linalg as spla

    rec = {}
    orig = spla.svds

    def svds(M, k=6, **kw):
        u, s, vt = orig(M, k=k, **kw)
        rec.update(u=u, s=s, vt=vt)
        return u, s, vt

    spla.svds = svds
    try:
        cwd = os.getcwd()
        os.chdir(root)
        _run_quiet(ref["svd"].svd_user_business, split, k)
    finally:
        os.chdir(cwd)
        spla.svds = orig
    d = os.path.join(root, "data", split)
    np.save(os.path.join(d, "svd_U.npy"), rec["u"])
    np.save(os.path.join(d, "svd_s.npy"), rec["s"])
    np.save(os.path.join(d, "svd_Vt.npy"), rec["vt"])


def _random_walks(ref, root):
    cwd = os.getcwd()
    os.chdir(root)
    try:
        _run_quiet(ref["random_walks"].run_random_walks, "train", False)
    finally:
        os.chdir(cwd)


def _eval(ref, root, methods):
    """eval.run_evaluation (eval.py:10-46): record exact AUC and the printed lines."""
    ev = ref["eval"]
    aucs = []
    orig_auc = ev.roc_auc_score

    def roc_auc_score(ys, ps):
        v = orig_auc(ys, ps)
        aucs.append(float(v))
        return v

    ev.roc_auc_score = roc_auc_score
    cwd = os.getcwd()
    os.chdir(root)
    try:
        examples = ref["util"].load_json("data/test/examples.json")
        _, out = _run_quiet(ev.run_evaluation, examples, methods)
    finally:
        os.chdir(cwd)
        ev.roc_auc_score = orig_auc
    lines = [l for l in out.splitlines() if l.strip()]
    res = {}
    i = 0
    for m, auc in zip(methods, aucs):
        assert lines[i] == "Method: " + m, lines[i]
        res[m] = {"precision_line": lines[i + 1].strip(), "auc_line": lines[i + 2].strip(), "auc": auc}
        i += 3
    return res


def _make_split(ref, d, reviews_graph, reviews_new, users, buses, rate, n_users, seed_extra=()):
    os.makedirs(d, exist_ok=True)
    _write_graph(d, reviews_graph)
    with open(os.path.join(d, "new_edges.txt"), "w") as f:
        for a, b in reviews_new:
            f.write("%d %d\n" % (a, b))
    review = {}
    for a, b in reviews_graph:
        review.setdefault(str(a), {}).setdefault(str(b), []).append({"date": "2011-01-01"})
    ref["util"].write_json(review, os.path.join(d, "review.json"))
    ref["util"].write_json({str(u): {"user_id": "u%d" % u} for u in users}, os.path.join(d, "user.json"))
    ref["util"].write_json({str(b): {"business_id": "b%d" % b} for b in buses}, os.path.join(d, "business.json"))
    random.seed(0)
    _run_quiet(ref["dataset_maker"].make_examples, d + "/", n_users=n_users, negative_sample_rate=rate)


def case_bip(ref, out):
    rng = np.random.default_rng(12345)
    root = tempfile.mkdtemp(prefix="blp_golden_")
    try:
        reviews = _bip_reviews(rng, n_users=150, n_bus=40, n_draws=700)
        ided, users, buses = _assign_ids(reviews)
        # time split: first 80% of reviews are the train graph, the rest are new edges
        ntr = int(0.8 * len(ided))
        seen = set()
        g_tr, new_tr = [], []
        for e in ided[:ntr]:
            g_tr.append(e)
            seen.add(e)
        new_tr = sorted({e for e in ided[ntr:] if e not in seen})
        # test split: the whole history is the graph; fresh draws are the new edges
        extra = _assign_ids(reviews + _bip_reviews(rng, 150, 40, 150))[0][len(reviews):]
        seen_all = set(ided)
        new_te = sorted({e for e in extra if e not in seen_all})
        tr_nodes = sorted({n for e in g_tr for n in e})
        tr_users = [u for u in users if u in set(tr_nodes)]
        tr_bus = [b for b in buses if b in set(tr_nodes)]
        dtr = os.path.join(root, "data", "train")
        dte = os.path.join(root, "data", "test")
        _make_split(ref, dtr, g_tr, new_tr, tr_users, tr_bus, 0.3, 40)
        _make_split(ref, dte, ided, new_te, users, buses, 0.3, 40)
        for d in (dtr, dte):
            _similarity(ref, d)
        _svd(ref, root, "train", 8)
        _svd(ref, root, "test", 8)
        _random_walks(ref, root)
        # eval over every method file the build produces (eval.py:49-64 subset)
        # b_adamic.json is {} (similarity.py:102 never matches), and eval.py:26 raises
        # ValueError on it (sklearn: 0 samples) -- recorded, not evaluated.
        methods = ["examples", "u_adamic", "u_cn", "u_jaccard", "b_cn", "b_jaccard", "svd"]
        ev = _eval(ref, root, methods)
        try:
            _eval(ref, root, ["b_adamic"])
            ev["b_adamic"] = {"raises": None}
        except ValueError as e:
            ev["b_adamic"] = {"raises": "ValueError"}
        for split in ("train", "test"):
            src = os.path.join(root, "data", split)
            dst = os.path.join(out, "bip", split)
            os.makedirs(dst, exist_ok=True)
            for f in os.listdir(src):
                if f in ("review.json",):
                    continue
                shutil.copy(os.path.join(src, f), dst)
        with open(os.path.join(out, "bip", "eval.json"), "w") as f:
            json.dump(ev, f, indent=1, sort_keys=True)
        # hop3: exact candidate set, every eligible user, rate 1.0 (dataset_maker.py:139-144)
        dh = os.path.join(root, "hop3")
        _make_split(ref, dh, g_tr, new_tr, tr_users, tr_bus, 1.0, len(tr_users))
        os.makedirs(os.path.join(out, "hop3"), exist_ok=True)
        for f in ("graph.txt", "new_edges.txt", "examples.json"):
            shutil.copy(os.path.join(dh, f), os.path.join(out, "hop3", f))
    finally:
        shutil.rmtree(root)


def case_edge(ref, out):
    """Hand-made edge cases for similarity.py's quirks."""
    d = os.path.join(out, "edge")
    os.makedirs(d, exist_ok=True)
    # users 0..7, businesses 100..105
    edges = [
        (0, 100), (0, 101), (1, 100), (1, 102), (2, 101), (2, 102), (2, 103),
        (3, 103), (4, 104), (5, 100), (5, 104), (6, 105), (7, 102),
        (1, 100), (100, 1),  # duplicate and reversed duplicate (SNAP dedups)
        (5, 5),              # self-loop: counted once in GetDeg (AA weight of user 5)
    ]
    _write_graph(d, edges, extra_lines=["# comment line skipped by LoadEdgeList\n"])
    examples = {
        "0": {"102": 1, "103": 0, "104": 0, "105": 0, "999": 0},  # 999: missing business
        "1": {"101": 0, "103": 1, "104": 1},
        "3": {"100": 0, "102": 1, "105": 0},                        # 3 has degree 1
        "4": {"100": 1, "101": 0},
        "6": {"100": 0, "105": 1},                                  # 105 is 6's own business
        "7": {"101": 1, "103": 0},
        "888": {"100": 0, "101": 1},                                # missing user
        "2": {},                                                    # empty candidate dict
    }
    ref["util"].write_json(examples, os.path.join(d, "examples.json"))
    _similarity(ref, d)


def case_general(ref, out):
    """Non-bipartite graph: hop sets must be *exact* distance (similarity.py:29,41,74,85)."""
    rng = np.random.default_rng(777)
    root = tempfile.mkdtemp(prefix="blp_golden_g_")
    try:
        n = 40
        edges = set()
        while len(edges) < 90:
            a, b = rng.integers(0, n, 2).tolist()
            if a != b:
                edges.add((a, b))
        # first-appearance relabel so random_walks' id == row invariant holds (random_walks.py:36,44)
        ids = {}
        el = []
        for a, b in sorted(edges, key=lambda e: rng.random()):
            for x in (a, b):
                if x not in ids:
                    ids[x] = len(ids)
            el.append((ids[a], ids[b]))
        d = os.path.join(root, "data", "train")
        os.makedirs(d)
        _write_graph(d, el)
        nodes = sorted(ids.values())
        ex = {}
        for u in rng.choice(nodes, 12, replace=False).tolist():
            vs = rng.choice(nodes, 8, replace=False).tolist()
            ex[str(u)] = {str(v): int(rng.integers(0, 2)) for v in vs if v != u}
        ref["util"].write_json(ex, os.path.join(d, "examples.json"))
        _similarity(ref, d)
        _random_walks(ref, root)
        dst = os.path.join(out, "general")
        os.makedirs(dst, exist_ok=True)
        for f in os.listdir(d):
            shutil.copy(os.path.join(d, f), dst)
    finally:
        shutil.rmtree(root)


def main():
    out = HERE
    ref = refload.load()
    case_edge(ref, out)
    case_general(ref, out)
    case_bip(ref, out)
    total = 0
    for dp, _, fs in os.walk(out):
        for f in fs:
            if dp != out:
                total += os.path.getsize(os.path.join(dp, f))
    print("fixtures written, %.1f KB" % (total / 1024.0))


if __name__ == "__main__":
    main()
