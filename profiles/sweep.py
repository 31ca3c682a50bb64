"""Tuning sweep (not a test, not the bench): build the config-2 graph and examples once, then
for each env setting (JSON list of dicts in SWEEP, read when the graph / batch is created)
re-create the device graph and batches and time the user and business scorers with the
library's own HIP-event timers, each pass alone (batches have their own streams and would
otherwise overlap). SWEEP_STEP=1 also times the co-scheduled step (blp_batches_score, wall).
Every setting's CN / Jaccard / AA must equal the first's.

  SWEEP='[{}, {"BLP_HOT_DENSITY": "32"}]' python profiles/sweep.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bipartite-link-prediction_amd"))
import blp  # noqa: E402
from blp import synth  # noqa: E402

cfg = os.environ.get("SWEEP_CONFIG", "c2")
settings = json.loads(os.environ.get("SWEEP", "[{}]"))
steps = int(os.environ.get("SWEEP_STEPS", "10"))
U, B, D = synth.CONFIGS[cfg]
a, b = synth.review_edges(U, B, D, seed=0)
G0 = blp.DeviceGraph(a, b, device=0)
ex_x, ex_y, _ = synth.make_examples(G0, U, B, D, n_users=10_000, rate=0.01, seed=0)
del G0
if os.environ.get("SWEEP_ONE_PAIR"):  # one pair per source: the H2 build alone
    _, first = np.unique(ex_x, return_index=True)
    ex_x, ex_y = ex_x[first], ex_y[first]
ref = None
for s in settings:
    saved = {k: os.environ.get(k) for k in s}
    os.environ.update({k: str(v) for k, v in s.items() if not k.startswith("_")})
    t0 = time.time()
    G = blp.DeviceGraph(a, b, device=0)
    tg = time.time() - t0
    um = int(s.get("_user_mask", 7))
    passes = [("user", G.batch(ex_x, ex_y), um), ("business", G.batch(ex_y, ex_x), 3)]
    for _, bt, m in passes:
        bt.score(m)
    blp.device_sync(0)
    for _, bt, _ in passes:
        bt.stats_reset()
    for _, bt, m in passes:  # each pass alone
        for _ in range(steps):
            bt.score(m)
        blp.device_sync(0)
    iso = {name: (bt.stats(0), bt.stats(1)) for name, bt, _ in passes}
    step_ms = None
    if os.environ.get("SWEEP_STEP"):
        t = time.perf_counter()
        for _ in range(steps):
            G.score_batches([(bt, m) for _, bt, m in passes])
        blp.device_sync(0)
        step_ms = (time.perf_counter() - t) / steps * 1e3
    prof = None
    if os.environ.get("SWEEP_PROF"):  # experiment build with -DBLP_PROF: per-phase clocks of k_score
        import ctypes
        L = blp._lib.lib()
        buf = (ctypes.c_ulonglong * 16)()
        L.blp_prof_read(buf)  # reset
        for name, bt, m in passes:
            L.blp_prof_read(buf)
            bt.score(m)
            blp.device_sync(0)
            L.blp_prof_read(buf)
            tot = sum(buf[:9]) or 1
            print(json.dumps({"phases_" + name: [round(buf[i] / tot, 3) for i in range(9)], "clk": tot}), flush=True)
    row = {"setting": s, "graph_s": round(tg, 2)}
    if step_ms is not None:
        row["step_ms"] = round(step_ms, 4)
    res = {}
    for name, bt, m in passes:
        (ms, n), (gms, gn) = iso[name]
        row[name + "_ms"] = round(ms / max(n, 1), 4)
        row[name + "_group_ms"] = round(gms / max(gn, 1), 4)
        res[name] = bt.fetch(m)
    if ref is None:
        ref = res
    else:
        same = all(np.array_equal(ref[k][f], res[k][f]) for k in res for f in res[k]
                   if res[k][f] is not None and ref[k][f] is not None)
        row["same"] = bool(same)
    print(json.dumps(row), flush=True)
    del passes, G
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
