"""Probe: time one side's scorer of the config-2 bench workload under engine knobs.

usage: python profiles/probe_sides.py SIDE MASK [KNOB=VALUE ...] [-- KNOB=VALUE ...]
Each '--'-separated group of knobs is one variant; prints ms per launch (HIP events)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bipartite-link-prediction_amd"))
import numpy as np  # noqa: E402

import blp  # noqa: E402
from blp import synth  # noqa: E402


def main():
    side, mask = sys.argv[1], int(sys.argv[2])
    groups, cur = [], []
    for a in sys.argv[3:]:
        if a == "--":
            groups.append(cur)
            cur = []
        else:
            cur.append(a)
    groups.append(cur)
    U, B, D = synth.CONFIGS[os.environ.get("PROBE_CONFIG", "c2")]
    a, b = synth.review_edges(U, B, D, seed=0)
    G = blp.DeviceGraph(a, b)
    x, y, _ = synth.make_examples(G, U, B, D, n_users=int(os.environ.get("PROBE_USERS", "10000")), rate=0.01, seed=0)
    xs, ys = (x, y) if side == "user" else (y, x)
    for knobs in groups:
        saved = dict(os.environ)
        for kv in knobs:
            k, v = kv.split("=", 1)
            os.environ[k] = v
        bt = G.batch(xs, ys)
        for _ in range(3):
            bt.score(mask)
        blp.device_sync(0)
        bt.stats_reset()
        t = time.perf_counter()
        for _ in range(10):
            bt.score(mask)
        blp.device_sync(0)
        wall = (time.perf_counter() - t) / 10
        ms, n = bt.stats(0)
        gms, gn = bt.stats(1)
        print("%-50s score %.3f ms  group %.3f ms  wall %.3f ms  plan %s" %
              (" ".join(knobs) or "(default)", ms / n, gms / gn, wall * 1e3, bt.plan()), flush=True)
        bt.close()
        os.environ.clear()
        os.environ.update(saved)


if __name__ == "__main__":
    main()
