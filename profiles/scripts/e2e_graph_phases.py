"""Where similarity.main's 'graph' phase goes at config 2: graph.txt parse, id map, device
CSR build, host mirror, graph handle (weights, hot and wedge indexes)."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "bipartite-link-prediction_amd"))
import numpy as np  # noqa: E402

import blp  # noqa: E402
from blp import synth  # noqa: E402
from blp.graph import DeviceGraph, parse_edge_list  # noqa: E402

U, B, D = synth.CONFIGS["c2"]
a, b = synth.review_edges(U, B, D, seed=0)
path = os.path.join(tempfile.mkdtemp(), "graph.txt")
np.savetxt(path, np.stack([a, b], 1), fmt="%d")
for rep in range(3):
    c = time.perf_counter
    t0 = c()
    pa, pb = parse_edge_list(path)
    t_parse = c() - t0
    t0 = c()
    G = DeviceGraph(pa, pb)
    t_graph = c() - t0
    print({"parse": round(t_parse, 4), "device_graph": round(t_graph, 4),
           **{k: round(v, 4) for k, v in G.build_times.items()}}, flush=True)
    G.close()
