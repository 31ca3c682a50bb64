"""Config-3 top-k phase clocks (experiment library built with -DBLP_PROF: BLP_LIB=...libblp_tkprof.so).
Sums of thread 0's clock64 deltas over all workgroups, per phase of k_topk:
0 dequeue/setup+filter, 1 counter zeroing, 2 count push (fused AA), 3 clear + CN/J selection,
4 AA from the fused sums, 5 AA hash path, 6 AA direct path, 7 list padding, 8 Jaccard selection
(3 is then the clear + CN selection); then the selection rounds walked per method and the
compactions (round 5)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "bipartite-link-prediction_amd"))
import numpy as np  # noqa: E402

import blp  # noqa: E402
from blp import synth  # noqa: E402
from blp.topk import TopK  # noqa: E402

U, B, D = synth.CONFIGS["c2"]
a, b = synth.review_edges(U, B, D, seed=0)
G = blp.DeviceGraph(a, b)
G.n_users_hint = U
src = synth.sample_users(G, 10000, seed=0)
T = TopK(G, "user")
T.set_sources(src)
mask = blp.JACCARD | blp.ADAMIC
buf = (ctypes.c_ulonglong * 16)()
T.run(20, mask)
blp.device_sync(0)
blp.lib().blp_topk_prof_read(buf)
T.run(20, mask)
blp.device_sync(0)
blp.lib().blp_topk_prof_read(buf)
v = np.array(buf[:10], np.float64)
names = ["setup", "zero", "push", "sel_cn", "aa_fused", "aa_hash", "aa_direct", "pad", "sel_j", "-"]
print({n: "%.1f%%" % (100 * x / v.sum()) for n, x in zip(names, v)}, "info", T.info(), flush=True)
print("wavesel=%s rounds per source: CN %.1f, Jaccard %.1f; compactions per source %.2f; per-wave 64-target "
      "blocks per source: CN %.1f, Jaccard %.1f" % (os.environ.get("BLP_TK_WAVESEL", "0"), buf[10] / len(src),
                                                    buf[11] / len(src), buf[12] / len(src), buf[13] / len(src),
                                                    buf[14] / len(src)), flush=True)
