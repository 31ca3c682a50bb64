"""The BLP_DEBUG build of the pair scorers (make debug -> libblp_debug.so): every
queue claim, long-slice queue slot, split-table row, hash-set probe chain and output index of
k_score / k_score_split / k_score_hash / k_split_combine is checked against its bound before
the access (pairs.hip PS_OK). Run in a child process with BLP_LIB pointing at the debug
library: (1) every scorer path on a graph scored bit-exact against the oracle with zero
violations (similarity.py:20-106); (2) a hash-set table deliberately overfilled (the debug
build takes BLP_HASH_WORK unclamped) is reported as a probe-bound violation by
blp_batch_fetch instead of spinning. Marked `gpu`."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "bipartite-link-prediction_amd", "blp", "libblp_debug.so")

pytestmark = pytest.mark.gpu

CHILD = r'''
import os, sys
import numpy as np
sys.path[:0] = [os.path.join(ROOT, "bipartite-link-prediction_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import blp, coracle
from helpers import bipartite_edges, dense_edges
assert blp._lib.LIB_PATH.endswith("libblp_debug.so"), blp._lib.LIB_PATH
rng = np.random.default_rng(3)
a, b = bipartite_edges(rng, 60000, 3000, 400000)
G = blp.DeviceGraph(a, b)
nu = G.n_col0
x = np.repeat(rng.choice(nu, 150, replace=False), 30).astype(np.int32)
y = rng.integers(nu, G.n, len(x)).astype(np.int32)
ids, oa, ob = dense_edges(a, b)
og = coracle.OracleGraph(len(ids), oa, ob)
mode = sys.argv[1]
for xs, ys in ((x, y), (y, x)):
    try:
        got = G.score_pairs(xs, ys, 7)
    except RuntimeError as e:
        print("FAILED:", e)
        sys.exit(3)
    cn, jac, aa, _ = og.score_pairs(np.searchsorted(ids, G.node_ids[xs]), np.searchsorted(ids, G.node_ids[ys]), 7)
    assert np.array_equal(got["cn"], cn) and np.array_equal(got["jaccard"], jac) and np.array_equal(got["adamic"], aa)
if mode == "oom":  # the create that ran out of memory released the wedge index and planned again
    import ctypes
    nv = ctypes.c_int64(0)
    blp.lib().blp_graph_wedge(G.handle, ctypes.byref(nv), None, None)
    assert nv.value == -1, nv.value
print("OK", mode)
'''


def _run(mode, extra):
    if not os.path.exists(LIB):
        pytest.fail("libblp_debug.so missing: run `make -C bipartite-link-prediction_amd/csrc debug`")
    env = dict(os.environ, BLP_LIB=LIB, **extra)
    return subprocess.run([sys.executable, "-c", "ROOT = %r\n" % ROOT + CHILD, mode], env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=240)


@pytest.mark.parametrize("mode,extra", [
    ("default", {}),
    ("split+hash", {"BLP_SPLIT": "3"}),
    ("split+hash big", {"BLP_SPLIT": "3", "BLP_HASH_BIG": "1"}),
    ("split big", {"BLP_SPLIT": "3", "BLP_SPLIT_BIG": "1", "BLP_NO_HASH": "1"}),
    ("split heavy", {"BLP_SPLIT": "8", "BLP_HEAVY_WORK": "50", "BLP_NO_HASH": "1"}),
    ("large", {"BLP_VARIANT": "2"}),
    ("global", {"BLP_FORCE_GLOBAL": "1"}),
    ("no short kernel", {"BLP_NO_SHORT_KERNEL": "1"}),
    ("grouped business", {"BLP_NO_WSET": "1"}),
])
def test_debug_build_no_violations(gpu, mode, extra):
    r = _run(mode, extra)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])


def test_debug_build_reports_overfilled_hash_table(gpu):
    """Every source routed to the 16,384-slot hash-set scorer, whatever its H2 size: the
    60K-user universe's large H2 sets fill the table, and the probe bound reports it."""
    r = _run("overfill", {"BLP_SPLIT": "3", "BLP_HASH_WORK": "1000000000"})
    assert r.returncode == 3, (r.stdout[-2000:], r.stderr[-2000:])
    assert "BLP_DEBUG" in r.stdout and "site 8" in r.stdout, r.stdout[-2000:]


@pytest.mark.parametrize("field,extra", [
    ("g_yb", {}),
    ("cn", {}),
    ("lq", {"BLP_SPLIT": "3"}),
    ("wedge", {"BLP_NO_WSET": "1"}),  # the grouped short-row scorer's wedge rows
    ("wset", {}),  # the wedge-set scorer's sets (k_score_wset, the business side by default)
])
def test_null_launch_pointer_is_refused(gpu, field, extra):
    """A launch path's device pointer nulled (BLP_DEBUG_NULL, debug build only) is refused on the
    host by blp_batch_score's pre-launch check (pairs.hip launch_pointers) with the pointer's
    name, before any kernel runs: the class of bug behind round 4's k_score_split fault (a
    dropped queue pointer) fails the call instead of the GPU."""
    r = _run("null " + field, dict(extra, BLP_DEBUG_NULL=field))
    assert r.returncode == 3, (r.stdout[-2000:], r.stderr[-2000:])
    assert "null device pointer" in r.stdout, r.stdout[-2000:]


def test_batch_oom_releases_wedge_index(gpu):
    """A batch create that runs out of HBM (BLP_DEBUG_OOM, debug build: the first create fails as
    hipMalloc would) releases the graph's wedge index -- no live batch reads it -- and plans the
    batch again without it; both sides still score bit-exact against the oracle."""
    r = _run("oom", {"BLP_DEBUG_OOM": "1"})
    assert r.returncode == 0 and "OK oom" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
