"""Headline-size parity in the GPU suite (BASELINE.json configs[1], "config 2"): the full
1M-user x 100K-business, 10M-draw graph the bench scores, a slice of its example users, both
passes of similarity.main enqueued as one co-scheduled step (blp_batches_score) exactly as the
bench's timed step runs them, checked bit-exact against the C oracle (the reference algorithm,
similarity.py:20-106, :108-126). The user pass must take the instance the bench times and
rooflines: the large block scorer's packed-count variant (k_score<1024, 31744, 896, 8, false,
true, true>, PKO: one LDS bitmap over the 1M-user universe, counts in the packed word); the
business pass the wedge-set scorer without Adamic-Adar (k_score_wset<false>, round 6: pair by pair
in caller order against the graph's dense wedge-set index, after the user pass) -- the kernels and
geometry of the headline number. Marked `gpu`."""
import os

import numpy as np
import pytest

import blp
import coracle
from blp import synth
from helpers import dense_edges

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("create", ["pair", "two"])
def test_config2_slice_both_sides_coscheduled(gpu, create):
    """create="pair": the bench's own creation (bench.py: G.batch_pair, blp_batch_create_pair --
    one upload of the pairs, the user pass on a highest-priority stream, the business pass's pairs
    copied device to device); "two": two independent blp_batch_create calls."""
    U, B, D = synth.CONFIGS["c2"]
    a, b = synth.review_edges(U, B, D, seed=0)
    G = blp.DeviceGraph(a, b, device=gpu)
    ex_x, ex_y, ex_l = synth.make_examples(G, U, B, D, n_users=220, rate=0.01, seed=7)
    assert len(ex_x) >= 150_000 and len(np.unique(ex_x)) == 220
    ub, bb = G.batch_pair(ex_x, ex_y) if create == "pair" else (G.batch(ex_x, ex_y), G.batch(ex_y, ex_x))
    plan = ub.plan()
    assert plan["block"] == 1024 and plan["chunks"] == 1 and plan["hi"] - plan["lo"] > 31744 * 16, plan
    assert ub.kernel(7) == "k_score<1024, 31744, 896, 8, false, true, true>", ub.kernel(7)  # bench.py's roofline kernel
    assert bb.kernel(3) == "k_score_wset<false>", bb.kernel(3)  # the business pass on the graph's wedge sets
    G.score_batches([(ub, 7), (bb, 3)])  # the bench's step: both passes concurrent, user pass on its CU share
    got_u, got_b = ub.fetch(7), bb.fetch(3)
    ids, oa, ob = dense_edges(a, b)
    og = coracle.OracleGraph(len(ids), oa, ob)
    xo = np.searchsorted(ids, G.node_ids[ex_x])
    yo = np.searchsorted(ids, G.node_ids[ex_y])
    nt = max(1, len(os.sched_getaffinity(0)))
    cn, jac, aa, _ = og.score_pairs(xo, yo, 7, nthreads=nt)
    np.testing.assert_array_equal(got_u["cn"], cn)
    np.testing.assert_array_equal(got_u["jaccard"], jac)
    np.testing.assert_array_equal(got_u["adamic"], aa)
    cn, jac, _, _ = og.score_pairs(yo, xo, 3, nthreads=nt)
    np.testing.assert_array_equal(got_b["cn"], cn)
    np.testing.assert_array_equal(got_b["jaccard"], jac)
    # a repeated step is bit-identical (order-independent exact arithmetic)
    G.score_batches([(ub, 7), (bb, 3)])
    again = ub.fetch(7)
    for k in ("cn", "jaccard", "adamic"):
        np.testing.assert_array_equal(again[k], got_u[k])
