"""Drop-in for the reference's similarity.py, computed by the HIP engine (libblp.so).

Same call surface (similarity.py:11-126) and the same score files: common_neighbors and
jaccard bit-exact; adamic_adar is the correctly rounded sum of the reference's own float
terms (exact integer sums on the device, rounded once: math.fsum of the same terms). The
reference adds those terms in Python set order with a rounding per add, so its last bits
depend on that order and differ from this value by a few ulps (~1e-15 relative):

* ``main(example_file, graph_file, u_methods, u_outfiles, b_methods, b_outfiles)``
* ``users(examples, G, methods, outfiles)`` / ``business(examples, G, methods, outfiles)``
* ``common_neighbors(s1, s2)``, ``jaccard(s1, s2)``, ``adamic_adar(s1, s2, G)``

``G`` is a :class:`blp.DeviceGraph` (from ``load_edge_list``), the engine's stand-in for
SNAP's PUNGraph. ``users``/``business`` score every (user, business) pair of
``examples`` in ONE fused device pass for all requested methods (the reference loops
once per method, similarity.py:48,91) and then write one JSON file per method in the
reference's dict order.

Reference behaviour kept on purpose:
* a pair with a node absent from the graph scores ``0`` (similarity.py:59-60,104-105);
* common_neighbors is a JSON int; jaccard a float; adamic_adar a float, or the int ``0``
  when nothing was added (similarity.py:118);
* an unknown method name assigns nothing for present pairs (no branch matches);
* business side: the Adamic-Adar branch only fires for the string at similarity.py:102,
  so ``'adamic_adar'`` yields a file holding only the missing-node zeros. Pass
  ``fix_adamic=True`` to score it instead (useful downstream, supervised_models.py:124);
* the per-pair ``print`` calls of business() (similarity.py:97,100) are not reproduced.
"""
import datetime
import os

import numpy as np

import blp
import util
from blp import scorefile

BUGGY_B_ADAMIC = "Beginning adamic adar coefficient computation"  # similarity.py:102
_U_BITS = {"common_neighbors": blp.CN, "jaccard": blp.JACCARD, "adamic_adar": blp.ADAMIC}
_B_BITS = {"common_neighbors": blp.CN, "jaccard": blp.JACCARD, BUGGY_B_ADAMIC: blp.ADAMIC}


# ----------------------------------------------------------------------------- host helpers
def flatten_examples(examples):
    """examples {u: {v: label}} -> (u_keys, v_keys, u_ids, v_ids) in dict order."""
    u_keys, v_keys = [], []
    for u, inner in examples.items():
        for v in inner:
            u_keys.append(u)
            v_keys.append(v)
    u_ids = np.array([int(k) for k in u_keys], dtype=np.int64)
    v_ids = np.array([int(k) for k in v_keys], dtype=np.int64)
    return u_keys, v_keys, u_ids, v_ids


def method_mask(methods, table):
    m = 0
    for name in methods:
        m |= table.get(name, 0)
    return m


def _values(method_bit, present, scores):
    """Per-pair Python values for one method, None where the reference assigns nothing."""
    n = len(present)
    if not method_bit:  # unknown method string: only the missing-node zeros are written
        vals = [None] * n
        for i in np.flatnonzero(~present).tolist():
            vals[i] = 0
        return vals
    if method_bit == blp.CN:
        got = scores["cn"].astype(np.int64).tolist()
    elif method_bit == blp.JACCARD:
        got = scores["jaccard"].tolist()
    else:
        a = scores["adamic"]
        got = a.tolist()
        for i in np.flatnonzero(a == 0.0).tolist():
            got[i] = 0  # similarity.py:118: the untouched int 0
    if present.all():
        return got
    vals = [0] * n  # similarity.py:59-60 / 104-105: missing node -> 0
    for k, i in enumerate(np.flatnonzero(present).tolist()):
        vals[i] = got[k]
    return vals


def assemble(examples, vals):
    """Nest per-pair values back into {u: {v: value}} (defaultdict(dict) semantics)."""
    out = {}
    i = 0
    for u, inner in examples.items():
        d = None
        for v in inner:
            val = vals[i]
            i += 1
            if val is not None:
                if d is None:
                    d = out[u] = {}
                d[v] = val
    return out


def score_examples(examples, G, side, mask):
    """Score every pair of `examples` on the device.

    Returns (present mask over the flattened pairs, scores dict over present pairs)."""
    _, _, u_ids, v_ids = flatten_examples(examples)
    du, pu = G.lookup(u_ids)
    dv, pv = G.lookup(v_ids)
    present = pu & pv
    if side == 0:
        scores = G.score_pairs(du[present], dv[present], mask)
    else:
        scores = G.score_pairs(dv[present], du[present], mask)
    return present, scores


def score_both_sides(examples, G, u_mask, b_mask):
    """Both passes of similarity.main in one device step: the user-side and the business-side
    batches are enqueued together (blp_batches_score) and run concurrently.

    Returns (present mask over the flattened pairs, user-side scores, business-side scores)."""
    _, _, u_ids, v_ids = flatten_examples(examples)
    return _score_both_ids(G, u_ids, v_ids, u_mask, b_mask)


def _score_both_ids(G, u_ids, v_ids, u_mask, b_mask, timings=None, text=False):
    """Id lookup, the two batches (blp_batch_create_pair: one upload, planned on the device),
    one concurrent device step, and the results; phase times into
    ``timings`` (score_lookup, score_create, score_device, score_fetch) when given. ``text``:
    the Jaccard / Adamic-Adar scores come back as their json.dumps text, formatted on the
    device (PairBatch.fetch_repr: "jaccard_repr" / "adamic_repr" slots), not as doubles."""
    import time

    t0 = time.perf_counter()
    du, pu = G.lookup(u_ids)
    dv, pv = G.lookup(v_ids)
    present = pu & pv
    xs, ys = (du, dv) if present.all() else (du[present], dv[present])
    t1 = time.perf_counter()
    ub, bb = G.batch_pair(xs, ys)  # one upload of the pairs for both passes
    try:
        t2 = time.perf_counter()
        G.score_batches([(ub, u_mask), (bb, b_mask)])
        blp.device_sync(G.device)  # the batches run on their own streams
        t3 = time.perf_counter()
        if text:
            ru = _fetch_text(ub, u_mask)
            t4 = time.perf_counter()
            res = present, ru, _fetch_text(bb, b_mask)
        else:
            ru = ub.fetch(u_mask)
            t4 = time.perf_counter()
            res = present, ru, bb.fetch(b_mask)
        if timings is not None:
            timings.update({"score_lookup": t1 - t0, "score_create": t2 - t1, "score_device": t3 - t2,
                            "score_fetch": time.perf_counter() - t3, "score_fetch_user": t4 - t3})
        return res
    finally:
        ub.close()
        bb.close()


def _fetch_text(batch, mask):
    """Counts as uint32; Jaccard / Adamic-Adar as device-formatted text slots (0.0 as the int 0
    for Adamic-Adar, similarity.py:118)."""
    res = batch.fetch(blp.CN)
    if mask & blp.JACCARD:
        res["jaccard_repr"] = batch.fetch_repr(blp.JACCARD)
    if mask & blp.ADAMIC:
        res["adamic_repr"] = batch.fetch_repr(blp.ADAMIC, zero_int=True)
    return res


def _run_side(examples, G, methods, outfiles, table, side, sidecar=False, scored=None):
    mask = method_mask(methods, table)
    present, scores = scored if scored is not None else score_examples(examples, G, side, mask | blp.CN)
    results = []
    for m, f in zip(methods, outfiles):
        sim = assemble(examples, _values(table.get(m, 0), present, scores))
        if f is not None:
            util.write_json(sim, f)
            if sidecar:
                util.write_sidecar(sim, f)
        results.append(sim)
    return results


def _write_jobs(ex, methods, outfiles, table, present, scores):
    """The score files of one side straight from the device arrays (util.write_json's text):
    one callable per file. The jobs take over the score arrays (``scores`` is emptied): each job
    drops its array when its file is written, so the array is released on that writer thread while
    the other files are still being written, not all at once after the last one."""
    import os

    pres = None if present.all() else present
    jobs = []
    for m, f in zip(methods, outfiles):
        if f is None:
            continue
        bit = table.get(m, 0)
        if bit == blp.CN:
            args = (scorefile.U32, pres, scores["cn"])
        elif bit == blp.JACCARD:
            args = ((scorefile.REPR24, pres, scores["jaccard_repr"]) if "jaccard_repr" in scores
                    else (scorefile.F64, pres, scores["jaccard"]))
        elif bit == blp.ADAMIC:
            args = ((scorefile.REPR24, pres, scores["adamic_repr"]) if "adamic_repr" in scores
                    else (scorefile.F64_INT0, pres, scores["adamic"]))
        else:  # a method the reference does not match: only missing-node zeros
            args = (scorefile.NONE, pres)

        def job(f=f, held=[args]):
            args = held.pop()  # from here on the only reference this job keeps
            ex.write(f, *args)
            del args
            if os.path.exists(f + ".npz"):  # as util.write_json: a stale sidecar goes
                os.unlink(f + ".npz")
        jobs.append(job)
    scores.clear()
    return jobs


def _write_files(jobs):
    """Run the file writes concurrently (each native write formats on its own threads and
    releases the GIL; files on different inodes do not serialise on one inode lock). The
    contents are what the reference's sequential writes give; a failure raises as there."""
    from concurrent.futures import ThreadPoolExecutor

    workers = max(1, int(os.environ.get("BLP_FILE_WRITERS", "6")))  # config 2: 6 -> 0.061-0.068 s, 3 -> 0.093-0.100 s
    if workers == 1 or len(jobs) < 2:
        while jobs:
            jobs.pop(0)()
        return
    with ThreadPoolExecutor(min(workers, len(jobs))) as pool:
        futs = [pool.submit(j) for j in jobs]
        jobs.clear()  # the executor holds the jobs now: each is released once it has run
        for fut in futs:
            fut.result()


# ----------------------------------------------------------------------------- reference API
def main(example_file, graph_file, u_methods, u_outfiles, b_methods, b_outfiles, *, sidecar=False, timings=None):
    """similarity.main (similarity.py:11-18). ``sidecar=True`` also writes each score file's
    binary twin ``<file>.npz`` (util.write_sidecar). ``timings``: an optional dict that receives
    the wall time of each phase in seconds (examples, graph, score, files)."""
    import time

    clock = time.perf_counter
    t = clock()
    datetime.datetime.now()
    print("Loading examples...")
    # examples.json of the reference's shape is read natively into flat arrays (anything else:
    # json.loads, as util.load_json); the score files are then written natively with the same
    # text json.dumps gives (blp/scorefile.py). With sidecar=True the dict path runs.
    import os
    from concurrent.futures import ThreadPoolExecutor

    def load_examples():
        # a missing or unreadable file raises what util.load_json raises (IOError / FileNotFoundError)
        e = None if sidecar or not os.path.isfile(example_file) else scorefile.Examples.load(example_file)
        return e, (util.load_json(example_file) if e is None else None)

    if not os.path.isfile(example_file):
        load_examples()  # raises (before any device work, as the reference does)
    # examples.json is parsed on a second thread while the graph loads (both native calls release
    # the GIL); a third starts the HIP runtime, whose first call costs a few tenths of a second
    pool = ThreadPoolExecutor(2)
    fut_ex = pool.submit(load_examples)
    if os.environ.get("BLP_NO_PREWARM"):  # A/B knob: the HIP runtime only
        pool.submit(blp.device_sync, 0)
    else:
        pool.submit(blp.prewarm, 0, 3)  # the HIP runtime, the pooled streams (parse / CSR / fetch in turn, the graph, two batches at most 3 at once) and the kernels' code objects
    ex = G = None
    try:
        print("Loading graph...")
        try:
            G = blp.load_edge_list(graph_file)
        except BaseException:
            if fut_ex.exception() is not None:  # the reference reports the examples file first
                raise fut_ex.exception()
            raise
        t_g = clock()
        ex, examples = fut_ex.result()
        t_ex = clock()
        # both passes in one concurrent device step, then the files in the reference's order
        print("Scoring user and business sides on the device...")
        masks = method_mask(u_methods, _U_BITS) | blp.CN, method_mask(b_methods, _B_BITS) | blp.CN
        if ex is None:
            present, u_scores, b_scores = score_both_sides(examples, G, *masks)
        else:
            present, u_scores, b_scores = _score_both_ids(G, ex.pair_user, ex.pair_business, *masks, timings=timings,
                                                          text=True)
        t_s = clock()
        if ex is None:
            _run_side(examples, G, u_methods, u_outfiles, _U_BITS, 0, sidecar, scored=(present, u_scores))
            _run_side(examples, G, b_methods, b_outfiles, dict(_B_BITS), 1, sidecar, scored=(present, b_scores))
        else:
            _write_files(_write_jobs(ex, u_methods, u_outfiles, _U_BITS, present, u_scores) +
                         _write_jobs(ex, b_methods, b_outfiles, _B_BITS, present, b_scores))
    finally:
        t_f = clock()
        pool.shutdown(wait=True)
        if ex is None and fut_ex.done() and fut_ex.exception() is None:
            ex = fut_ex.result()[0]
        if ex is not None:
            ex.close()
        t_c = clock()
        # (no locals(): its snapshot dict would hold every array of this frame until main returns)
        if G is not None:  # the reference's graph goes when main returns; so does this one (HBM freed here)
            G.close()
    if timings is not None:
        # examples and graph load concurrently: "graph" is the graph load, "examples" the extra
        # wait for examples.json after it
        timings.update({"graph": t_g - t, "examples": t_ex - t_g, "score": t_s - t_ex, "files": t_f - t_s,
                        "teardown": t_c - t_f, "graph_release": clock() - t_c, "pairs": int(present.sum())})
        timings["graph_detail"] = dict(getattr(G, "build_times", None) or {})
        # what returning releases, timed: the score arrays, the examples, the host half of the graph
        if os.environ.get("BLP_E2E_REFDEBUG"):  # diagnostics: who else holds them at this point
            import gc
            import sys

            for name, obj in (("u_scores", u_scores), ("u_jaccard_repr", u_scores.get("jaccard_repr")), ("ex", ex),
                              ("G", G), ("present", present)):
                if obj is None:
                    continue
                refs = [type(r).__name__ for r in gc.get_referrers(obj)]
                print("[refdebug] %s refcount %d referrers %s" % (name, sys.getrefcount(obj), refs[:8]), file=sys.stderr)
        t_r = clock()
        del present, u_scores, b_scores
        t_r1 = clock()
        del ex, fut_ex
        t_r2 = clock()
        del G
        timings.update({"release_scores": t_r1 - t_r, "release_examples": t_r2 - t_r1, "release_graph": clock() - t_r2})
        timings["_clock_entry"], timings["_clock_exit"] = t, clock()  # the caller times the call and return around them


def users(examples, G, methods, outfiles, *, sidecar=False):
    """similarity.users (similarity.py:20-61): x = user (exact 2-hop set), y = business."""
    print("Scoring user side on the device...")
    return _run_side(examples, G, methods, outfiles, _U_BITS, side=0, sidecar=sidecar)


def business(examples, G, methods, outfiles, *, fix_adamic=False, sidecar=False):
    """similarity.business (similarity.py:63-106): x = business (exact 2-hop set), y = user."""
    print("Scoring business side on the device...")
    table = dict(_B_BITS)
    if fix_adamic:
        table["adamic_adar"] = blp.ADAMIC
    return _run_side(examples, G, methods, outfiles, table, side=1, sidecar=sidecar)


# Scalar set-level definitions (similarity.py:108-126), kept for API compatibility with
# callers that hold their own Python sets. The batch path above never calls them.
def jaccard(setone, settwo):
    intersection = len(setone.intersection(settwo))
    union = len(setone.union(settwo))
    return float(intersection) / float(union)


def common_neighbors(setone, settwo):
    return len(setone.intersection(settwo))


def adamic_adar(setone, settwo, G):
    import math

    total = 0
    for i in setone.intersection(settwo):
        deg = G.GetDeg(i)
        if deg > 1:
            total += math.log(deg) ** -1
        else:
            total += 0
    return total


if __name__ == "__main__":
    names = ["common_neighbors", "jaccard", "adamic_adar"]
    for split in ("train", "test"):
        d = "./data/%s/" % split
        main(d + "examples.json", d + "graph.txt", names,
             [d + "u_cn.json", d + "u_jaccard.json", d + "u_adamic.json"], names,
             [d + "b_cn.json", d + "b_jaccard.json", d + "b_adamic.json"])
