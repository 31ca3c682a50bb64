"""Round 5: fold the A/B runs under gpurun_out/ into compact records under profiles/ (one JSON per
experiment family: every run's step, scorer and grouping times, parity, end-to-end phases).

usage: python profiles/scripts/r05_collect.py OUT_NAME "note" PREFIX [PREFIX ...]
Each PREFIX matches gpurun_out/<PREFIX>*.json (the bench's last JSON line per file)."""
import glob
import json
import os
import sys


def last_json(path):
    with open(path) as f:
        lines = [ln for ln in f.read().strip().splitlines() if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def fields(d):
    r = {}
    if "e2e_s" in d:
        r["e2e_s"] = round(d["e2e_s"], 4)
        r["phases_s"] = {k: round(v, 4) for k, v in (d.get("phases_s") or {}).items()}
        r["graph_detail_s"] = {k: round(v, 4) for k, v in (d.get("graph_phase_detail_s") or {}).items()}
        r["files_equal_oracle"] = d.get("ok")
        return r
    for k in ("ms_per_step", "value"):
        if k in d:
            r[k] = d[k]
    km = d.get("kernels_ms") or {}
    for side, v in km.items():
        if isinstance(v, dict):
            for kk, vv in v.items():
                r["%s_%s" % (side, kk)] = vv
    if d.get("parity") is not None:
        p = d["parity"]
        r["parity_ok"] = p.get("ok") if isinstance(p, dict) else p
    ibc = d.get("including_batch_create")
    if ibc:
        r["batch_create_s"] = ibc.get("batch_create_s")
    for k in ("topk", "factorization", "exchange"):
        if isinstance(d.get(k), dict):
            r[k] = {kk: vv for kk, vv in d[k].items() if isinstance(vv, (int, float, str, bool))}
    return r


def main():
    out, note, prefixes = sys.argv[1], sys.argv[2], sys.argv[3:]
    runs = []
    for pre in prefixes:
        for p in sorted(glob.glob(os.path.join("gpurun_out", pre + "*.json"))):
            d = last_json(p)
            if d is None:
                continue
            runs.append({"run": os.path.basename(p)[:-5], **fields(d)})
    with open(os.path.join("profiles", out + ".json"), "w") as f:
        json.dump({"note": note, "runs": runs}, f, indent=1)
    print(out, len(runs), "runs")


if __name__ == "__main__":
    main()
