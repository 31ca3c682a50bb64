"""Summarise rocprofv3 outputs (rocpd SQLite) into profiles/<name>.json + .md.

usage: python profiles/summarize.py NAME TRACE_DB [FETCH_DB] [WRITE_DB]

TRACE_DB comes from `rocprofv3 --kernel-trace --stats`; FETCH_DB / WRITE_DB from separate
`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes (they cannot share a pass on
gfx950: MI355X_MICROARCH.md, rocprofv3 PMC slots). Per the same guide (HBM section),
FETCH_SIZE counts 64 B per 128-B read request on gfx950, so the corrected read bytes are
2 x FETCH_SIZE; WRITE_SIZE is taken as reported. Both are reported raw and corrected.
"""
import json
import os
import sqlite3
import sys


def kernel_stats(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
                       "max(lds_size), max(vgpr_count), max(sgpr_count), max(workgroup_x), max(grid_x) "
                       "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [{"kernel": r[0], "calls": r[1], "total_us": r[2] / 1e3, "avg_us": r[3] / 1e3, "min_us": r[4] / 1e3,
             "max_us": r[5] / 1e3, "pct": 100.0 * r[2] / tot, "lds_bytes": r[6], "vgpr": r[7], "sgpr": r[8],
             "block": r[9], "grid_threads": r[10]} for r in rows]


def counter(db, name):
    con = sqlite3.connect(db)
    rows = con.execute("select kernel_name, count(*), avg(value), avg(duration) from counters_collection "
                       "where counter_name = ? group by kernel_name", (name,)).fetchall()
    return {r[0]: {"dispatches": r[1], "avg_kb": r[2], "avg_us": r[3] / 1e3} for r in rows}


def main():
    name, trace = sys.argv[1], sys.argv[2]
    fetch = sys.argv[3] if len(sys.argv) > 3 else None
    write = sys.argv[4] if len(sys.argv) > 4 else None
    ks = kernel_stats(trace)
    fc = counter(fetch, "FETCH_SIZE") if fetch else {}
    wc = counter(write, "WRITE_SIZE") if write else {}
    for k in ks:
        f = fc.get(k["kernel"])
        w = wc.get(k["kernel"])
        k["fetch_kb_raw"] = f["avg_kb"] if f else None
        k["write_kb"] = w["avg_kb"] if w else None
        if f and w:
            k["hbm_bytes_corrected"] = 2 * f["avg_kb"] * 1024 + w["avg_kb"] * 1024
    here = os.environ.get("PROFILE_OUT") or os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, name + ".json"), "w") as fh:
        json.dump(ks, fh, indent=1)
    lines = ["# %s — rocprofv3 --kernel-trace --stats (+ separate FETCH_SIZE / WRITE_SIZE passes)" % name, "",
             "| kernel | calls | avg us | total us | % | LDS B | VGPR | FETCH KB (raw) | WRITE KB | HBM bytes (2xFETCH+WRITE) |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for k in ks:
        lines.append("| `%s` | %d | %.1f | %.1f | %.1f | %s | %s | %s | %s | %s |" % (
            k["kernel"][:90], k["calls"], k["avg_us"], k["total_us"], k["pct"], k["lds_bytes"], k["vgpr"],
            "%.0f" % k["fetch_kb_raw"] if k["fetch_kb_raw"] is not None else "-",
            "%.0f" % k["write_kb"] if k["write_kb"] is not None else "-",
            "%.3e" % k["hbm_bytes_corrected"] if k.get("hbm_bytes_corrected") else "-"))
    with open(os.path.join(here, name + ".md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
