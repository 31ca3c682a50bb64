"""Round 5: the slow HIP API calls and copies of a rocprofv3 CSV timeline (r05_e2e_trace.sh).

usage: python profiles/scripts/r05_trace_slow.py DIR [min_ms]
Prints, in time order, every HIP API call and memory copy longer than min_ms (default 1), and
the kernels overlapping each slow call, with times relative to the first record."""
import csv
import glob
import gzip
import os
import sys


def rows(d, pat):
    out = []
    for p in glob.glob(os.path.join(d, pat)):
        op = gzip.open if p.endswith(".gz") else open
        with op(p, "rt") as f:
            out += list(csv.DictReader(f))
    return out


def main():
    d = sys.argv[1]
    thr = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    api = rows(d, "*hip_api_trace.csv*")
    cp = rows(d, "*memory_copy_trace.csv*")
    kt = rows(d, "*kernel_trace.csv*")
    t0 = min(int(r["Start_Timestamp"]) for r in api)
    ev = []
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ev.append((s, e, "api", r.get("Function", "?"), r.get("Thread_Id", "")))
    for r in cp:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ev.append((s, e, "copy", r.get("Direction", r.get("Kind", "?")), ""))
    kern = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in kt)
    ev.sort()
    print("records: %d api, %d copies, %d kernels" % (len(api), len(cp), len(kt)))
    for s, e, kind, name, tid in ev:
        ms = (e - s) / 1e6
        if ms < thr:
            continue
        over = [k for k in kern if k[0] < e and k[1] > s]
        ks = "; ".join("%s %.2fms" % (k[2], (k[1] - k[0]) / 1e6) for k in over[:3])
        print("%10.3f ms  %8.3f ms  %-4s %-28s tid %s  | %d kernels overlap %s" %
              ((s - t0) / 1e6, ms, kind, name[:28], tid, len(over), ks))


if __name__ == "__main__":
    main()
