"""Print every PMC counter of every kernel in rocprofv3 rocpd databases (one row per kernel).

usage: python profiles/pmc_report.py DB [DB ...]   (counters averaged over dispatches)"""
import sqlite3
import sys


def main():
    rows = {}
    for db in sys.argv[1:]:
        con = sqlite3.connect(db)
        for k, c, v, n, d in con.execute("select kernel_name, counter_name, avg(value), count(*), avg(duration) "
                                         "from counters_collection group by kernel_name, counter_name"):
            rows.setdefault(k, {"_us": d / 1e3, "_n": n})[c] = v
    for k, cs in sorted(rows.items(), key=lambda t: -t[1]["_us"]):
        print("%s  (%d dispatches, %.1f us)" % (k[:100], cs.pop("_n"), cs.pop("_us")))
        for c in sorted(cs):
            print("    %-28s %.6g" % (c, cs[c]))


if __name__ == "__main__":
    main()
