"""Kernel summary (name, calls, total/avg/min/max ns, %) from a rocprofv3 --kernel-trace database.

Usage: python java-rsync_amd/tools/prof_summary.py <results.db> <out.csv>
"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                          "max(end - start) from kernels group by name order by sum(end - start) desc"))
    total = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
        for name, calls, tot, avg, mn, mx in rows:
            w.writerow([name, calls, tot, round(avg, 1), mn, mx, round(100.0 * tot / total, 3)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
