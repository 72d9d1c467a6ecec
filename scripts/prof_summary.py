"""Summarise a rocprofv3 run (rocpd .db or *_kernel_stats.csv) into a CSV of
per-kernel calls / total / average / min / max duration (microseconds)."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(end-start)/1e3, avg(end-start)/1e3, min(end-start)/1e3, "
                     "max(end-start)/1e3 from kernels group by name order by sum(end-start) desc").fetchall()
    return rows


def main(d, out):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    rows = []
    for p in dbs:
        rows += from_db(p)
    tot = sum(r[2] for r in rows) or 1.0
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "pct"])
        for r in rows:
            name = r[0].split("(")[0]
            w.writerow([name, r[1], "%.1f" % r[2], "%.2f" % r[3], "%.2f" % r[4], "%.2f" % r[5], "%.2f" % (100 * r[2] / tot)])
    print(open(out).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
