"""Per-dispatch kernel durations from a rocprofv3 SQLite output (rocpd).
Usage: python scripts/prof_db.py DB [name-substring] [--seq]"""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
rows = list(c.execute(f"select {name}, start, end, grid_x, grid_y from kernels order by start"))
if "--seq" in sys.argv:
    for n, s, e, gx, gy in rows:
        if pat in n:
            print("%-50s %9.2f us grid %d x %d" % (n[:50], (e - s) / 1e3, gx, gy))
else:
    agg = defaultdict(list)
    for n, s, e, gx, gy in rows:
        if pat in n:
            agg[(n, gx, gy)].append((e - s) / 1e3)
    for (n, gx, gy), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print("%-50s grid %8d x %3d  n %3d  avg %9.2f  min %9.2f us" % (n[:50], gx, gy, len(v), sum(v) / len(v), min(v)))
