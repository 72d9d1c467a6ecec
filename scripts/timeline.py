"""Kernel timeline from a rocprofv3 db: busy fraction (union of kernel
intervals / span) and time-weighted mean number of concurrent kernels."""
import glob, os, sqlite3, sys
rows = []
for p in glob.glob(os.path.join(sys.argv[1], "**", "*.db"), recursive=True):
    c = sqlite3.connect(p)
    rows += c.execute("select start, end, name from kernels").fetchall()
rows.sort()
ev = []
for s, e, n in rows:
    ev.append((s, 1)); ev.append((e, -1))
ev.sort()
t0, t1 = ev[0][0], ev[-1][0]
cur, last, busy, area = 0, t0, 0, 0
hist = {}
for t, d in ev:
    if cur > 0:
        busy += t - last
    area += cur * (t - last)
    hist[cur] = hist.get(cur, 0) + (t - last)
    cur += d
    last = t
span = t1 - t0
print("span %.1f ms, busy %.1f%%, mean concurrent kernels %.2f" % (span / 1e6, 100 * busy / span, area / span))
print({k: round(100 * v / span, 1) for k, v in sorted(hist.items())})
