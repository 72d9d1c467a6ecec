"""Compare the bench line's roofline launches (HIP events) with rocprofv3's
kernel durations of the same run: the 10 k_dwt_fwd01 launches before the
last one are the roofline's lone 9/7 encodes (5 span-timed + 5 event-timed,
after the timed region); the last is the lone-frame T1 figure's encode.
  python scripts/roofline_check.py PROF_DIR BENCH_JSON"""
import glob
import json
import sqlite3
import sys


def main(d, bench):
    line = json.loads(open(bench).read().strip().splitlines()[-1])
    launches = line["roofline"]["launches"]
    db = glob.glob(d + "/**/*.db", recursive=True)[0]
    rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
    fwd01 = [(e - s) / 1e3 for n, s, e in rows if "k_dwt_fwd01<true" in n][-11:-1]
    print("k_dwt_fwd01<9/7>: rocprof mean of the roofline's 10 lone launches %.2f us (min %.2f, max %.2f); "
          "bench HIP events %.2f us" % (sum(fwd01) / len(fwd01), min(fwd01), max(fwd01), launches[0]["us"]))
    print("bench roofline frac %.4f (whole-frame DWT span %.2f us)" % (line["roofline"]["frac"], line["roofline"]["dwt_us"]))


if __name__ == "__main__":
    main(*sys.argv[1:3])
