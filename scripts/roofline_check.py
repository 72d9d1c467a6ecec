"""Compare the bench line's roofline (HIP-event device times of the 9/7
forward DWT launches of 5 lone encodes after the timed region) with
rocprofv3's kernel durations of the same launches in the same run.  Each 9/7
encode launches one k_dwt_fwd01 (levels 0 + 1) and one k_dwt_fwd per further
level; the last encode of the run is the lone-frame T1 figure's, the 5 before
it the roofline's event-timed ones.
  python scripts/roofline_check.py PROF_DIR BENCH_JSON"""
import glob
import json
import sqlite3
import sys


def main(d, bench):
    line = json.loads(open(bench).read().strip().splitlines()[-1])
    launches = line["roofline"]["launches"]
    n = len(launches)
    db = glob.glob(d + "/**/*.db", recursive=True)[0]
    rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
    fwd = [(n_, (e - s) / 1e3) for n_, s, e in rows if "k_dwt_fwd01<true" in n_ or "k_dwt_fwd<true" in n_]
    sel = fwd[-6 * n:-n]  # the 5 event-timed encodes before the last one
    per = [sum(d_ for _, d_ in sel[i * n:(i + 1) * n]) for i in range(5)]
    first = [sel[i * n][1] for i in range(5)]
    print("forward 9/7 DWT of the frame: rocprof mean of the roofline's 5 lone encodes %.2f us (min %.2f, max %.2f); "
          "bench HIP events %.2f us" % (sum(per) / 5, min(per), max(per), line["roofline"]["dwt_us"]))
    print("  %s: rocprof %.2f us, bench %.2f us" % (launches[0]["kernel"], sum(first) / 5, launches[0]["us"]))
    print("bench roofline frac %.4f; by rocprof %.4f" % (line["roofline"]["frac"],
                                                       line["roofline"]["algorithmic_bytes"] / (sum(per) / 5 * 1e-6) / 8e12))


if __name__ == "__main__":
    main(*sys.argv[1:3])
