"""Compare the bench line's roofline with rocprofv3's kernel durations of the
same launches in the same run.  Each 9/7 encode launches one k_dwt_fwd01
(levels 0 + 1) and one k_dwt_fwd per further level.  The forward launches of
the run end with: 6 span-timed encodes (events around the level sequence
only; the first is a warm-up), the encode whose stream the decode timing
uses, 6 launch-timed encodes (an event after every launch; the first a
warm-up), then the lone-frame T1 figure's encode.
The inverse launches (k_dwt_inv per level, then k_dwt_inv01 for the last two)
end with 6 span-timed decodes, 6 launch-timed decodes, then the lone-frame
T1 figure's decode.
  python scripts/roofline_check.py PROF_DIR BENCH_JSON"""
import glob
import json
import sqlite3
import sys


def main(d, bench):
    line = json.loads(open(bench).read().strip().splitlines()[-1])
    rl = line["roofline"]
    launches = rl["launches"]
    n = len(launches)
    db = glob.glob(d + "/**/*.db", recursive=True)[0]
    rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
    fwd = [(n_, s, e) for n_, s, e in rows if "k_dwt_fwd01<true" in n_ or "k_dwt_fwd<true" in n_]

    def enc(sel):
        runs = [sel[i * n:(i + 1) * n] for i in range(len(sel) // n)]
        ksum = [sum((e - s) / 1e3 for _, s, e in r) for r in runs]
        span = [(r[-1][2] - r[0][1]) / 1e3 for r in runs]
        return ksum, span

    lk, ls = enc(fwd[-6 * n:-n])        # launch-timed encodes 2..6
    sk, ss = enc(fwd[-13 * n:-8 * n])   # span-timed encodes 2..6
    first = [fwd[-6 * n + i * n] for i in range(5)]
    mean = lambda v: sum(v) / len(v)
    print("forward 9/7 DWT of the frame (%d launches):" % n)
    print("  span-timed encodes: bench span_us %.2f; rocprof kernel sum %.2f (min %.2f, max %.2f), first start to "
          "last end %.2f" % (rl["span_us"], mean(sk), min(sk), max(sk), mean(ss)))
    print("  launch-timed encodes: bench per-launch sum dwt_us %.2f; rocprof kernel sum %.2f, first start to last "
          "end %.2f" % (rl["dwt_us"], mean(lk), mean(ls)))
    print("  %s: rocprof %.2f us, bench %.2f us" % (launches[0]["kernel"], mean([(e - s) / 1e3 for _, s, e in first]),
                                                   launches[0]["us"]))
    b = rl["algorithmic_bytes"]
    print("bench roofline frac %.4f (span); by rocprof kernel sum %.4f, by rocprof span %.4f"
          % (rl["frac"], b / (mean(sk) * 1e-6) / 8e12, b / (mean(ss) * 1e-6) / 8e12))
    inv = rl["inverse"]
    m = len(inv["launches"])
    ifw = [(n_, s, e) for n_, s, e in rows if "k_dwt_inv<true" in n_ or "k_dwt_inv01<true" in n_]
    n = m
    ik, iss = enc(ifw[-12 * m:-7 * m])  # span-timed decodes 2..6
    lk2, _ = enc(ifw[-6 * m:-m])         # launch-timed decodes 2..6
    print("inverse 9/7 DWT of the frame (%d launches): bench span_us %.2f, rocprof kernel sum %.2f (first start to "
          "last end %.2f); launch-timed: bench dwt_us %.2f, rocprof kernel sum %.2f"
          % (m, inv["span_us"], mean(ik), mean(iss), inv["dwt_us"], mean(lk2)))
    print("bench inverse frac %.4f (span); by rocprof kernel sum %.4f" % (inv["frac"], b / (mean(ik) * 1e-6) / 8e12))


if __name__ == "__main__":
    main(*sys.argv[1:3])
