"""Forward-DWT launch times of the 8K frame (9/7 and 5/3) under several
grkgpu_dwt_options settings, alternating settings per round: per launch the
mean device time of 10 encodes (grkgpu_set_launch_timing) and the frame's
sum, with the B_DWT fraction of 8 TB/s.
  python scripts/dwt_pair_probe.py - pair_kernel=0 pair_rows=126 ..."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]

import torch  # noqa: E402

import grokimagecompression_amd as grk  # noqa: E402
import synth  # noqa: E402


def opts(spec):
    d = {}
    for kv in filter(None, spec.split(",")):
        if kv in ("-", "default"):
            continue
        k, v = kv.split("=", 1)
        d[k] = int(v)
    return d


def main():
    specs = sys.argv[1:] or ["-"]
    t = torch.from_numpy(synth.synth_image(4320, 7680, 3, 12, 3)).cuda()
    codec = grk.Codec(0)
    codec.set_launch_timing(True)
    res = {}
    for _ in range(2):
        for irrev in (True, False):
            p = grk.CParams.make(irreversible=irrev)
            for s in specs:
                key = ("97 " if irrev else "53 ") + s
                with grk.dwt_options(**opts(s)):
                    for k in range(6):
                        codec.compress(t, 12, p, view=True)
                        if k:
                            res.setdefault(key, []).append(codec.launch_times())
    out = {}
    for key, runs in res.items():
        n = len(runs[0])
        per = []
        for i in range(n):
            ms = [r[i]["ms"] for r in runs]
            per.append("%s L%d+%d %.1fus" % (runs[0][i]["kernel"], runs[0][i]["level0"], runs[0][i]["levels"],
                                               1e3 * statistics.mean(ms)))
        tot = [sum(x["ms"] for x in r) for r in runs]
        b = sum(x["bytes"] for x in runs[0])
        out[key] = {"sum_us": round(1e3 * statistics.mean(tot), 1), "frac": round(b / (statistics.mean(tot) * 1e-3) / 8e12, 4),
                    "launches": per}
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
