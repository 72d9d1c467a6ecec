"""DWT span A/B on one box: the 8K 9/7 frame's forward DWT (HIP events before
the first / after the last level launch, no per-launch events), alternating
grkgpu_dwt_options settings; mean of 10 encodes per setting and round.
  python scripts/dwt_span_ab.py - "f01_small_min_samples=18446744073709551615"   ("-": the defaults)
  python scripts/dwt_span_ab.py --inverse - inv01=0 inv01=4   (the decode's inverse DWT)"""
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
        if kv in ("-", "default", '""'):
            continue
        k, v = kv.split("=", 1)
        d[k] = int(v)
    return d


def main():
    inverse = "--inverse" in sys.argv
    specs = [a for a in sys.argv[1:] if a != "--inverse"] or [""]
    t = torch.from_numpy(synth.synth_image(4320, 7680, 3, 12, 3)).cuda()
    codec = grk.Codec(0)
    p = grk.CParams.make(irreversible=True)
    cs = codec.compress(t, 12, p)
    out = torch.empty_like(t)
    res = {s: [] for s in specs}
    for _ in range(3):
        for s in specs:
            with grk.dwt_options(**opts(s)):
                for k in range(11):
                    if inverse:
                        codec.decompress(cs, out=out)
                    else:
                        codec.compress(t, 12, p, view=True)
                    if k:
                        res[s].append(1e3 * codec.stats()["dwt_ms"])
    print(json.dumps({s or "(default)": {"mean_us": round(statistics.mean(v), 2), "median_us": round(statistics.median(v), 2)}
                      for s, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
