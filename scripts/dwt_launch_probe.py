"""Per-launch forward DWT times on the GPU box (HIP events, grkgpu_set_launch_timing):
the 8K 12-bit RGB frame, 9/7 and 5/3 encodes, mean over N runs.  Each argument is
a comma-separated list of grkgpu_dwt_options fields (NAME=VALUE); every spec
runs in its own child process.
  python scripts/dwt_launch_probe.py "" "f01_small_min_samples=1048576" ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]


def one(n=8):
    import torch
    import grokimagecompression_amd as grk
    import synth
    img = synth.synth_image(4320, 7680, 3, 12, 3)
    t = torch.from_numpy(img).cuda()
    codec = grk.Codec(0)
    codec.set_launch_timing(True)
    opts = {}
    for kv in filter(None, os.environ.get("DWT_OPTS", "").split(",")):
        k, v = kv.split("=", 1)
        opts[k] = int(v)
    grk.dwt_options(**opts).__enter__()
    out = {}
    for irrev in (True, False):
        p = grk.CParams.make(irreversible=irrev)
        runs = []
        for i in range(n + 1):
            codec.compress(t, 12, p, view=True)
            if i:
                runs.append((codec.stats()["dwt_ms"], codec.launch_times()))
        ls = []
        for k, l in enumerate(runs[0][1]):
            ms = sum(r[1][k]["ms"] for r in runs) / n
            ls.append("%s L%d+%d %.1fus %.2fTB/s" % (l["kernel"], l["level0"], l["levels"], 1e3 * ms,
                                                  l["bytes"] / (ms * 1e-3) / 1e12))
        tot = sum(sum(x["ms"] for x in r[1]) for r in runs) / n
        span = sum(r[0] for r in runs) / n
        out["97" if irrev else "53"] = {"kernels_us": round(1e3 * tot, 1), "span_us": round(1e3 * span, 1),
                                        "launches": ls}
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        one()
        sys.exit(0)
    for spec in sys.argv[1:] or [""]:
        env = dict(os.environ, DWT_OPTS=spec)
        print("==", spec or "(default)", flush=True)
        subprocess.run([sys.executable, __file__, "--one"], env=env, check=True, timeout=300)
