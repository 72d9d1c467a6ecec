"""DWT timing probe on the GPU box: encode+decode the 8K 12-bit RGB frame
(9/7 and 5/3) through the codec and report the DWT event times.  With
--sweep, rerun in child processes for each GRKGPU_DWT_TH value."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]


def one():
    import torch
    import grokimagecompression_amd as grk
    import synth
    img = synth.synth_image(4320, 7680, 3, 12, 3)
    t = torch.from_numpy(img).cuda()
    codec = grk.Codec(0)
    out = {}
    for irrev in (True, False):
        p = grk.CParams.make(irreversible=irrev)
        res = []
        for _ in range(4):
            b = codec.compress(t, 12, p, view=True)
            e = codec.stats()["dwt_ms"]
            mct = codec.stats()["dcshift_mct_ms"]
            o = torch.empty_like(t)
            codec.decompress(b, out=o)
            d = codec.stats()["dwt_ms"]
            res.append((e, d, mct))
        out["97" if irrev else "53"] = {"enc_dwt_ms": round(min(r[0] for r in res), 4),
                                        "dec_dwt_ms": round(min(r[1] for r in res), 4),
                                        "mct_ms": round(min(r[2] for r in res), 4)}
    print(json.dumps(out), flush=True)


def stage():
    """Stage entry point only (for rocprofv3 --pmc): forward + inverse DWT of
    three 8K planes, 9/7 then 5/3."""
    import numpy as np
    import torch
    import grokimagecompression_amd as grk
    rng = np.random.default_rng(0)
    a = torch.from_numpy(rng.integers(-(1 << 20), 1 << 20, size=(4320, 7680)).astype(np.int32)).cuda()
    for irrev in (True, False):
        for _ in range(3):
            t = a.clone()
            grk.dwt_fwd(t, 0, 0, 6, irrev)
            grk.dwt_inv(t, 0, 0, 6, irrev)
    torch.cuda.synchronize()
    print("stage ok", flush=True)


if __name__ == "__main__":
    if "--stage" in sys.argv:
        stage()
    elif "--sweep" in sys.argv:
        # each remaining argument: comma-separated ENV=VALUE settings of one run
        specs = [a for a in sys.argv[1:] if a != "--sweep"] or ["GRKGPU_DWT_STRIP=0"]
        for spec in specs:
            env = dict(os.environ)
            for kv in filter(None, spec.split(",")):
                k, v = kv.split("=", 1)
                env[k] = v
            print("==", spec, flush=True)
            subprocess.run([sys.executable, __file__], env=env, check=True, timeout=300)
    else:
        one()
