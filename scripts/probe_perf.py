"""Quick per-stage timing probe on the GPU box (not the bench)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np
import torch
import grokimagecompression_amd as grk
import synth

# arguments: configs ("512", "4k", "8k", "16k") and plan options key=value
# (grkgpu_dwt_options fields, e.g. t1_dec_sort=1 f64_lift=1) for the whole run
opts = dict(a.split("=") for a in sys.argv[1:] if "=" in a)
configs = [a for a in sys.argv[1:] if "=" not in a] or ["4k", "8k"]
if opts:
    grk.dwt_options(**{k: int(v) for k, v in opts.items()}).__enter__()
    print("options", opts, flush=True)
codec = grk.Codec(0)
dcodec = grk.Codec(0)  # decode context: reads the encoder's pinned output in place
for cfg in configs:
    kw = {}
    if cfg == "512":  # BASELINE configs[0]
        h, w, c, bits, modes, seed = 512, 512, 1, 8, [False], 1
    elif cfg == "4k":  # configs[1]
        h, w, c, bits, modes, seed = 2160, 3840, 3, 8, [False], 2
    elif cfg == "16k":  # configs[3]: 1024^2 tiles, 7 resolutions (6 DWT levels)
        h, w, c, bits, modes, seed = 16384, 16384, 1, 16, [False], 4
        kw = dict(numresolution=7, tiles=(1024, 1024))
    else:  # configs[2]
        h, w, c, bits, modes, seed = 4320, 7680, 3, 12, [True, False], 3
    img = synth.synth_image(h, w, c, bits, seed)
    t = torch.from_numpy(img).cuda()
    del img
    for irrev in modes:
        p = grk.CParams.make(irreversible=irrev, **kw)
        for it in range(3):
            torch.cuda.synchronize()
            t0 = time.time()
            # zero-copy result (a view of the context's pinned output buffer):
            # the latency of the codec, not of copying 100 MB into a new bytes
            b = codec.compress(t, bits, p, view=True)
            t1 = time.time()
            se = codec.stats()
            out = dcodec.decompress(b, device_out=True)
            torch.cuda.synchronize()
            t2 = time.time()
            sd = dcodec.stats()
        ok = irrev or torch.equal(out, t)
        print(f"{cfg} irrev={irrev} bytes={b.size} enc {1e3*(t1-t0):.1f} ms dec {1e3*(t2-t1):.1f} ms "
              f"Mpix/s={h*w/1e6/(t2-t0):.1f} lossless_ok={ok}", flush=True)
        print("  enc", {k: round(v, 3) if isinstance(v, float) else v for k, v in se.items()}, flush=True)
        print("  dec", {k: round(v, 3) if isinstance(v, float) else v for k, v in sd.items()}, flush=True)
