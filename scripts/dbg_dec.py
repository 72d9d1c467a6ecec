"""Lossless round trip of a large config (decoded == source), with the
mismatch located: per component, the count and the bounding box of the
differing samples and the 64x64 code-block grid cells they fall in.
  python scripts/dbg_dec.py C2_4k_rgb8 [C1_512_gray8 ...]"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import synth  # noqa: E402
from conftest import load_manifest  # noqa: E402
import grokimagecompression_amd as grk  # noqa: E402
import torch  # noqa: E402

LARGE = load_manifest(large=True)
c = grk.Codec(0)
for name in sys.argv[1:]:
    m = LARGE[name]
    h, w, nc, bits = m["shape"]
    img = synth.synth_image(h, w, nc, bits, m["seed"], m["kind"])
    p, off = grk.CParams.from_cli(m["args"])
    b = c.compress(torch.from_numpy(img).cuda(), bits, p, offset=off)
    d = np.asarray(c.decompress(b))
    d = d.reshape(img.shape) if d.size == img.size else d
    print(name, "lib", os.environ.get("GRKGPU_LIB", "default"), "cs", len(b), "cs hash ok",
          hashlib.sha256(bytes(b)).hexdigest() == m["j2k_sha256"], "dec shape", d.shape, flush=True)
    for k in range(nc):
        a = img[k] if img.ndim == 3 and img.shape[0] == nc else img[..., k]
        e = d[k] if d.ndim == 3 and d.shape[0] == nc else d[..., k]
        diff = a.astype(np.int64) != e.astype(np.int64)
        n = int(diff.sum())
        if not n:
            print("  comp", k, "exact")
            continue
        ys, xs = np.nonzero(diff)
        cells = sorted(set(zip((ys // 64).tolist(), (xs // 64).tolist())))
        print("  comp", k, "diff", n, "bbox y", ys.min(), ys.max(), "x", xs.min(), xs.max(), "cells", len(cells), cells[:12])
        print("  first", [(int(y), int(x), int(a[y, x]), int(e[y, x])) for y, x in list(zip(ys, xs))[:6]])
c.close()
