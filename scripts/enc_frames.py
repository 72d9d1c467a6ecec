"""Encode (and optionally decode) the bench's 8K 12-bit RGB frame a few times
on one context -- a short, fixed workload for rocprofv3 counter passes.
  python scripts/enc_frames.py [N=3] [97|53] [dec]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]

import torch  # noqa: E402

import grokimagecompression_amd as grk  # noqa: E402
import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
irrev = (sys.argv[2] if len(sys.argv) > 2 else "97") == "97"
dec = len(sys.argv) > 3 and sys.argv[3] == "dec"
t = torch.from_numpy(synth.synth_image(4320, 7680, 3, 12, 3)).cuda()
codec = grk.Codec(0)
p = grk.CParams.make(irreversible=irrev)
out = torch.empty_like(t)
for _ in range(n):
    cs = codec.compress(t, 12, p)
    if dec:
        codec.decompress(cs, out=out)
torch.cuda.synchronize()
print("frames", n, "bytes", len(cs), flush=True)
