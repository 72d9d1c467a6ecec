"""A few 8K encodes under one grkgpu_dwt_options setting, for rocprofv3
counter passes on the DWT kernels (scripts/gpu_run.sh dwtpmc).
  python scripts/dwt_enc_once.py 97|53 [k=v ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]

import torch  # noqa: E402

import grokimagecompression_amd as grk  # noqa: E402
import synth  # noqa: E402

irrev = sys.argv[1] == "97"
opts = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in sys.argv[2:]}
t = torch.from_numpy(synth.synth_image(4320, 7680, 3, 12, 3)).cuda()
codec = grk.Codec(0)
p = grk.CParams.make(irreversible=irrev)
with grk.dwt_options(**opts):
    for _ in range(3):
        codec.compress(t, 12, p, view=True)
torch.cuda.synchronize()
print("ok", flush=True)
