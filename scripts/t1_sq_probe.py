"""One encode + one decode of the 8K 12-bit RGB 9/7 frame (for rocprofv3 --pmc
passes: scripts/gpu_sq.sh).  A call alone on the GPU packs 16 blocks per
wavefront (lone_bpw); the coders are forced to 64 per wavefront here, as under
the bench's 16 frames in flight, so the counters describe the batch's code
(argv[1] = "lone": keep the lone packing)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]

import torch  # noqa: E402

import grokimagecompression_amd as grk  # noqa: E402
import synth  # noqa: E402

t = torch.from_numpy(synth.synth_image(4320, 7680, 3, 12, 3)).cuda()
codec = grk.Codec(0)
bpw = 0 if sys.argv[1:] == ["lone"] else 64
with grk.dwt_options(t1_dec_bpw=bpw, t1_enc_bpw=bpw):
    b = bytes(codec.compress(t, 12, grk.CParams.make(irreversible=True), view=True))
    o = torch.empty_like(t)
    codec.decompress(b, out=o)
torch.cuda.synchronize()
print("ok", len(b), flush=True)
