"""T1 timing probe for A/B runs (GRKGPU_LIB selects the library build): the 8K
12-bit RGB frame, 9/7 and 5/3.  Lone frame: median device T1 time of 5
encodes / 5 decodes per codec.  Batch: 16 contexts (8 x 9/7, 8 x 5/3), each
on its own stream and host thread, encoding then decoding its frame 3 times;
wall time -> frames / s.  One JSON line."""
import json
import os
import statistics
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]

import torch  # noqa: E402

import grokimagecompression_amd as grk  # noqa: E402
import synth  # noqa: E402


def main():
    img = synth.synth_image(4320, 7680, 3, 12, 3)
    frame = torch.from_numpy(img).cuda()
    out = {}
    codec = grk.Codec(0)
    o = torch.empty_like(frame)
    for tag, irr in (("97", True), ("53", False)):
        p = grk.CParams.make(irreversible=irr)
        enc, dec = [], []
        for _ in range(6):
            b = bytes(codec.compress(frame, 12, p, view=True))
            enc.append(codec.stats()["t1_ms"])
            codec.decompress(b, out=o)
            dec.append(codec.stats()["t1_ms"])
        out["enc" + tag] = round(statistics.median(enc[1:]), 3)
        out["dec" + tag] = round(statistics.median(dec[1:]), 3)
    codecs = [grk.Codec(0) for _ in range(16)]
    streams = [torch.cuda.Stream() for _ in range(16)]
    outs = [torch.empty_like(frame) for _ in range(16)]
    params = [grk.CParams.make(irreversible=(i % 2 == 0)) for i in range(16)]

    def job(i, n):
        with torch.cuda.stream(streams[i]):
            for _ in range(n):
                b = codecs[i].compress(frame, 12, params[i], view=True)
                codecs[i].decompress(b, out=outs[i])
        torch.cuda.current_stream().synchronize()

    with ThreadPoolExecutor(16) as pool:
        list(pool.map(lambda i: job(i, 1), range(16)))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        list(pool.map(lambda i: job(i, 3), range(16)))
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    out["batch_mpix_s"] = round(16 * 3 * 4320 * 7680 / el / 1e6, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
