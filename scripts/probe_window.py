"""Window decode latency (grk_set_decode_area / grkgpu_decompress_window) on
the 8K 12-bit RGB frame (9/7 and 5/3, one tile): the full decode against
windows of 256^2 .. 2048^2 in the middle; stats of the last of 5 decodes."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]

import torch  # noqa: E402

import grokimagecompression_amd as grk  # noqa: E402
import synth  # noqa: E402


def main():
    t = torch.from_numpy(synth.synth_image(4320, 7680, 3, 12, 3)).cuda()
    codec = grk.Codec(0)
    res = {}
    for irrev in (True, False):
        cs = codec.compress(t, 12, grk.CParams.make(irreversible=irrev))
        for side in (0, 256, 1024, 2048):
            win = None if not side else (3840 - side // 2, 2160 - side // 2, 3840 + side // 2, 2160 + side // 2)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                codec.decompress(cs, device_out=True, window=win)
                torch.cuda.synchronize()
                ts.append(1e3 * (time.perf_counter() - t0))
            st = codec.stats()
            res["%s %s" % ("9/7" if irrev else "5/3", side or "full")] = {
                "wall_ms": round(min(ts), 2), "t1_ms": round(st["t1_ms"], 3), "idwt_ms": round(st["dwt_ms"], 3),
                "cblks": st["num_cblks"]}
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
