"""C4 (16K 16-bit gray, 1024^2 tiles, 7 resolutions) on one GPU: the tile-shard
calls (compress_tiles with row0 / decompress_tiles) against compress /
decompress of the same image, with the codec's stage times."""
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
    H = W = 16384
    p, _ = grk.CParams.from_cli(["-t", "1024,1024", "-n", "7"])
    img = synth.synth_plane(H, W, 16, 4, 0, "smooth")[None]
    frame = torch.from_numpy(img).cuda()
    out = torch.empty_like(frame)
    codec = grk.Codec(0)

    def timeit(name, f, n=3):
        f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize()
            ts.append(1e3 * (time.perf_counter() - t0))
        st = codec.stats()
        print(json.dumps({"call": name, "ms": round(min(ts), 2),
                          "stats": {k: round(v, 3) if isinstance(v, float) else v for k, v in st.items()}}), flush=True)

    cs = {}
    timeit("compress(view)", lambda: cs.__setitem__("a", codec.compress(frame, 16, p, view=True)))
    timeit("compress_tiles(row0, view)", lambda: cs.__setitem__(
        "b", codec.compress_tiles(frame, 16, p, 0, 256, parts=grk.PART_ALL, row0=0, height=H, view=True)))
    a = bytes(cs["a"])
    timeit("decompress(out)", lambda: codec.decompress(a, out=out))
    timeit("decompress_tiles", lambda: codec.decompress_tiles(a, 0, 256, out))
    assert torch.equal(out, frame)
    print("ok", flush=True)


if __name__ == "__main__":
    main()
