"""Host analysis of the T1 decoder's lane utilisation (tests/cpp/t1_walk_sim.cpp):
a crop of the bench's synthetic 12-bit frame, 5/3 DWT by the C oracle,
64x64 code-blocks in the library's order (resolution, band, block raster),
coded by the oracle and decoded by the GPU walk compiled for the host.
  python scripts/t1_walk_sim.py [H W]"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "oracle")]

import pyoracle  # noqa: E402
import synth  # noqa: E402


def blocks(coef, numres):
    """(x0, y0, w, h, orient) of every 64x64 block of the Mallat layout."""
    H, W = coef.shape
    out = []
    hs = [H]
    ws = [W]
    for _ in range(numres - 1):
        hs.append((hs[-1] + 1) // 2)
        ws.append((ws[-1] + 1) // 2)
    L = numres - 1
    bands = [(0, 0, ws[L], hs[L], 0)]
    for d in range(L, 0, -1):  # coarse to fine
        lw, lh, fw, fh = ws[d], hs[d], ws[d - 1], hs[d - 1]
        bands += [(lw, 0, fw - lw, lh, 1), (0, lh, lw, fh - lh, 2), (lw, lh, fw - lw, fh - lh, 3)]
    for bx, by, bw, bh, o in bands:
        for y in range(0, bh, 64):
            for x in range(0, bw, 64):
                out.append((bx + x, by + y, min(64, bw - x), min(64, bh - y), o))
    return out


def main():
    H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (2048, 4096)
    q = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # drop q bit-planes (a lossy encode's quantisation)
    pyoracle.build()
    img = synth.synth_plane(H, W, 12, 3, 0, "smooth").astype(np.int32) - 2048
    coef = np.ascontiguousarray(img)
    pyoracle.dwt_fwd(coef, 0, 0, 6, False)
    if q:
        coef = (np.sign(coef) * (np.abs(coef) >> q)).astype(np.int32)
    exe = os.path.join(tempfile.gettempdir(), "t1_walk_sim")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas", "-o", exe,
                    os.path.join(ROOT, "tests/cpp/t1_walk_sim.cpp"), "-L" + os.path.join(ROOT, "oracle", "build"),
                    "-lgrk_oracle", "-Wl,-rpath," + os.path.join(ROOT, "oracle", "build")], check=True)
    bl = blocks(coef, 6)
    parts = [np.array([len(bl)], dtype="<u4").tobytes()]
    for x, y, w, h, o in bl:
        parts.append(np.array([w, h, o, 1, 0], dtype="<i4").tobytes())
        parts.append(np.ascontiguousarray(coef[y:y + h, x:x + w], dtype="<i4").tobytes())
    r = subprocess.run([exe], input=b"".join(parts), capture_output=True, check=True)
    print(r.stdout.decode().strip())
    print(r.stderr.decode().strip())


if __name__ == "__main__":
    main()
