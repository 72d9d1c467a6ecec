"""Generate (or check) the tile-streaming fixtures with the REFERENCE codec.

Test infrastructure; runs only in the build container (needs oracle/_ref/
tile_driver, built from /root/reference by oracle/ref.mk).  The driver
restates the reference's own tile programs (oracle/tile_driver.cpp):
test_tile_encoder (ctest tte0..tte5), test_tile_decoder (ttd0..ttd2) and
j2k_random_tile_access (rta1..rta5), tests/CMakeLists.txt:92-124.  The .jp2
variants (tte2, ttd2, rta2) are left out: JP2 boxes are outside the path
(codestream/ row).

Stores:
  tests/golden/tiles/<case>.j2k  the reference's grk_write_tile codestream
  tests/golden/tiles.json        per case: encoder arguments, sha256 of the
      codestream; of the tile-by-tile decode without a decode area; of the
      random-access decode; and, for the ttd decode area (0,0,1024,1024), the
      tile headers only (index, rectangle, components, data size).  The
      reference's SAMPLES under a decode area are not the tile's (most
      code-blocks come out as zero coefficients; DESIGN.md "Tile streaming"),
      so they are not a parity target.

Usage:  python oracle/make_tile_golden.py [--check]
"""
import argparse
import hashlib
import json
import os
import struct
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = os.path.join(ROOT, "tests", "golden")
DRIVER = os.path.join(HERE, "_ref", "tile_driver")

# ctest name, test_tile_encoder arguments (tests/CMakeLists.txt:92-97; tte0 = the
# program's defaults, test_tile_encoder.cpp:128-136)
CASES = [
    ("tte0", [3, 2000, 2000, 1000, 1000, 8, 1]),
    ("tte1", [3, 2048, 2048, 1024, 1024, 8, 1]),
    ("tte3", [1, 2048, 2048, 1024, 1024, 8, 1]),
    ("tte4", [1, 256, 256, 128, 128, 8, 0]),
    ("tte5", [1, 512, 512, 256, 256, 8, 0]),
    # subsampled components through grk_write_tile / grk_read_tile_header /
    # grk_decode_tile_data (not a ctest case: the test_tile_encoder program
    # with its components on 2 x 2 / 2 x 1 grids)
    ("tte420", [3, 512, 512, 256, 256, 8, 1, "OUT", 420]),
    ("tte422_I", [3, 768, 512, 256, 256, 8, 0, "OUT", 422]),
]
AREA = [0, 0, 1024, 1024]  # ttd1 (tests/CMakeLists.txt:106)


def sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def tile_headers(path):
    """(index, x0, y0, x1, y1, ncomps, size) per tile of a `dec` output."""
    out = []
    with open(path, "rb") as f:
        while True:
            h = f.read(56)
            if not h:
                return out
            v = struct.unpack("<7Q", h)
            out.append(list(v))
            f.seek(v[6], 1)


def run(*args):
    r = subprocess.run([DRIVER] + [str(a) for a in args], capture_output=True, text=True, timeout=600)
    if r.returncode:
        sys.exit("tile_driver %s failed (%d): %s" % (" ".join(map(str, args)), r.returncode, r.stderr))


def generate(outdir):
    os.makedirs(os.path.join(outdir, "tiles"), exist_ok=True)
    man = {}
    with tempfile.TemporaryDirectory() as tmp:
        for name, args in CASES:
            j2k = os.path.join(outdir, "tiles", name + ".j2k")
            run("enc", *[j2k if a == "OUT" else a for a in args] + ([] if "OUT" in args else [j2k]))
            full, area, rta = (os.path.join(tmp, name + s) for s in (".full", ".area", ".rta"))
            run("dec", 0, 0, 0, 0, j2k, full)
            run("dec", *AREA, j2k, area)
            run("rta", j2k, rta)
            man[name] = {"args": args, "j2k_sha256": sha(j2k), "full_sha256": sha(full),
                         "full_bytes": os.path.getsize(full), "rta_sha256": sha(rta),
                         "rta_bytes": os.path.getsize(rta), "area": AREA, "area_tiles": tile_headers(area)}
    with open(os.path.join(outdir, "tiles.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    return man


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    if not os.path.exists(DRIVER):
        sys.exit("oracle/_ref/tile_driver not built: make -f oracle/ref.mk")
    if not a.check:
        generate(GOLD)
        return
    with tempfile.TemporaryDirectory() as tmp:
        man = generate(tmp)
        with open(os.path.join(GOLD, "tiles.json")) as f:
            committed = json.load(f)
        bad = [n for n in man if man[n] != committed.get(n)]
        if bad:
            sys.exit("tile fixtures differ: %s" % bad)
    print("tile fixtures match the reference")


if __name__ == "__main__":
    main()
