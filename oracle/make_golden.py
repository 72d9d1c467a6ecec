"""Generate the golden fixtures under tests/golden/ from the REFERENCE codec.

Runs ONLY in the build container (never on the GPU box; nothing at test/bench
time imports this file).  It feeds images from tests/golden/synth.py to the
reference CLI (grk_compress / grk_decompress of Grok v5.1.0, built out of tree
from /root/reference by the survey step -- binaries located via $GRK_REF_BIN,
default /tmp/grkbuild/bin; this repo ships no recipe for that build, see
DESIGN.md "Oracle") and stores:

  tests/golden/<case>.j2k        reference codestream (byte-exact parity target)
  tests/golden/<case>.dec.npy    reference decode of that codestream, int32 (c,h,w)
  tests/golden/manifest.json     per case: image spec, grk_compress args,
                                 sha256 of input image / j2k / decoded image
  tests/golden/manifest_large.json  same hashes for the BASELINE.json configs
                                 (full-size streams are too big to commit)

Usage:  python oracle/make_golden.py [--large]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "..", "tests", "golden")
sys.path.insert(0, GOLD)
import synth  # noqa: E402

REF = os.environ.get("GRK_REF_BIN", "/tmp/grkbuild/bin")

# name, (h, w, c, bits), kind, seed, extra grk_compress args
CASES = [
    ("g8_64", (64, 64, 1, 8), "smooth", 11, []),
    ("g8_100x77", (77, 100, 1, 8), "smooth", 12, []),
    ("g8_256", (256, 256, 1, 8), "smooth", 13, []),
    ("g8_uniform_96", (96, 96, 1, 8), "uniform", 14, []),
    ("g8_const_64", (64, 64, 1, 8), "const", 15, []),
    ("g8_1x37", (37, 1, 1, 8), "smooth", 16, []),
    ("g8_45x1", (1, 45, 1, 8), "smooth", 17, []),
    ("g8_3x5", (5, 3, 1, 8), "uniform", 18, []),
    ("g8_n1", (48, 40, 1, 8), "smooth", 19, ["-n", "1"]),
    ("g8_n3", (48, 40, 1, 8), "smooth", 20, ["-n", "3"]),
    ("g8_n8", (70, 90, 1, 8), "smooth", 21, ["-n", "8"]),
    ("g8_b32", (130, 100, 1, 8), "smooth", 22, ["-b", "32,32"]),
    ("g8_b16x64", (100, 130, 1, 8), "smooth", 23, ["-b", "16,64"]),
    ("g8_b64x16", (100, 130, 1, 8), "smooth", 24, ["-b", "64,16"]),
    ("g8_b8", (24, 20, 1, 8), "uniform", 25, ["-b", "8,8"]),
    ("g8_off35", (61, 53, 1, 8), "smooth", 26, ["-d", "3,5"]),
    ("g8_off_tiles", (150, 200, 1, 8), "smooth", 27, ["-d", "7,3", "-t", "64,48", "-T", "5,1"]),
    ("g8_tiles64", (150, 200, 1, 8), "smooth", 28, ["-t", "64,64"]),
    ("g10_80x60", (60, 80, 1, 10), "smooth", 29, []),
    ("g12_70x50", (50, 70, 1, 12), "smooth", 30, []),
    ("g16_128", (128, 128, 1, 16), "smooth", 31, []),
    ("g16_uniform_64", (64, 64, 1, 16), "uniform", 32, []),
    ("rgb8_128x96", (96, 128, 3, 8), "smooth", 33, []),
    ("rgb8_uniform_64", (64, 64, 3, 8), "uniform", 34, []),
    ("rgb8_nomct", (64, 80, 3, 8), "smooth", 35, ["-Y", "0"]),
    ("rgb12_96x80", (80, 96, 3, 12), "smooth", 36, []),
    ("rgb16_64", (64, 64, 3, 16), "smooth", 37, []),
    # irreversible 9/7 (integer encode path, float decode path)
    ("g8_64_I", (64, 64, 1, 8), "smooth", 40, ["-I"]),
    ("g12_70x50_I", (50, 70, 1, 12), "smooth", 41, ["-I"]),
    ("g8_off_I", (61, 53, 1, 8), "smooth", 42, ["-I", "-d", "3,5"]),
    ("g8_n8_I", (70, 90, 1, 8), "smooth", 43, ["-I", "-n", "8"]),
    ("g8_uniform_I", (96, 96, 1, 8), "uniform", 44, ["-I"]),
    ("g16_I", (64, 64, 1, 16), "smooth", 45, ["-I"]),
    ("rgb8_I", (96, 128, 3, 8), "smooth", 46, ["-I"]),
    ("rgb12_I", (80, 96, 3, 12), "smooth", 47, ["-I"]),
    ("rgb12_tiles_I", (150, 200, 3, 12), "smooth", 48, ["-I", "-t", "64,64"]),
    ("g8_b32_I", (130, 100, 1, 8), "smooth", 49, ["-I", "-b", "32,32"]),
    ("g8_1x37_I", (37, 1, 1, 8), "smooth", 50, ["-I"]),
]

# BASELINE.json configs (hash-only; C5 cinema needs PCRD rate control -> next)
LARGE = [
    ("C1_512_gray8", (512, 512, 1, 8), "smooth", 1, []),
    ("C2_4k_rgb8", (2160, 3840, 3, 8), "smooth", 2, []),
    ("C3_8k_rgb12_I", (4320, 7680, 3, 12), "smooth", 3, ["-I"]),
    ("C3_8k_rgb12", (4320, 7680, 3, 12), "smooth", 3, []),
    ("C4_16k_gray16_tiled", (16384, 16384, 1, 16), "smooth", 4, ["-t", "1024,1024", "-n", "7"]),
]


def sha(b):
    return hashlib.sha256(b).hexdigest()


def run_case(name, shape, kind, seed, args, tmp, keep_files):
    h, w, c, bits = shape
    img = synth.synth_image(h, w, c, bits, seed, kind)
    ext = "ppm" if c == 3 else "pgm"
    src = os.path.join(tmp, f"{name}.{ext}")
    synth.write_pnm(src, img, bits)
    j2k = os.path.join(tmp, f"{name}.j2k")
    env = dict(os.environ, LD_LIBRARY_PATH=REF)
    subprocess.run([os.path.join(REF, "grk_compress"), "-i", src, "-o", j2k] + args,
                   check=True, env=env, stdout=subprocess.DEVNULL)
    raw = os.path.join(tmp, f"{name}.raw")
    subprocess.run([os.path.join(REF, "grk_decompress"), "-i", j2k, "-o", raw],
                   check=True, env=env, stdout=subprocess.DEVNULL)
    d = open(raw, "rb").read()
    dt = np.uint8 if bits <= 8 else np.dtype(">u2")
    dec = np.frombuffer(d, dtype=dt).reshape(c, h, w).astype(np.int32)
    jb = open(j2k, "rb").read()
    diff = (dec.astype(np.int64) - img).ravel()
    mse = float((diff.astype(np.float64) ** 2).mean())
    rec = dict(shape=[h, w, c, bits], kind=kind, seed=seed, args=args,
               image_sha256=synth.image_sha256(img), j2k_sha256=sha(jb), j2k_len=len(jb),
               dec_sha256=synth.image_sha256(dec),
               dec_vs_src_maxabs=int(np.abs(diff).max()) if diff.size else 0,
               dec_vs_src_mse=mse)
    if keep_files:
        open(os.path.join(GOLD, f"{name}.j2k"), "wb").write(jb)
        np.save(os.path.join(GOLD, f"{name}.dec.npy"), dec)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--large", action="store_true")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        if a.large:
            man = {}
            for case in LARGE:
                print("large", case[0], flush=True)
                man[case[0]] = run_case(*case, tmp, keep_files=False)
                for f in os.listdir(tmp):
                    os.unlink(os.path.join(tmp, f))
            json.dump(man, open(os.path.join(GOLD, "manifest_large.json"), "w"), indent=1)
        else:
            man = {}
            for case in CASES:
                man[case[0]] = run_case(*case, tmp, keep_files=True)
            json.dump(man, open(os.path.join(GOLD, "manifest.json"), "w"), indent=1)
    print("ok", len(man))


if __name__ == "__main__":
    main()
