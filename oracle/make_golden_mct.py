"""Custom-MCT fixtures (Part 2 array-based MCT, grk_set_MCT, grok.cpp:606):
images encoded by the REFERENCE (oracle/_ref/ref_driver -mct, which calls
grk_set_MCT with the matrix and DC shifts given) -- the encoding matrix in
13-bit fixed point (mct.cpp:429-475), its float inverse from
matrix_inversion_f in CBD / MCT / MCC / MCO marker segments
(j2k.cpp:2580-2741, 5615-6333), rate control weighted by the inverse's
column norms.  The reference's own decoder refuses these streams (COD MCT
byte 2: "Invalid MCT value", j2k.cpp:3869-3872), so each fixture records
that refusal instead of a decode.
Writes tests/golden/mct_<name>.j2k and manifest_mct.json.
  python oracle/make_golden_mct.py [--check]"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE]

import make_golden as mg  # noqa: E402

YCC = "0.299,0.587,0.114,-0.16875,-0.33126,0.5,0.5,-0.41869,-0.08131"
M4 = "0.5,0.25,0.125,0.125,-0.5,0.5,0,0,0.1,0.2,0.3,0.4,0,0,-1,1"
# name, (h, w, c, bits), kind, seed, options
CASES = [
    ("rgb8_ycc", (64, 80, 3, 8), "smooth", 601, ["-mct", YCC + ":128,128,128"]),
    ("rgb8_ycc_uniform", (64, 64, 3, 8), "uniform", 602, ["-mct", YCC + ":128,128,128"]),
    ("rgba8_m4_tiles", (100, 130, 4, 8), "smooth", 603, ["-mct", M4 + ":128,128,128,0", "-t", "64,64"]),
    ("rgb12_ycc_r", (96, 128, 3, 12), "smooth", 604, ["-mct", YCC + ":2048,2048,2048", "-r", "20,5"]),
    ("rgb12_ycc_q", (80, 96, 3, 12), "smooth", 605, ["-mct", YCC + ":2048,0,-7", "-q", "30,45", "-n", "4"]),
    ("g16_scale", (64, 70, 1, 16), "smooth", 606, ["-mct", "0.75:32768", "-r", "10"]),
]


def main():
    check = "--check" in sys.argv
    mg.build_ref()
    path = os.path.join(mg.GOLD, "manifest_mct.json")
    old = json.load(open(path)) if os.path.exists(path) else {}
    man, bad = {}, 0
    with tempfile.TemporaryDirectory() as tmp:
        for name, (h, w, c, bits), kind, seed, args in CASES:
            tag = "mct_" + name
            img = mg.synth.synth_image(h, w, c, bits, seed, kind)
            cs = mg.ref_encode(img, bits, args, tmp)
            try:
                mg.ref_decode(cs, tmp)
                dec = "decoded"
            except subprocess.CalledProcessError:
                dec = "error"
            rec = dict(shape=[h, w, c, bits], kind=kind, seed=seed, args=args, image_sha256=mg.synth.image_sha256(img),
                       j2k_sha256=mg.sha(cs), j2k_len=len(cs), dec=dec)
            man[tag] = rec
            if check:
                ok = old.get(tag) == rec and open(os.path.join(mg.GOLD, tag + ".j2k"), "rb").read() == cs
                print(tag, "ok" if ok else "MISMATCH", flush=True)
                bad += not ok
                continue
            with open(os.path.join(mg.GOLD, tag + ".j2k"), "wb") as f:
                f.write(cs)
            print(tag, len(cs), dec, flush=True)
    if check:
        print("mismatches", bad)
        sys.exit(1 if bad else 0)
    with open(path, "w") as f:
        json.dump(man, f, indent=1)


if __name__ == "__main__":
    main()
