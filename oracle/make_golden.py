"""Generate (or check) the golden fixtures under tests/golden/ with the REFERENCE codec.

Test infrastructure; runs only in the build container (the GPU box has no
/root/reference).  The reference is Grok v5.1.0's own libgrok, compiled
straight from /root/reference/src/lib/jp2 by the committed recipe
oracle/ref.mk (no CMake, no stand-ins), driven through its grk_* C API by
oracle/ref_driver.cpp (the grk_compress / grk_decompress option mapping for
the options below).  Images come from tests/golden/synth.py.

Stores:
  tests/golden/<case>.j2k        reference codestream (byte-exact parity target)
  tests/golden/<case>.dec.npy    reference decode of that codestream, int32 (c,h,w)
  tests/golden/manifest.json     per case: image spec, grk_compress args,
                                 sha256 of input image / j2k / decoded image
  tests/golden/manifest_large.json  same hashes for the BASELINE.json configs
                                 (full-size streams are too big to commit)

Usage:  python oracle/make_golden.py [--large] [--check] [--only NAME ...]
  --check  regenerate into a temporary directory and compare with the
           committed files instead of overwriting them (exit 1 on a mismatch)
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
ROOT = os.path.dirname(HERE)
GOLD = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, GOLD)
import synth  # noqa: E402

DRIVER = os.path.join(HERE, "_ref", "ref_driver")

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
    # round 2: quality layers + rate control (PCRD), precincts, progressions,
    # POC, SOP / EPH, tile-parts, cinema profiles
    ("g8_r40_20_10", (96, 128, 1, 8), "smooth", 60, ["-r", "40,20,10"]),
    ("g8_r5", (100, 77, 1, 8), "uniform", 61, ["-r", "5"]),
    ("rgb8_r20_I", (96, 128, 3, 8), "smooth", 62, ["-I", "-r", "20"]),
    ("rgb12_r30_10_1_I", (80, 96, 3, 12), "smooth", 63, ["-I", "-r", "30,10,1"]),
    ("g12_r8_A1", (70, 90, 1, 12), "smooth", 64, ["-r", "16,8", "-A", "1"]),
    ("rgb8_r10_tiles", (150, 200, 3, 8), "smooth", 65, ["-r", "10", "-t", "64,64"]),
    ("g8_prec", (130, 100, 1, 8), "smooth", 66, ["-c", "[32,32],[16,16]"]),
    ("rgb8_prec_rpcl", (96, 128, 3, 8), "smooth", 67, ["-c", "[64,64],[32,32]", "-p", "RPCL"]),
    ("rgb8_prec_pcrl", (96, 128, 3, 8), "smooth", 68, ["-c", "[64,64],[32,32]", "-p", "PCRL"]),
    ("rgb8_prec_cprl", (96, 128, 3, 8), "smooth", 69, ["-c", "[64,64],[32,32]", "-p", "CPRL"]),
    ("rgb8_rlcp_layers", (96, 128, 3, 8), "smooth", 70, ["-p", "RLCP", "-r", "30,10"]),
    ("g8_sop_eph", (96, 128, 1, 8), "smooth", 71, ["-S", "-E", "-r", "20,5"]),
    ("rgb8_tp_R", (96, 128, 3, 8), "smooth", 72, ["-u", "R", "-r", "8"]),
    ("rgb8_tp_C_cprl", (96, 128, 3, 8), "smooth", 73, ["-u", "C", "-p", "CPRL", "-c", "[32,32]"]),
    ("rgb8_tp_L", (96, 128, 3, 8), "smooth", 74, ["-u", "L", "-r", "30,10,3"]),
    ("rgb8_poc", (96, 128, 3, 8), "smooth", 75, ["-P", "T1=0,0,1,3,3,LRCP/T1=3,0,1,6,3,RPCL"]),
    ("rgb12_cinema4k", (216, 384, 3, 12), "smooth", 76, ["-cinema4K", "24"]),
    ("rgb12_cinema2k", (108, 192, 3, 12), "smooth", 77, ["-cinema2K", "24"]),
    ("rgb12_cinema4k_48", (120, 256, 3, 12), "uniform", 78, ["-cinema4K", "48"]),
    # rate control over precinct partitions / POC (plugin-tree coverage)
    ("rgb8_prec_r20_rpcl", (150, 200, 3, 8), "smooth", 79, ["-c", "[32,32],[16,16]", "-p", "RPCL", "-r", "20,5"]),
    ("g12_prec_r12_A1", (130, 170, 1, 12), "smooth", 80, ["-c", "[64,64],[32,32],[16,16]", "-r", "12", "-A", "1",
                                                          "-b", "32,32"]),
    ("rgb8_poc_r15_I", (96, 128, 3, 8), "smooth", 81, ["-I", "-r", "15,4",
                                                       "-P", "T1=0,0,2,3,3,CPRL/T1=3,0,2,6,3,LRCP"]),
    # code-block mode switches (-M: 2 RESET, 4 RESTART = terminate every pass,
    # 8 VSC, 16 PTERM = predictable termination, 32 SEGSYM)
    ("g8_M2_reset", (96, 128, 1, 8), "smooth", 90, ["-M", "2"]),
    ("g8_M8_vsc", (96, 128, 1, 8), "smooth", 91, ["-M", "8"]),
    ("g8_M32_segsym", (96, 128, 1, 8), "smooth", 92, ["-M", "32"]),
    ("g8_M4_termall", (96, 128, 1, 8), "smooth", 93, ["-M", "4"]),
    ("g8_M16_pterm", (96, 128, 1, 8), "smooth", 94, ["-M", "16"]),
    ("g8_M20_termall_pterm", (96, 128, 1, 8), "uniform", 95, ["-M", "20"]),
    ("g8_M8_vsc_odd", (77, 100, 1, 8), "uniform", 98, ["-M", "8"]),
    ("rgb8_M62_I_r", (96, 128, 3, 8), "smooth", 96, ["-M", "62", "-I", "-r", "20,5"]),
    ("rgb12_M46_tiles", (150, 200, 3, 12), "smooth", 97, ["-M", "46", "-t", "64,64"]),
    ("g12_M4_layers", (70, 90, 1, 12), "smooth", 99, ["-M", "4", "-r", "16,4,1"]),
    ("g8_M42_b16", (100, 130, 1, 8), "smooth", 100, ["-M", "42", "-b", "16,16", "-r", "12,3"]),
    # BYPASS (-M 1): raw significance / refinement passes below the top four bit-planes
    ("g8_M1_lazy", (96, 128, 1, 8), "smooth", 101, ["-M", "1"]),
    ("g12_M1_lazy", (70, 90, 1, 12), "uniform", 102, ["-M", "1"]),
    ("rgb8_M1_I_r", (96, 128, 3, 8), "smooth", 103, ["-M", "1", "-I", "-r", "20,5"]),
    ("g16_M5_lazy_termall", (64, 64, 1, 16), "smooth", 104, ["-M", "5"]),
    ("g12_M17_lazy_pterm", (70, 90, 1, 12), "uniform", 105, ["-M", "17"]),
    ("g12_M63", (70, 90, 1, 12), "smooth", 106, ["-M", "63"]),
    ("g16_M3_lazy_reset", (64, 64, 1, 16), "uniform", 107, ["-M", "3", "-r", "8,2,1"]),
    # region of interest (-R c=<comp>,U=<shift>): RGN marker, band bit-planes
    # raised by the shift, decoder scales magnitudes >= 2^shift back down
    ("g8_roi_U5", (96, 128, 1, 8), "smooth", 110, ["-R", "c=0,U=5"]),
    ("rgb8_roi_c1_I_r", (96, 128, 3, 8), "smooth", 111, ["-R", "c=1,U=7", "-I", "-r", "20,5"]),
    ("g12_roi_M1_tiles", (130, 170, 1, 12), "uniform", 112, ["-R", "c=0,U=3", "-M", "1", "-t", "64,64"]),
    ("rgb12_roi_c2_U12", (70, 90, 3, 12), "smooth", 113, ["-R", "c=2,U=12"]),
    # fixed-quality layers (-q PSNR[,PSNR..]: cp_fixed_quality, PCRD to a
    # distortion target per layer, TileProcessor.cpp pcrd_bisect_simple /
    # _feasible with the distortion criterion), 5/3 and 9/7, one and several
    # layers, both PCRD algorithms
    ("g8_q30", (96, 128, 1, 8), "smooth", 120, ["-q", "30"]),
    ("rgb8_q28_36_44", (96, 128, 3, 8), "smooth", 121, ["-q", "28,36,44"]),
    ("rgb12_q40_I", (80, 96, 3, 12), "smooth", 122, ["-I", "-q", "40"]),
    ("g12_q30_40_50_I", (70, 90, 1, 12), "smooth", 123, ["-I", "-q", "30,40,50"]),
    ("g12_q35_45_A1", (70, 90, 1, 12), "uniform", 124, ["-q", "35,45", "-A", "1"]),
    ("rgb8_q32_40_I_A1_prec", (150, 200, 3, 8), "smooth", 125, ["-I", "-q", "32,40", "-A", "1", "-c",
                                                                 "[32,32],[16,16]", "-p", "RPCL"]),
]

# Reference decodes with grk_decompress options (-l layers, -r reduce), per
# case: stored as <case>.<tag>.dec.npy, tag = the options without dashes
# ("l1", "r1l2"), with the decoded header in the manifest under "variants".
# Not g8_off35 -r 1: at an odd image offset the reference sizes the reduced
# component as ceil(w / 2^r) (grk_image_comp_header_update) while it decodes
# ceil(x1 / 2^r) - ceil(x0 / 2^r) samples (27 x 31 planes holding 26 x 30)
# and returns uninitialised samples in the extra row / column -- its output
# differs from run to run.  Ours sizes the planes the same way and zeroes
# the extra samples (tests/test_gpu_parity.py assert_reduced_plane).
DEC_VARIANTS = {
    "g8_r40_20_10": [["-l", "1"], ["-l", "2"], ["-r", "1", "-l", "2"]],
    "rgb12_r30_10_1_I": [["-l", "1"], ["-l", "2"], ["-r", "2"]],
    "rgb8_rlcp_layers": [["-l", "1"]],
    "rgb8_tp_L": [["-l", "2"]],
    "g8_sop_eph": [["-l", "1"]],
    "rgb8_poc_r15_I": [["-l", "1"]],
    "rgb8_prec_r20_rpcl": [["-l", "1"], ["-r", "1"]],
    "g12_prec_r12_A1": [["-r", "2"]],
    "rgb8_128x96": [["-r", "1"], ["-r", "1", "-d", "10,6,91,77"], ["-r", "2", "-d", "17,9,128,96"]],
    "rgb12_I": [["-r", "2"], ["-r", "1", "-d", "9,13,70,61"]],
    "g8_off_tiles": [["-r", "2"], ["-r", "1", "-d", "40,30,170,121"]],
    "g16_128": [["-r", "2", "-d", "33,20,100,99"]],
    "rgb12_cinema4k": [["-r", "1"]],
    "rgb8_prec_cprl": [["-r", "1"]],
    "g16_I": [["-r", "3"]],
    "g12_M4_layers": [["-l", "1"], ["-l", "2"]],
    "rgb8_M62_I_r": [["-l", "1"], ["-r", "1"]],
    "g16_M3_lazy_reset": [["-l", "1"], ["-l", "2"]],
    "rgb8_M1_I_r": [["-l", "1"]],
    "rgb8_roi_c1_I_r": [["-l", "1"], ["-r", "1"]],
    "g8_roi_U5": [["-r", "2"]],
    "rgb8_q28_36_44": [["-l", "1"], ["-l", "2"]],
    "g12_q30_40_50_I": [["-l", "1"]],
}


def variant_tag(args):
    return "".join(a.lstrip("-") for a in args).replace(",", "_")


# BASELINE.json configs (hash-only)
LARGE = [
    ("C1_512_gray8", (512, 512, 1, 8), "smooth", 1, []),
    ("C2_4k_rgb8", (2160, 3840, 3, 8), "smooth", 2, []),
    ("C3_8k_rgb12_I", (4320, 7680, 3, 12), "smooth", 3, ["-I"]),
    ("C3_8k_rgb12", (4320, 7680, 3, 12), "smooth", 3, []),
    ("C4_16k_gray16_tiled", (16384, 16384, 1, 16), "smooth", 4, ["-t", "1024,1024", "-n", "7"]),
    # round 2: the secondary C3 run (rate-controlled) and C5, the DCI 4K cinema frame
    ("C3_8k_rgb12_I_r20", (4320, 7680, 3, 12), "smooth", 3, ["-I", "-r", "20"]),
    ("C5_dci4k_rgb12_cinema", (2160, 4096, 3, 12), "smooth", 5, ["-cinema4K", "24"]),
    ("C5b_dci2k_rgb12_cinema", (1080, 2048, 3, 12), "smooth", 6, ["-cinema2K", "24"]),
    # round 6: SURVEY 8(d)'s other input distributions of the C3 frame --
    # uniform full-range noise (the T1 worst case: every bit-plane coded, the
    # most MQ symbols) and a constant mid-grey frame (empty code-blocks)
    ("C3_8k_rgb12_I_uniform", (4320, 7680, 3, 12), "uniform", 3, ["-I"]),
    ("C3_8k_rgb12_uniform", (4320, 7680, 3, 12), "uniform", 3, []),
    ("C3_8k_rgb12_I_const", (4320, 7680, 3, 12), "const", 3, ["-I"]),
    ("C3_8k_rgb12_const", (4320, 7680, 3, 12), "const", 3, []),
]


def sha(b):
    return hashlib.sha256(b).hexdigest()


def build_ref():
    """Compile oracle/_ref from /root/reference (no-op when up to date)."""
    subprocess.run(["make", "-s", "-f", "oracle/ref.mk", "-j8"], cwd=ROOT, check=True)


def ref_encode(img, bits, args, tmp, signed=False):
    c, h, w = img.shape
    src = os.path.join(tmp, "in.i32")
    out = os.path.join(tmp, "out.j2k")
    np.ascontiguousarray(img, dtype="<i4").tofile(src)
    subprocess.run([DRIVER, "enc", src, out, str(w), str(h), str(c), str(bits), str(int(signed))] + list(args),
                   check=True, stdout=subprocess.DEVNULL)
    with open(out, "rb") as f:
        return f.read()


def ref_decode(j2k, tmp, extra=()):
    """Reference decode -> (int32 array (c,h,w), header tuple)."""
    src = os.path.join(tmp, "in.j2k")
    out = os.path.join(tmp, "out.i32")
    with open(src, "wb") as f:
        f.write(j2k)
    r = subprocess.run([DRIVER, "dec", src, out] + list(extra), check=True, capture_output=True, text=True)
    x0, y0, x1, y1, nc, prec, sgnd, cw, ch = map(int, r.stdout.splitlines()[0].split())
    dec = np.fromfile(out, dtype="<i4").reshape(nc, ch, cw)
    return dec, (x0, y0, x1, y1, prec, sgnd)


def ref_decode_planes(j2k, tmp, extra=()):
    """Reference decode of a stream whose components may differ in size
    (subsampled) -> ([int32 (h_k, w_k) per component], [(dx, dy) per component])."""
    src = os.path.join(tmp, "in.j2k")
    out = os.path.join(tmp, "out.i32")
    with open(src, "wb") as f:
        f.write(j2k)
    r = subprocess.run([DRIVER, "dec", src, out] + list(extra), check=True, capture_output=True, text=True)
    f = list(map(int, r.stdout.splitlines()[1].split()[1:]))
    raw = np.fromfile(out, dtype="<i4")
    planes, subs, off = [], [], 0
    for k in range(len(f) // 4):
        w, h, dx, dy = f[4 * k:4 * k + 4]
        planes.append(raw[off:off + w * h].reshape(h, w))
        subs.append((dx, dy))
        off += w * h
    return planes, subs


def run_case(name, shape, kind, seed, args, tmp, keep_dir=None):
    h, w, c, bits = shape
    img = synth.synth_image(h, w, c, bits, seed, kind)
    jb = ref_encode(img, bits, args, tmp)
    dec, _ = ref_decode(jb, tmp)
    diff = (dec.astype(np.int64) - img).ravel()
    mse = float((diff.astype(np.float64) ** 2).mean())
    rec = dict(shape=[h, w, c, bits], kind=kind, seed=seed, args=args,
               image_sha256=synth.image_sha256(img), j2k_sha256=sha(jb), j2k_len=len(jb),
               dec_sha256=synth.image_sha256(dec),
               dec_vs_src_maxabs=int(np.abs(diff).max()) if diff.size else 0,
               dec_vs_src_mse=mse)
    if keep_dir:
        with open(os.path.join(keep_dir, f"{name}.j2k"), "wb") as f:
            f.write(jb)
        np.save(os.path.join(keep_dir, f"{name}.dec.npy"), dec)
    variants = {}
    for vargs in DEC_VARIANTS.get(name, []):
        vdec, hdr = ref_decode(jb, tmp, vargs)
        tag = variant_tag(vargs)
        variants[tag] = dict(args=vargs, dec_sha256=synth.image_sha256(vdec), header=list(hdr))
        if keep_dir:
            np.save(os.path.join(keep_dir, f"{name}.{tag}.dec.npy"), vdec)
    if variants:
        rec["variants"] = variants
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--large", action="store_true")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--only", nargs="*")
    a = ap.parse_args()
    build_ref()
    cases = LARGE if a.large else CASES
    if a.only:
        cases = [cs for cs in cases if cs[0] in a.only]
    mname = "manifest_large.json" if a.large else "manifest.json"
    committed = {}
    if os.path.exists(os.path.join(GOLD, mname)):
        with open(os.path.join(GOLD, mname)) as f:
            committed = json.load(f)
    bad = 0
    man = dict(committed)
    with tempfile.TemporaryDirectory() as tmp:
        keep = None if (a.large or a.check) else GOLD
        for case in cases:
            rec = run_case(*case, tmp, keep_dir=keep)
            if a.check:
                ref = committed.get(case[0])
                same = ref is not None and all(ref.get(k) == rec.get(k)
                                               for k in ("j2k_sha256", "dec_sha256", "image_sha256", "variants"))
                if not a.large and same:
                    with open(os.path.join(GOLD, f"{case[0]}.j2k"), "rb") as f:
                        same = sha(f.read()) == rec["j2k_sha256"]
                    same = same and synth.image_sha256(np.load(os.path.join(GOLD, f"{case[0]}.dec.npy"))) == rec["dec_sha256"]
                    for tag, v in rec.get("variants", {}).items():
                        vd = np.load(os.path.join(GOLD, f"{case[0]}.{tag}.dec.npy"))
                        same = same and synth.image_sha256(vd) == v["dec_sha256"]
                print(case[0], "ok" if same else "MISMATCH", flush=True)
                bad += not same
            else:
                man[case[0]] = rec
                print(case[0], rec["j2k_len"], flush=True)
    if a.check:
        print("mismatches", bad)
        sys.exit(1 if bad else 0)
    with open(os.path.join(GOLD, mname), "w") as f:
        json.dump(man, f, indent=1)
    print("ok", len(cases))


if __name__ == "__main__":
    main()
