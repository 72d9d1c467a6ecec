"""Subsampled-component fixtures (SIZ XRsiz / YRsiz != 1): images whose
components lie on their own grids, encoded AND decoded by the REFERENCE
(oracle/_ref/ref_driver, Grok 5.1.0 built from /root/reference; the driver's
-sub option builds the grk_image with per-component dx / dy, as an
application hands it to grk_compress's library).  Component k of an image
[x0, x0 + w) x [y0, y0 + h) is [ceil(x0 / dx), ceil((x0 + w) / dx)) x ... on
its grid (TileComponent.cpp:150-196); the first three components of
different subsampling disable the MCT (j2k.cpp:1963-1971).

Writes tests/golden/sub_<name>.j2k, sub_<name>.dec.npz (the reference's
decode: one array per component, c0, c1, ...), sub_<name>.<variant>.dec.npz
for -r / -d decodes, and manifest_sub.json.  The source planes are
regenerated from the manifest (synth.synth_image per component, seed + k).
  python oracle/make_golden_sub.py [--check]"""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE]

import numpy as np  # noqa: E402

import make_golden as mg  # noqa: E402

# name, (w, h) of the image, bits, per-component (dx, dy), seed, kind, grk_compress options
CASES = [
    ("420_rgb8", (97, 75), 8, [(1, 1), (2, 2), (2, 2)], 401, "smooth", []),
    ("uniform2_rgb8", (128, 96), 8, [(2, 2), (2, 2), (2, 2)], 402, "smooth", []),
    ("422_I_tiles", (150, 110), 12, [(1, 1), (2, 1), (2, 1)], 403, "smooth",
     ["-I", "-t", "64,64", "-d", "3,5", "-r", "20"]),
    ("gray_3x2_rpcl", (131, 90), 8, [(3, 2)], 404, "uniform", ["-c", "[32,32],[16,16]", "-p", "RPCL"]),
    ("mixed_pcrl", (120, 100), 8, [(1, 1), (2, 2), (4, 4)], 405, "smooth",
     ["-c", "[32,32],[16,16]", "-p", "PCRL", "-n", "4"]),
    # (CPRL with precinct partitions over subsampled components runs the
    # reference encoder out of memory here; without -c it codes)
    ("cprl_tiles_layers", (140, 90), 10, [(1, 1), (2, 3), (3, 2)], 406, "smooth",
     ["-p", "CPRL", "-t", "48,40", "-r", "30,8"]),
]
VARIANTS = {"420_rgb8": [["-r", "1"], ["-d", "10,7,71,60"]], "422_I_tiles": [["-r", "2"], ["-d", "40,30,120,95"]],
            "mixed_pcrl": [["-r", "1"]], "cprl_tiles_layers": [["-l", "1"], ["-d", "5,5,77,51"]]}


def comp_shape(size, off, dx, dy):
    cd = lambda v, s: -(-v // s)  # noqa: E731
    return cd(off[1] + size[1], dy) - cd(off[1], dy), cd(off[0] + size[0], dx) - cd(off[0], dx)


def offset_of(args):
    return tuple(int(v) for v in args[args.index("-d") + 1].split(",")) if "-d" in args else (0, 0)


def planes_of(case):
    name, size, bits, subs, seed, kind, args = case
    off = offset_of(args)
    return [mg.synth.synth_image(*comp_shape(size, off, dx, dy), 1, bits, seed + k, kind)[0]
            for k, (dx, dy) in enumerate(subs)]


def sub_arg(subs):
    return ["-sub", "/".join("%d,%d" % s for s in subs)]


def planes_sha(planes):
    return mg.sha(b"".join(np.ascontiguousarray(p, dtype="<i4").tobytes() for p in planes))


def encode(case, tmp):
    name, size, bits, subs, seed, kind, args = case
    src = os.path.join(tmp, "in.i32")
    out = os.path.join(tmp, "out.j2k")
    with open(src, "wb") as f:
        for p in planes_of(case):
            f.write(np.ascontiguousarray(p, dtype="<i4").tobytes())
    mg.subprocess.run([mg.DRIVER, "enc", src, out, str(size[0]), str(size[1]), str(len(subs)), str(bits), "0"] +
                      list(args) + sub_arg(subs), check=True, stdout=mg.subprocess.DEVNULL)
    return open(out, "rb").read()


def vtag(a):
    return "".join(x.strip("-").replace(",", "_") for x in a)


def main():
    check = "--check" in sys.argv
    mg.build_ref()
    mpath = os.path.join(mg.GOLD, "manifest_sub.json")
    old = json.load(open(mpath)) if os.path.exists(mpath) else {}
    man, bad = {}, 0
    with tempfile.TemporaryDirectory() as tmp:
        for case in CASES:
            name, size, bits, subs, seed, kind, args = case
            tag = "sub_" + name
            src = planes_of(case)
            cs = encode(case, tmp)
            dec, dsubs = mg.ref_decode_planes(cs, tmp)
            assert dsubs == [tuple(s) for s in subs]
            rec = {"size": list(size), "bits": bits, "subsampling": [list(s) for s in subs], "seed": seed,
                   "kind": kind, "args": args, "src_sha256": planes_sha(src), "j2k_sha256": mg.sha(cs),
                   "dec_sha256": planes_sha(dec), "lossless": all(np.array_equal(a, b) for a, b in zip(dec, src))}
            vdecs = {}
            for va in VARIANTS.get(name, []):
                vd, _ = mg.ref_decode_planes(cs, tmp, va)
                vdecs[vtag(va)] = vd
                rec.setdefault("variants", {})[vtag(va)] = {"args": va, "dec_sha256": planes_sha(vd)}
            man[tag] = rec
            if check:
                ok = old.get(tag) == rec and open(os.path.join(mg.GOLD, tag + ".j2k"), "rb").read() == cs
                for vt, vd in [("", dec)] + list(vdecs.items()):
                    f = os.path.join(mg.GOLD, "%s%s.dec.npz" % (tag, "." + vt if vt else ""))
                    z = np.load(f)
                    ok = ok and planes_sha([z["c%d" % k] for k in range(len(subs))]) == planes_sha(vd)
                print(tag, "ok" if ok else "MISMATCH", flush=True)
                bad += not ok
                continue
            with open(os.path.join(mg.GOLD, tag + ".j2k"), "wb") as f:
                f.write(cs)
            np.savez(os.path.join(mg.GOLD, tag + ".dec.npz"), **{"c%d" % k: a for k, a in enumerate(dec)})
            for vt, vd in vdecs.items():
                np.savez(os.path.join(mg.GOLD, "%s.%s.dec.npz" % (tag, vt)), **{"c%d" % k: a for k, a in enumerate(vd)})
            print(tag, len(cs), "lossless" if rec["lossless"] else "lossy", flush=True)
    if check:
        print("mismatches", bad)
        sys.exit(1 if bad else 0)
    with open(mpath, "w") as f:
        json.dump(man, f, indent=1)


if __name__ == "__main__":
    main()
