"""Cut-stream fixtures: golden codestreams truncated at many positions (inside
and at the edges of tile-part headers, right after SOD, inside tile data, and
at fixed distances from the end), decoded by the reference itself
(oracle/_ref/ref_driver, Grok 5.1.0 built from /root/reference).  A decode of
a stream lost at its tail must return what Grok returns -- the same image, or
the same refusal: the reference decodes a tile from the tile-parts it has
read, leaves tiles it never reaches at zero, and fails when the stream ends
inside a tile-part header or between the tile-parts of a tile
(j2k_decode_tiles, j2k.cpp:1136-1224).  Writes tests/golden/manifest_cut.json:
per stream, per cut length either "error" or {"sha": sha256 of the decoded
(c, h, w) int32 image, "tiles": tiles holding a non-zero sample}.  The cut
streams are prefixes of the committed goldens, so no stream is stored.
TEST INFRASTRUCTURE ONLY.
  python oracle/make_golden_cut.py [--check]"""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE]

import numpy as np  # noqa: E402

import make_golden as mg  # noqa: E402

# multi-tile, tile-parts (by resolution / layer / component), TLM + cinema,
# SOP / EPH, PPM / PPT, single tile (5/3, 9/7), precincts + layers
STREAMS = ["g8_tiles64", "rgb12_tiles_I", "g8_off_tiles", "rgb8_r10_tiles", "rgb12_M46_tiles", "g12_roi_M1_tiles",
           "rgb8_tp_R", "rgb8_tp_L", "rgb8_tp_C_cprl", "rgb12_cinema2k", "g8_sop_eph", "mk_ppt_tparts", "mk_ppm",
           "g8_256", "rgb12_I", "rgb8_rlcp_layers", "sub_422_I_tiles"]


def rd16(b, o):
    return (b[o] << 8) | b[o + 1]


def rd32(b, o):
    return (rd16(b, o) << 16) | rd16(b, o + 2)


def layout(cs):
    """(siz fields, [(sot, tile, psot, sod)]) of a well-formed stream."""
    pos, siz = 2, None
    while pos + 4 <= len(cs):
        m, L = rd16(cs, pos), rd16(cs, pos + 2)
        if m == 0xFF51:
            p = pos + 4
            siz = dict(x1=rd32(cs, p + 2), y1=rd32(cs, p + 6), x0=rd32(cs, p + 10), y0=rd32(cs, p + 14),
                       tdx=rd32(cs, p + 18), tdy=rd32(cs, p + 22), tx0=rd32(cs, p + 26), ty0=rd32(cs, p + 30),
                       dx=[cs[p + 37 + 3 * k] for k in range(rd16(cs, p + 34))],
                       dy=[cs[p + 38 + 3 * k] for k in range(rd16(cs, p + 34))])
        if m == 0xFF90:
            break
        pos += 2 + L
    tps = []
    while pos + 12 <= len(cs) and rd16(cs, pos) == 0xFF90:
        t, psot = rd16(cs, pos + 4), rd32(cs, pos + 6)
        q = pos + 12
        while rd16(cs, q) != 0xFF93:
            q += 2 + rd16(cs, q + 2)
        tps.append((pos, t, psot, q))
        if not psot:
            break
        pos += psot
    return siz, tps


def cuts(cs, tps):
    n = len(cs)
    c = {n - k for k in (1, 2, 3, 40, 300, 1000) if k < n - 64}
    pick = tps[:2] + tps[len(tps) // 2:len(tps) // 2 + 2] + tps[-2:]
    for sot, t, psot, sod in pick:
        c |= {sot + d for d in (0, 1, 2, 3, 4, 6, 11, 12, 13, 14)}
        c |= {sod + d for d in (-1, 0, 1, 2, 3, 4, 10, 40)}
        end = sot + psot if psot else n - 2
        c |= {(sod + end) // 2, end - 1, end + 1}
    return sorted(x for x in c if 64 < x < n)


def tiles_nonzero(dec, siz):
    """Tiles of the (c, h, w) image (component grid of component 0) holding a
    non-zero sample."""
    tw = -(-(siz["x1"] - siz["tx0"]) // siz["tdx"])
    th = -(-(siz["y1"] - siz["ty0"]) // siz["tdy"])
    dx, dy = siz["dx"][0], siz["dy"][0]
    cx0, cy0 = -(-siz["x0"] // dx), -(-siz["y0"] // dy)
    out = []
    for t in range(tw * th):
        i, j = t % tw, t // tw
        X0 = max(siz["tx0"] + i * siz["tdx"], siz["x0"])
        Y0 = max(siz["ty0"] + j * siz["tdy"], siz["y0"])
        X1 = min(siz["tx0"] + (i + 1) * siz["tdx"], siz["x1"])
        Y1 = min(siz["ty0"] + (j + 1) * siz["tdy"], siz["y1"])
        x0, y0, x1, y1 = -(-X0 // dx) - cx0, -(-Y0 // dy) - cy0, -(-X1 // dx) - cx0, -(-Y1 // dy) - cy0
        if np.any(dec[:, y0:y1, x0:x1]):
            out.append(t)
    return out


def main():
    check = "--check" in sys.argv
    mg.build_ref()
    man = {}
    with tempfile.TemporaryDirectory() as tmp:
        for name in STREAMS:
            cs = open(os.path.join(mg.GOLD, name + ".j2k"), "rb").read()
            siz, tps = layout(cs)
            rec = {}
            for n in cuts(cs, tps):
                try:
                    if siz["dx"] != [1] * len(siz["dx"]) or siz["dy"] != [1] * len(siz["dy"]):
                        planes, _ = mg.ref_decode_planes(cs[:n], tmp)
                        flat = np.concatenate([p.ravel() for p in planes])
                        rec[str(n)] = {"sha": mg.synth.image_sha256(flat), "tiles": None}
                    else:
                        dec, _ = mg.ref_decode(cs[:n], tmp)
                        rec[str(n)] = {"sha": mg.synth.image_sha256(dec), "tiles": tiles_nonzero(dec, siz)}
                except Exception:
                    rec[str(n)] = "error"
            man[name] = {"len": len(cs), "j2k_sha256": mg.sha(cs), "cuts": rec}
            ne = sum(v == "error" for v in rec.values())
            print(name, len(rec), "cuts,", ne, "refused", flush=True)
    path = os.path.join(mg.GOLD, "manifest_cut.json")
    if check:
        old = json.load(open(path))
        bad = sum(old.get(k) != v for k, v in man.items())
        print("mismatches", bad)
        sys.exit(1 if bad else 0)
    with open(path, "w") as f:
        json.dump(man, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
