"""Coding-parameter marker fixtures: codestreams that carry COC / QCC in the
main header, COD / COC / QCD / QCC / RGN in tile-part headers, and packed
packet headers (PPM in the main header, PPT in tile-part headers), each
decoded by the REFERENCE (oracle/_ref/ref_driver, Grok 5.1.0 built from
/root/reference).  Grok's encoder writes none of these, so the streams are
assembled at the marker level from streams the reference encoder did write:

- tile / component splicing: a tile-component's packets depend only on its
  own coding parameters and its absolute geometry, so a tile coded as a
  separate image at the same offset (-d) and a component coded as a
  separate grey image in CPRL order (component-major, pi_next_cprl) are
  spliced into a multi-tile / multi-component stream whose per-tile and
  per-component parameters then come from COD / COC / QCD / QCC.  Lossless
  throughout, so the decode also equals the source image;
- marker moves: the main header's COD / QCD / RGN copied or moved into
  tile-part headers (j2k.cpp:3829-4990 precedence);
- packed headers: streams coded with SOP + EPH are split at those markers
  into packet headers (ending with EPH) and bodies (starting with SOP); the
  headers go into PPM (one Nppm chunk per tile-part, over several markers)
  or PPT (several markers per tile, written out of Zppt order).

Writes tests/golden/mk_<name>.j2k / .dec.npy and manifest_markers.json (a
decode the reference refuses is recorded as "error").
  python oracle/make_golden_markers.py [--check]"""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE]

import numpy as np  # noqa: E402

import make_golden as mg  # noqa: E402

SOC, SOT, SOD, EOC = 0xFF4F, 0xFF90, 0xFF93, 0xFFD9
COD, COC, QCD, QCC, RGN, PPM, PPT = 0xFF52, 0xFF53, 0xFF5C, 0xFF5D, 0xFF5E, 0xFF60, 0xFF61


def u16(b, o):
    return int.from_bytes(b[o:o + 2], "big")


def seg(m, payload):
    return m.to_bytes(2, "big") + (len(payload) + 2).to_bytes(2, "big") + bytes(payload)


def parse(cs):
    """-> (main header [(marker, payload)], tile-parts [dict(isot, tpsot, tnsot, hdr, body)])."""
    assert u16(cs, 0) == SOC
    pos, main, tps = 2, [], []
    while u16(cs, pos) != SOT:
        m, L = u16(cs, pos), u16(cs, pos + 2)
        main.append((m, bytes(cs[pos + 4:pos + 2 + L])))
        pos += 2 + L
    while u16(cs, pos) == SOT:
        isot, psot = u16(cs, pos + 4), int.from_bytes(cs[pos + 6:pos + 10], "big")
        tpsot, tnsot = cs[pos + 10], cs[pos + 11]
        end = pos + psot if psot else len(cs) - 2
        p = pos + 12
        hdr = []
        while u16(cs, p) != SOD:
            m, L = u16(cs, p), u16(cs, p + 2)
            hdr.append((m, bytes(cs[p + 4:p + 2 + L])))
            p += 2 + L
        tps.append(dict(isot=isot, tpsot=tpsot, tnsot=tnsot, hdr=hdr, body=bytes(cs[p + 2:end])))
        pos = end
    assert u16(cs, pos) == EOC
    return main, tps


def write(main, tps):
    out = bytearray(SOC.to_bytes(2, "big"))
    for m, pl in main:
        out += seg(m, pl)
    for tp in tps:
        hdr = b"".join(seg(m, pl) for m, pl in tp["hdr"])
        psot = 12 + len(hdr) + 2 + len(tp["body"])
        out += SOT.to_bytes(2, "big") + (10).to_bytes(2, "big") + tp["isot"].to_bytes(2, "big")
        out += psot.to_bytes(4, "big") + bytes([tp["tpsot"], tp["tnsot"]])
        out += hdr + SOD.to_bytes(2, "big") + tp["body"]
    out += EOC.to_bytes(2, "big")
    return bytes(out)


def find(main, m):
    return [pl for mm, pl in main if mm == m]


def coc_of(cod, comp):
    """COD payload -> COC payload for `comp` (Scoc = precinct bit, SPcoc = SPcod)."""
    return bytes([comp, cod[0] & 1]) + cod[5:]


def qcc_of(qcd, comp):
    return bytes([comp]) + qcd


def split_packets(body):
    """SOP+EPH tile-part body -> [(header incl. EPH, body incl. SOP)] (one per packet)."""
    sops = []
    i = 0
    while i + 1 < len(body):
        if body[i] == 0xFF and body[i + 1] == 0x91:
            sops.append(i)
            i += 6
        else:
            i += 1
    assert sops and sops[0] == 0, "every packet starts with SOP"
    out = []
    for k, s in enumerate(sops):
        e = sops[k + 1] if k + 1 < len(sops) else len(body)
        pk = body[s:e]
        j = 6
        while not (pk[j] == 0xFF and pk[j + 1] == 0x92):
            j += 1
        out.append((pk[6:j + 2], pk[:6] + pk[j + 2:]))
    return out


# ---------------------------------------------------------------- the cases
def synth(h, w, c, bits, seed):
    return mg.synth.synth_image(h, w, c, bits, seed, "smooth")


def enc(img, bits, args, tmp):
    return mg.ref_encode(img, bits, args, tmp)


def case_tile_cod(tmp):
    """Two tiles, tile 1 with its own COD / QCD (numres, code-block size,
    precincts, progression and layer count all differ from the main header)."""
    img = synth(64, 128, 1, 8, 301)
    full = enc(img, 8, ["-t", "64,64", "-n", "3", "-b", "32,32"], tmp)
    t1 = enc(img[:, :, 64:], 8, ["-d", "64,0", "-T", "64,0", "-t", "64,64", "-n", "6", "-b", "16,16", "-p", "RPCL",
                                 "-c", "[32,32],[16,16]"], tmp)
    main, tps = parse(full)
    m1, tp1 = parse(t1)
    assert len(tp1) == 1
    tps = [tps[0], dict(isot=1, tpsot=0, tnsot=1, hdr=[(COD, find(m1, COD)[0]), (QCD, find(m1, QCD)[0])],
                        body=tp1[0]["body"])]
    return write(main, tps), img


def rgb_from_greys(imgs, plist, bits, tmp, offset=None, tiles=None):
    """Code each component as a grey CPRL image with its own options."""
    out = []
    for k, (im, opts) in enumerate(zip(imgs, plist)):
        a = ["-p", "CPRL"] + opts
        if offset:
            a += ["-d", "%d,%d" % offset, "-T", "%d,%d" % offset]
        if tiles:
            a += ["-t", "%d,%d" % tiles]
        out.append(parse(enc(im[None], bits, a, tmp)))
    return out


P0 = ["-n", "4", "-b", "32,32"]
P1 = ["-n", "2", "-b", "64,16"]
P2 = ["-n", "6", "-b", "16,16", "-c", "[32,32],[16,16]"]
P3 = ["-n", "3", "-b", "16,64"]


def case_main_coc(tmp):
    """One tile, three components: main COD / QCD for components 0 and 2,
    main COC / QCC for component 1 (other numres, code-block and
    precinct sizes); CPRL so each component's packets are contiguous."""
    img = synth(70, 90, 3, 8, 302)
    g = rgb_from_greys([img[0], img[1], img[2]], [P0, P2, P0], 8, tmp)
    ref, _ = parse(enc(img, 8, ["-p", "CPRL", "-Y", "0"] + P0, tmp))  # SIZ / COD with three components
    main = []
    for m, pl in ref:
        main.append((m, pl))
        if m == COD:
            main.append((COC, coc_of(find(g[1][0], COD)[0], 1)))
        if m == QCD:
            main.append((QCC, qcc_of(find(g[1][0], QCD)[0], 1)))
    body = b"".join(gk[1][0]["body"] for gk in g)
    return write(main, [dict(isot=0, tpsot=0, tnsot=1, hdr=[], body=body)]), img


def case_tile_coc(tmp):
    """Two tiles, three components.  Main: COD P0, COC(1) P1.  Tile 0 uses
    them.  Tile 1's header: COD P2, COC(2) P3, QCD P2, QCC(2) P3 -- so tile 1
    codes component 0 and 1 with P2 (a tile COD beats a main COC) and
    component 2 with P3."""
    img = synth(64, 128, 3, 8, 303)
    left = [img[k][:, :64] for k in range(3)]
    right = [img[k][:, 64:] for k in range(3)]
    g0 = rgb_from_greys(left, [P0, P1, P0], 8, tmp, tiles=(64, 64))
    g1 = rgb_from_greys(right, [P2, P2, P3], 8, tmp, offset=(64, 0), tiles=(64, 64))
    ref, _ = parse(enc(img, 8, ["-p", "CPRL", "-Y", "0", "-t", "64,64"] + P0, tmp))
    main = []
    for m, pl in ref:
        main.append((m, pl))
        if m == COD:
            main.append((COC, coc_of(find(g0[1][0], COD)[0], 1)))
        if m == QCD:
            main.append((QCC, qcc_of(find(g0[1][0], QCD)[0], 1)))
    # tile 1's COD: P2's with the main header's progression / layers / MCT
    cod2 = bytearray(find(g1[0][0], COD)[0])
    cod2[1:5] = find(ref, COD)[0][1:5]
    hdr1 = [(COD, bytes(cod2)), (COC, coc_of(find(g1[2][0], COD)[0], 2)),
            (QCD, find(g1[0][0], QCD)[0]), (QCC, qcc_of(find(g1[2][0], QCD)[0], 2))]
    tps = [dict(isot=0, tpsot=0, tnsot=1, hdr=[], body=b"".join(g[1][0]["body"] for g in g0)),
           dict(isot=1, tpsot=0, tnsot=1, hdr=hdr1, body=b"".join(g[1][0]["body"] for g in g1))]
    return write(main, tps), img


def case_tp_cod_copy(tmp):
    """Every tile's first tile-part repeats the main COD / QCD (values unchanged)."""
    img = synth(150, 200, 3, 12, 304)
    main, tps = parse(enc(img, 12, ["-I", "-t", "64,64", "-u", "R", "-r", "12"], tmp))
    seen = set()
    for tp in tps:
        if tp["isot"] not in seen:
            seen.add(tp["isot"])
            tp["hdr"] = [(COD, find(main, COD)[0]), (QCD, find(main, QCD)[0])] + tp["hdr"]
    return write(main, tps), None


def case_tp_cod_conflict(tmp):
    """Coding parameters that change in a later tile-part (the standard allows
    COD / QCD only in a tile's first tile-part; the reference reads them from
    any tile-part header, warns about a second COD and lets the last one win,
    j2k.cpp:3816-3825, since a tile's packets are parsed only after all its
    tile-parts, j2k.cpp:1136-1224).  Tile 0's second tile-part repeats the COD
    with the MCT switched off; tile 1's last tile-part repeats the QCD with
    other step-size mantissas (same exponents, so the packets parse alike)."""
    img = synth(96, 160, 3, 12, 306)
    main, tps = parse(enc(img, 12, ["-I", "-t", "96,96", "-u", "R", "-n", "3", "-r", "10"], tmp))
    cod = bytearray(find(main, COD)[0])
    assert cod[4] == 1
    cod[4] = 0
    qcd = bytearray(find(main, QCD)[0])
    for o in range(1, len(qcd) - 1, 2):  # SPqcd: expn << 11 | mant
        qcd[o + 1] ^= 0x55
    t0 = [tp for tp in tps if tp["isot"] == 0]
    t1 = [tp for tp in tps if tp["isot"] == 1]
    assert len(t0) >= 2 and len(t1) >= 2
    t0[1]["hdr"] = [(COD, bytes(cod))] + t0[1]["hdr"]
    t1[-1]["hdr"] = [(QCD, bytes(qcd))] + t1[-1]["hdr"]
    return write(main, tps), None


def case_tile_rgn(tmp):
    """ROI shift carried by tile 1's header only (main RGN removed): tile 0
    decodes without the shift it was coded with, as the reference does."""
    img = synth(96, 128, 1, 8, 305)
    main, tps = parse(enc(img, 8, ["-R", "c=0,U=5", "-t", "64,64"], tmp))
    rgn = find(main, RGN)[0]
    main = [(m, pl) for m, pl in main if m != RGN]
    for tp in tps:
        if tp["isot"] == 1:
            tp["hdr"] = [(RGN, rgn)] + tp["hdr"]
    return write(main, tps), None


def packed(cs, mode):
    """SOP+EPH stream -> packed headers in PPM (mode 'ppm') or PPT ('ppt')."""
    main, tps = parse(cs)
    chunks = []
    for tp in tps:
        pk = split_packets(tp["body"]) if tp["body"] else []
        chunks.append(b"".join(h for h, _ in pk))
        tp["body"] = b"".join(b for _, b in pk)
    if mode == "ppm":
        data = b"".join(len(c).to_bytes(4, "big") + c for c in chunks)
        # several PPM markers, written in reverse Zppm order, split mid-chunk
        n = 3
        cut = [len(data) * i // n for i in range(n + 1)]
        ppms = [(PPM, bytes([z]) + data[cut[z]:cut[z + 1]]) for z in range(n)][::-1]
        i = max(k for k, (m, _) in enumerate(main) if m in (COD, QCD, COC, QCC)) + 1
        main = main[:i] + ppms + main[i:]
    else:
        z = {}
        for tp, c in zip(tps, chunks):
            k = z.get(tp["isot"], 0)
            half = len(c) // 2
            parts = [(PPT, bytes([k]) + c[:half]), (PPT, bytes([k + 1]) + c[half:])]
            tp["hdr"] = tp["hdr"] + parts[::-1]
            z[tp["isot"]] = k + 2
    return write(main, tps)


def case_ppt(tmp):
    img = synth(96, 128, 3, 8, 306)
    return packed(enc(img, 8, ["-S", "-E", "-r", "20,5", "-t", "64,64", "-c", "[32,32]"], tmp), "ppt"), None


def case_ppm(tmp):
    """Four tiles of two tile-parts each (-u L).  (Tiles split by resolution,
    -u R, are refused by the reference once their headers move to PPM -- its
    T2.cpp:375 reads them through one running pointer -- though it decodes
    the same stream with PPT; that combination is not a fixture.)"""
    img = synth(96, 128, 3, 8, 307)
    return packed(enc(img, 8, ["-S", "-E", "-r", "30,10", "-t", "64,64", "-u", "L"], tmp), "ppm"), None


def case_ppt_tparts(tmp):
    img = synth(96, 128, 3, 8, 307)
    return packed(enc(img, 8, ["-S", "-E", "-r", "30,10", "-t", "64,64", "-u", "R"], tmp), "ppt"), None


def case_ppm_1tile(tmp):
    img = synth(77, 100, 1, 12, 308)
    return packed(enc(img, 12, ["-S", "-E", "-I", "-r", "20,5,2"], tmp), "ppm"), None


def case_mixed_wavelet(tmp):
    """Main COD 5/3, main COC(1) 9/7: one tile, components with different
    wavelets (the reference decodes it; see the test for ours)."""
    img = synth(64, 64, 2, 8, 309)
    g = rgb_from_greys([img[0], img[1]], [P0, P0 + ["-I"]], 8, tmp)
    ref, _ = parse(enc(img, 8, ["-p", "CPRL", "-Y", "0"] + P0, tmp))
    main = []
    for m, pl in ref:
        main.append((m, pl))
        if m == COD:
            main.append((COC, coc_of(find(g[1][0], COD)[0], 1)))
        if m == QCD:
            main.append((QCC, qcc_of(find(g[1][0], QCD)[0], 1)))
    body = b"".join(gk[1][0]["body"] for gk in g)
    return write(main, [dict(isot=0, tpsot=0, tnsot=1, hdr=[], body=body)]), None


def case_siqnt(tmp):
    """9/7 stream whose QCD is rewritten to scalar-derived (style 1): only
    the LL step size travels, every other band derives its exponent from it
    (Quantizer.cpp:326-336)."""
    img = synth(80, 96, 3, 12, 311)
    main, tps = parse(enc(img, 12, ["-I", "-n", "5"], tmp))
    out = []
    for m, pl in main:
        if m == QCD:
            pl = bytes([(pl[0] & 0xE0) | 1]) + pl[1:3]
        out.append((m, pl))
    return write(out, tps), None


def case_qcd_short(tmp):
    """Reversible QCD with fewer exponents than the 3 L + 1 bands: the
    reference refuses it (j2k.cpp:889-895)."""
    img = synth(64, 64, 1, 8, 312)
    main, tps = parse(enc(img, 8, ["-n", "4"], tmp))
    out = [(m, pl[:-3] if m == QCD else pl) for m, pl in main]
    return write(out, tps), None


def case_coc_then_cod(tmp):
    """A main-header COC written BEFORE the COD: the COD then sets every
    component (j2k_copy_tile_component_parameters, j2k.cpp:3889), so the
    COC's values are dropped.  The stream is a plain single-component one
    with a COC of other parameters placed ahead of its COD."""
    img = synth(64, 64, 1, 8, 313)
    main, tps = parse(enc(img, 8, ["-n", "4", "-b", "32,32"], tmp))
    other = parse(enc(img, 8, ["-n", "2", "-b", "16,16"], tmp))[0]
    out = []
    for m, pl in main:
        if m == COD:
            out.append((COC, coc_of(find(other, COD)[0], 0)))
        out.append((m, pl))
    return write(out, tps), img


def case_mixed_cblksty(tmp):
    """Main COC(1) and COC(2) carrying code-block styles other than the
    COD's: component 0 plain, component 1 every mode switch (-M 63),
    component 2 RESET + vertically causal + SEGSYM (-M 42); two layers."""
    img = synth(72, 100, 3, 8, 314)
    opts = [P0 + ["-r", "20,4"], P0 + ["-r", "20,4", "-M", "63"], P0 + ["-r", "20,4", "-M", "42"]]
    g = rgb_from_greys([img[0], img[1], img[2]], opts, 8, tmp)
    ref, _ = parse(enc(img, 8, ["-p", "CPRL", "-Y", "0"] + opts[0], tmp))
    main = []
    for m, pl in ref:
        main.append((m, pl))
        if m == COD:
            main += [(COC, coc_of(find(g[k][0], COD)[0], k)) for k in (1, 2)]
    body = b"".join(gk[1][0]["body"] for gk in g)
    return write(main, [dict(isot=0, tpsot=0, tnsot=1, hdr=[], body=body)]), None


def _tnsot(tmp, short):
    """Tiles split into tile-parts by resolution (-u R, 3 parts each) whose
    TNsot is rewritten one short (TPsot == TNsot on the last part) for the
    tiles in `short` (None: all)."""
    img = synth(96, 160, 3, 12, 308)
    main, tps = parse(enc(img, 12, ["-I", "-t", "64,64", "-u", "R", "-n", "3", "-r", "10"], tmp))
    count = {}
    for tp in tps:
        count[tp["isot"]] = count.get(tp["isot"], 0) + 1
    assert all(n == 3 for n in count.values()) and all(tp["tnsot"] == 3 for tp in tps)
    for tp in tps:
        if short is None or tp["isot"] in short:
            tp["tnsot"] = count[tp["isot"]] - 1
    return write(main, tps), None


def case_tnsot_all(tmp):
    """Every tile's TNsot one short: the reference's Issue-254 correction
    (j2k.cpp:809-835: found by looking past the first tile's 'last'
    tile-part, then every tile-part count + 1) decodes the whole image."""
    return _tnsot(tmp, None)


def case_tnsot_tile0(tmp):
    """Only tile 0's TNsot short: the correction also adds 1 to the other
    tiles' (correct) counts, so none of them is complete by count; they are
    decoded when the stream ends (j2k_decode_tiles), as the reference does."""
    return _tnsot(tmp, {0})


def case_tnsot_last(tmp):
    """Only the last tile's TNsot short: the one look-ahead (after tile 0)
    finds nothing to correct, and that tile's third part then exceeds its
    count -- the reference refuses the stream."""
    return _tnsot(tmp, {5})


CASES = [("tile_cod", case_tile_cod), ("main_coc", case_main_coc), ("tile_coc", case_tile_coc),
         ("tp_cod_copy", case_tp_cod_copy), ("tp_cod_conflict", case_tp_cod_conflict), ("tile_rgn", case_tile_rgn), ("ppt", case_ppt), ("ppm", case_ppm), ("ppt_tparts", case_ppt_tparts),
         ("ppm_1tile", case_ppm_1tile), ("mixed_wavelet", case_mixed_wavelet), ("siqnt", case_siqnt),
         ("qcd_short", case_qcd_short), ("coc_then_cod", case_coc_then_cod), ("mixed_cblksty", case_mixed_cblksty),
         ("tnsot_all", case_tnsot_all), ("tnsot_tile0", case_tnsot_tile0), ("tnsot_last", case_tnsot_last)]


# reference decodes with grk_decompress options, -> mk_<name>.<tag>.dec.npy
VARIANTS = {"tile_coc": [["-r", "1"]], "main_coc": [["-r", "1"]], "tile_cod": [["-r", "2"]],
            "ppt_tparts": [["-r", "1"], ["-l", "1"]], "ppm": [["-l", "1"]], "mixed_wavelet": [["-r", "1"]],
            "mixed_cblksty": [["-l", "1"], ["-r", "1"]]}


def variant_tag(a):
    return "".join(x.strip("-") for x in a)


def main():
    check = "--check" in sys.argv
    mg.build_ref()
    man = {}
    bad = 0
    with tempfile.TemporaryDirectory() as tmp:
        for name, fn in CASES:
            tag = "mk_" + name
            cs, src = fn(tmp)
            try:
                dec, _ = mg.ref_decode(cs, tmp)
                rec = {"j2k_sha256": mg.sha(cs), "dec_sha256": mg.synth.image_sha256(dec)}
                if src is not None:  # lossless splice: the reference decode is the source
                    rec["dec_is_source"] = bool(np.array_equal(dec, src))
                vdecs = {}
                for va in VARIANTS.get(name, []):
                    vd, _ = mg.ref_decode(cs, tmp, va)
                    vdecs[variant_tag(va)] = vd
                    rec.setdefault("variants", {})[variant_tag(va)] = {
                        "args": va, "dec_sha256": mg.synth.image_sha256(vd)}
            except Exception:
                dec, rec = None, {"j2k_sha256": mg.sha(cs), "dec": "error"}
            man[tag] = rec
            if check:
                old = json.load(open(os.path.join(mg.GOLD, "manifest_markers.json"))).get(tag)
                ok = old == rec and open(os.path.join(mg.GOLD, tag + ".j2k"), "rb").read() == cs
                if ok and dec is not None:
                    ok = mg.synth.image_sha256(np.load(os.path.join(mg.GOLD, tag + ".dec.npy"))) == rec["dec_sha256"]
                    for vt, v in rec.get("variants", {}).items():
                        vd = np.load(os.path.join(mg.GOLD, "%s.%s.dec.npy" % (tag, vt)))
                        ok = ok and mg.synth.image_sha256(vd) == v["dec_sha256"]
                print(tag, "ok" if ok else "MISMATCH", flush=True)
                bad += not ok
                continue
            with open(os.path.join(mg.GOLD, tag + ".j2k"), "wb") as f:
                f.write(cs)
            if dec is not None:
                np.save(os.path.join(mg.GOLD, tag + ".dec.npy"), dec)
                for vt, vd in vdecs.items():
                    np.save(os.path.join(mg.GOLD, "%s.%s.dec.npy" % (tag, vt)), vd)
            print(tag, len(cs), sorted(rec), flush=True)
    if check:
        print("mismatches", bad)
        sys.exit(1 if bad else 0)
    with open(os.path.join(mg.GOLD, "manifest_markers.json"), "w") as f:
        json.dump(man, f, indent=1)


if __name__ == "__main__":
    main()
