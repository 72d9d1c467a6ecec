"""Guard-bit fixtures: golden codestreams whose QCD guard-bit count (Sqcd >> 5)
is patched from Grok's 2 to 1 or 3, decoded by the reference itself
(oracle/_ref/ref_driver, Grok 5.1.0 built from /root/reference).  Every band's
bit-plane count is expn + guard bits - 1 (j2k_read_SQcd_SQcc, Quantizer.cpp),
so the decoder must take the count from the marker, not assume 2.  Writes
tests/golden/<name>.gb<N>.j2k / .dec.npy and manifest_gbits.json (a decode the
reference refuses is recorded as "error").
  python oracle/make_golden_gbits.py [--check]"""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE]

import numpy as np  # noqa: E402

import make_golden as mg  # noqa: E402

CASES = [("g8_256", 1), ("g8_256", 3), ("rgb12_I", 1), ("rgb12_I", 3), ("g16_128", 3)]


def qcd_sqcd_offset(cs):
    pos = 2
    while pos + 4 <= len(cs):
        m = int.from_bytes(cs[pos:pos + 2], "big")
        L = int.from_bytes(cs[pos + 2:pos + 4], "big")
        if m == 0xFF5C:
            return pos + 4
        if m == 0xFF90:
            break
        pos += 2 + L
    raise KeyError("QCD")


def patched(name, gb):
    cs = bytearray(open(os.path.join(mg.GOLD, name + ".j2k"), "rb").read())
    o = qcd_sqcd_offset(cs)
    cs[o] = (cs[o] & 0x1F) | (gb << 5)
    return bytes(cs)


def main():
    check = "--check" in sys.argv
    mg.build_ref()
    man = {}
    bad = 0
    with tempfile.TemporaryDirectory() as tmp:
        for name, gb in CASES:
            tag = "%s.gb%d" % (name, gb)
            cs = patched(name, gb)
            try:
                dec, _ = mg.ref_decode(cs, tmp)
                rec = {"j2k_sha256": mg.sha(cs), "dec_sha256": mg.synth.image_sha256(dec)}
            except Exception:
                dec, rec = None, {"j2k_sha256": mg.sha(cs), "dec": "error"}
            man[tag] = rec
            if check:
                old = json.load(open(os.path.join(mg.GOLD, "manifest_gbits.json"))).get(tag)
                ok = old == rec and open(os.path.join(mg.GOLD, tag + ".j2k"), "rb").read() == cs
                if ok and dec is not None:  # the committed decode is the reference's
                    ok = mg.synth.image_sha256(np.load(os.path.join(mg.GOLD, tag + ".dec.npy"))) == rec["dec_sha256"]
                print(tag, "ok" if ok else "MISMATCH", flush=True)
                bad += not ok
                continue
            with open(os.path.join(mg.GOLD, tag + ".j2k"), "wb") as f:
                f.write(cs)
            if dec is not None:
                np.save(os.path.join(mg.GOLD, tag + ".dec.npy"), dec)
            print(tag, rec.get("dec", "ok"), flush=True)
    if check:
        print("mismatches", bad)
        sys.exit(1 if bad else 0)
    with open(os.path.join(mg.GOLD, "manifest_gbits.json"), "w") as f:
        json.dump(man, f, indent=1)


if __name__ == "__main__":
    main()
