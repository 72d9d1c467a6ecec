"""grk_get_cstr_index fixtures: the REFERENCE's codestream index
(oracle/_ref/ref_driver index: grk_get_cstr_index after grk_read_header and
after a full grk_decode, every field printed) for every golden codestream,
into tests/golden/cstr_index.json.  The GPU test runs the same driver relinked
against our libgrok.so (ref_driver_mi355x) and compares the text.
  python oracle/make_golden_index.py [--check]"""
import glob
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE]

import make_golden as mg  # noqa: E402


def main():
    check = "--check" in sys.argv
    mg.build_ref()
    out = {}
    for f in sorted(glob.glob(os.path.join(mg.GOLD, "*.j2k"))):
        r = subprocess.run([mg.DRIVER, "index", f], capture_output=True, text=True, timeout=120)
        out[os.path.basename(f)] = r.stdout if r.returncode == 0 else "error"
    path = os.path.join(mg.GOLD, "cstr_index.json")
    if check:
        old = json.load(open(path))
        bad = sum(old.get(k) != v for k, v in out.items()) + len(set(old) ^ set(out))
        print("mismatches", bad)
        sys.exit(1 if bad else 0)
    with open(path, "w") as fh:
        json.dump(out, fh, indent=0, sort_keys=True)
    print(len(out), "streams,", sum(v == "error" for v in out.values()), "refused")


if __name__ == "__main__":
    main()
