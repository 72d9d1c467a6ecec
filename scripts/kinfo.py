"""Compile a HIP source for gfx950 to assembly and print each kernel's VGPRs,
occupancy, LDS bytes, scratch instructions and (with --mix) its instruction
histogram.
Usage: python scripts/kinfo.py SRC.hip [name-regex] [--mix]"""
import collections
import os
import re
import subprocess
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
src = os.path.abspath(args[0])
pat = re.compile(args[1]) if len(args) > 1 else None
out = "/tmp/kinfo_%s.s" % os.path.basename(src)
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                "--cuda-device-only", "-S", src, "-o", out], check=True, cwd=os.path.dirname(src))
s = open(out).read()
for m in re.finditer(r"^(_Z\S*):", s, re.M):
    name = m.group(1)
    if pat and not pat.search(name):
        continue
    i = s.find(".Lfunc_end", m.end())
    if i < 0:
        continue
    body = s[m.end():i]

    def field(key):
        j = s.find(key, i)
        return s[j:j + 40].split()[2] if j >= 0 else "?"
    print("%-64s vgpr %4s sgpr %4s occ %2s lds %6s scratch %d" % (
        name[:64], field("; NumVgprs:"), field("; NumSgprs:"), field("; Occupancy:"), field("; LDSByteSize:"),
        body.count("scratch_")))
    if "--mix" in sys.argv:
        ops = collections.Counter(l.split()[0] for l in body.split("\n") if l.startswith("\t") and
                                  not l.startswith("\t.") and not l.startswith("\t;") and l.split())
        print("   ", sum(ops.values()), "instructions:", ", ".join("%s %d" % kv for kv in ops.most_common(40)))
