"""Instruction counts of the T1 decoder's magnitude-refinement decision loop
(the innermost loop of k_t1_decode_ub<64, false, 4, 4> that holds both the
ctz of the refinement word and the MQ renormalisation's clz), from the
gfx950 assembly: VALU / SALU / LDS / VMEM per iteration along the common
path (the carry-event and dry-ring blocks excluded, the word-ring refill
counted both ways).
  python scripts/t1_isa_count.py [kernels.hip]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "grokimagecompression_amd", "csrc", "kernels.hip")
out = "/tmp/t1_isa_%d.s" % os.getpid()
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                "--cuda-device-only", "-S", src, "-o", out], check=True, cwd=os.path.dirname(src),
               stderr=subprocess.DEVNULL)
s = open(out).read()
os.unlink(out)
name = re.search(r"^(_ZN6grkgpu14k_t1_decode_ubILi64ELb0ELi4ELi4E\S*):", s, re.M).group(1)
body = s[s.index(name + ":"):]
body = body[:body.index(".Lfunc_end")]
lines = body.split("\n")
blocks, cur, order, loopof = {}, None, [], {}
for ln in lines:
    m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):\s*(.*)$", ln)
    if m:
        cur = m.group(1).replace("; ", "")
        blocks[cur] = []
        order.append(cur)
        h = re.search(r"Header=BB(\d+_\d+)", m.group(2))
        loopof[cur] = ("BB" + h.group(1)) if h else (cur[1:] if "Loop Header" in m.group(2) else None)
        continue
    if cur is None:
        continue
    h = re.search(r"; (?:in Loop: )?Header=BB(\d+_\d+)", ln)
    if h and not blocks[cur]:
        loopof[cur] = "BB" + h.group(1)
    elif "Loop Header" in ln and not blocks[cur]:
        loopof[cur] = cur.lstrip(".L")
    if ln.startswith("\t") and not ln.startswith("\t;") and not ln.startswith("\t."):
        blocks[cur].append(ln.strip())
# the MRP loop: the innermost loop whose header starts with the ctz (v_ffbl)
# of the refinement word and whose body holds the renormalisation clz
hdrs = [b for b in order if blocks[b] and blocks[b][0].startswith("v_ffbl_b32")]
best = None
for hb in hdrs:
    key = hb.lstrip(".L")
    body_blocks = [b for b in order if loopof.get(b) == key or b == hb]
    if any(x.startswith("v_ffbh_u32") for b in body_blocks for x in blocks[b]):
        best = (hb, body_blocks)
if best is None:
    sys.exit("MRP loop not found")


def kind(x):
    op = x.split()[0]
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


tot = {"valu": 0, "salu": 0, "lds": 0, "vmem": 0, "other": 0}
used, rare = [], []
for b in best[1]:
    ins = blocks[b]
    # blocks entered only for a carry event (global_load of the next event)
    # or a dry word ring (global_load_dwordx4 of a chunk) are off the common path
    if any(x.startswith("global_load") for x in ins):
        rare.append(b)
        continue
    used.append(b)
    for x in ins:
        tot[kind(x)] += 1
print("MRP decision loop of %s (header %s): common-path blocks %s; rare blocks %s" % (
    name[:48], best[0], " ".join(used), " ".join(rare)))
print("per decision (common path, ring refill taken by some lane): VALU %d  SALU %d  LDS %d  VMEM %d"
      % (tot["valu"], tot["salu"], tot["lds"], tot["vmem"]))
