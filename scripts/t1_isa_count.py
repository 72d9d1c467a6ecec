"""Instruction counts of the T1 decoder's magnitude-refinement decision loop
(the innermost loop of k_t1_decode_ub<64, false, 4, 4> that holds both the
ctz of the refinement word and the MQ renormalisation's clz), from the
gfx950 assembly: VALU / SALU / LDS / VMEM per iteration along the common
path (every exec-masked region of the loop skipped: the carry-event and
dry-ring blocks, entered only when a lane needs them).
  python scripts/t1_isa_count.py [kernels.hip]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else os.path.join(ROOT, "grokimagecompression_amd", "csrc", "kernels.hip")
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
mrp = []
for hb in hdrs:
    key = hb.lstrip(".L")
    body_blocks = [b for b in order if loopof.get(b) == key or b == hb]
    if any(x.startswith("v_ffbh_u32") for b in body_blocks for x in blocks[b]):
        mrp.append((hb, body_blocks))
if not mrp:
    sys.exit("MRP loop not found")
# the single-segment path comes last in the kernel: its two MRP loops are the
# two-way one (contexts 15 / 16, taken unless a lane needs context 14) and the
# three-way one
mrp = mrp[-2:]
best = mrp[0]


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


def common_path(hdr, loop_blocks):
    """instruction counts along the loop's common path: from the header, every
    exec-masked region inside the loop skipped (its s_cbranch_execz taken:
    the carry-event / dry-ring paths, entered only when one of the
    wavefront's lanes needs them), back to the header"""
    tot = {"valu": 0, "salu": 0, "lds": 0, "vmem": 0, "other": 0}
    inloop = set(loop_blocks)
    pos = order.index(hdr)
    used, seen = [], set()
    while True:
        b = order[pos]
        if b in seen:
            break
        seen.add(b)
        used.append(b)
        nxt = pos + 1
        for x in blocks[b]:
            tot[kind(x)] += 1
            m = re.match(r"s_(cbranch_execz|branch)\s+(\S+)", x)
            if m:
                if m.group(1) == "branch" or m.group(2) in inloop:
                    nxt = order.index(m.group(2))
                break
        if nxt >= len(order) or order[nxt] not in inloop:
            break
        pos = nxt
    return tot, used


for label, lp in zip(("two-way (15 / 16)", "three-way (14 / 15 / 16)"), mrp):
    tot, used = common_path(lp[0], lp[1])
    rare = [b for b in lp[1] if b not in used]
    print("MRP decision loop, %s contexts, of %s (header %s): common-path blocks %s; skipped %s" % (
        label, name[:48], lp[0], " ".join(used), " ".join(rare)))
    print("  per decision (common path: no lane in a carry event or on a dry ring): VALU %d  SALU %d  LDS %d  VMEM %d"
          % (tot["valu"], tot["salu"], tot["lds"], tot["vmem"]))
if "--all" in sys.argv:
    # every innermost loop with a decode site (the MQ table read), in code order
    for hb in order:
        key = hb.lstrip(".L")
        lb = [b for b in order if loopof.get(b) == key or b == hb]
        if len(lb) < 2 or not any(x.startswith("ds_read_b32") for b in lb for x in blocks[b]):
            continue
        if not any(x.startswith("v_ffbh_u32") for b in lb for x in blocks[b]):
            continue
        # the whole body less the bit reader's rare region: the blocks from
        # the one after the renormalisation's limit branch (the block with
        # the window alignbit ends in it) up to that branch's target
        rare = set()
        for b in lb:
            if any(x.startswith("v_alignbit_b32") for x in blocks[b]) and blocks[b][-1].startswith("s_cbranch_execz"):
                tgt = blocks[b][-1].split()[1]
                i, j = order.index(b) + 1, order.index(tgt)
                rare.update(order[i:j])
        t = {"valu": 0, "salu": 0, "lds": 0, "vmem": 0, "other": 0}
        for b in lb:
            if b not in rare:
                for x in blocks[b]:
                    t[kind(x)] += 1
        print("  loop %s: %d blocks; all but the bit reader's rare path (every masked region entered): VALU %d SALU %d LDS %d"
              % (hb, len(lb), t["valu"], t["salu"], t["lds"]))
