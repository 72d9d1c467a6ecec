"""Per-kernel SQ counter table from scripts/gpu_sq_env.sh output:
python scripts/sq_table.py gpurun_out/TAG [kernel-regex]"""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else "t1")
for d in sorted(glob.glob(os.path.join(root, "e*_sq1"))):
    tag = os.path.basename(d)[:-4]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for sd in (d, d[:-1] + "2"):
        for p in glob.glob(sd + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(p)):
                k = r["Kernel_Name"].split("(")[0].replace("void grkgpu::", "").replace("grkgpu::", "")
                if not pat.search(k):
                    continue
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                n[(k, r["Counter_Name"])] += 1
    for k, c in sorted(agg.items()):
        m = {name: v / n[(k, name)] for name, v in c.items()}
        util = m.get("SQ_THREAD_CYCLES_VALU", 0) / max(1, 64 * m.get("SQ_ACTIVE_INST_VALU", 1))
        print("%-4s %-40s valu %.3g salu %.3g lds %.3g vmem %.3g/%.3g wave_cyc %.3g wait %.2f active %.2f lane_util %.2f" % (
            tag, k[:40], m.get("SQ_INSTS_VALU", 0), m.get("SQ_INSTS_SALU", 0), m.get("SQ_INSTS_LDS", 0),
            m.get("SQ_INSTS_VMEM_RD", 0), m.get("SQ_INSTS_VMEM_WR", 0), m.get("SQ_WAVE_CYCLES", 0),
            m.get("SQ_WAIT_ANY", 0) / max(1, m.get("SQ_WAVE_CYCLES", 1)),
            m.get("SQ_ACTIVE_INST_ANY", 0) / max(1, m.get("SQ_WAVE_CYCLES", 1)), util))
