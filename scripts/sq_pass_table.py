"""Per-kernel SQ counters from rocprofv3 --pmc pass directories (scripts/gpu_sq.sh):
python scripts/sq_pass_table.py DIR1 DIR2 ...  (values per dispatch, averaged)"""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for d in sys.argv[1:]:
    for p in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void grkgpu::", "").replace("grkgpu::", "")
            if "t1" not in k and "dwt" not in k:
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(k, r["Counter_Name"])] += 1
for k, c in sorted(agg.items()):
    m = {name: v / n[(k, name)] for name, v in c.items()}
    util = m.get("SQ_THREAD_CYCLES_VALU", 0) / max(1, 64 * m.get("SQ_ACTIVE_INST_VALU", 1))
    print("%-36s valu %.3g salu %.3g lds %.3g vmem %.3g/%.3g wave_cyc %.3g wait %.2f active %.2f lane_util %.2f" % (
        k[:36], m.get("SQ_INSTS_VALU", 0), m.get("SQ_INSTS_SALU", 0), m.get("SQ_INSTS_LDS", 0),
        m.get("SQ_INSTS_VMEM_RD", 0), m.get("SQ_INSTS_VMEM_WR", 0), m.get("SQ_WAVE_CYCLES", 0),
        m.get("SQ_WAIT_ANY", 0) / max(1, m.get("SQ_WAVE_CYCLES", 1)),
        m.get("SQ_ACTIVE_INST_ANY", 0) / max(1, m.get("SQ_WAVE_CYCLES", 1)), util))
