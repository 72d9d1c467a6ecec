"""Print per-kernel SQ counter sums from rocprofv3 csv runs (scripts/pmc_sq.sh)."""
import collections, csv, glob, os, sys
for d in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            acc[r["Kernel_Name"].split("(")[0][-40:]][r["Counter_Name"]] += float(r["Counter_Value"])
    print("==", d)
    for k, v in acc.items():
        if "t1" not in k and "dwt" not in k:
            continue
        w = v.get("SQ_WAVES", 1) or 1
        print("%-40s waves %7d  valu/wave %9.0f salu/wave %8.0f lds/wave %8.0f cyc/wave %10.0f wait %.2f waitinst %.2f active %.2f" % (
            k, w, v["SQ_INSTS_VALU"] / w, v["SQ_INSTS_SALU"] / w, v["SQ_INSTS_LDS"] / w, v["SQ_WAVE_CYCLES"] / w,
            v["SQ_WAIT_ANY"] / max(v["SQ_WAVE_CYCLES"], 1), v["SQ_WAIT_INST_ANY"] / max(v["SQ_WAVE_CYCLES"], 1),
            v["SQ_ACTIVE_INST_ANY"] / max(v["SQ_WAVE_CYCLES"], 1)))
