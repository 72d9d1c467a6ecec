"""Summarise scripts/pmc_dwt_variants.sh output: per DWT kernel (grid) counter sums per dispatch."""
import csv
import glob
import sys
from collections import defaultdict

for vd in sorted(glob.glob(sys.argv[1] + "/v*")):
    acc = defaultdict(lambda: defaultdict(float))
    nd = defaultdict(set)
    for f in glob.glob(vd + "/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "dwt" not in k:
                continue
            key = (k.split("(")[0][-34:], r.get("Grid_Size", ""))
            acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
            nd[key, r["Counter_Name"]].add(r["Dispatch_Id"])
    print("==", vd)
    for key, v in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:4]:
        per = {c: v[c] / max(1, len(nd[key, c])) for c in v}
        w = per.get("SQ_WAVES", 1) or 1
        print("  %-34s grid %9s" % key,
              "waves %6d cyc/wave %6.0f busy %8.0f wait %.2f waitinst %.2f valu %.2f vmem %.2f | fetch %.0f MB hit %.2f write %.0f MB dramrd %.0f MB" % (
                  w, per.get("SQ_WAVE_CYCLES", 0) / w, per.get("SQ_BUSY_CYCLES", 0),
                  per.get("SQ_WAIT_ANY", 0) / max(1, per.get("SQ_WAVE_CYCLES", 1)),
                  per.get("SQ_WAIT_INST_ANY", 0) / max(1, per.get("SQ_WAVE_CYCLES", 1)),
                  per.get("SQ_ACTIVE_INST_VALU", 0) / max(1, per.get("SQ_WAVE_CYCLES", 1)),
                  per.get("SQ_ACTIVE_INST_VMEM", 0) / max(1, per.get("SQ_WAVE_CYCLES", 1)),
                  per.get("FETCH_SIZE", 0) * 2 / 1024, per.get("TCC_HIT_sum", 0) / max(1, per.get("TCC_HIT_sum", 0) + per.get("TCC_MISS_sum", 0)),
                  per.get("WRITE_SIZE", 0) / 1024, per.get("TCC_EA0_RDREQ_DRAM_sum", 0) * 64 / 1e6))
