"""Per-kernel counters per dispatch from scripts/gpu_run.sh dwtpmc runs:
python scripts/pmc_dwt_summary.py gpurun_out/TAG/s1 ... (FETCH_SIZE doubled for
gfx950's half count, KiB -> bytes)."""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    nd = collections.defaultdict(set)
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("grkgpu::", "")
            if "dwt" not in k and "dcshift" not in k:
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            nd[(k, r["Counter_Name"])].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    print("==", d, open(os.path.join(d, "SQ_WA.log")).read().strip()[-40:] if os.path.exists(os.path.join(d, "SQ_WA.log")) else "")
    for k, v in sorted(acc.items()):
        def per(c):
            n = len(nd[(k, c)]) or 1
            return v.get(c, 0.0) / n
        w = per("SQ_WAVES") or 1
        line = "%-48s" % k[:48]
        if "SQ_WAVES" in v:
            cyc = max(per("SQ_WAVE_CYCLES"), 1)
            line += " waves %6d valu/w %7.0f salu/w %6.0f cyc/w %8.0f wait %.2f waitinst %.2f valu_act %.2f any_act %.2f" % (
                w, per("SQ_INSTS_VALU") / w, per("SQ_INSTS_SALU") / w, cyc / w, per("SQ_WAIT_ANY") / cyc,
                per("SQ_WAIT_INST_ANY") / cyc, per("SQ_ACTIVE_INST_VALU") / cyc, per("SQ_ACTIVE_INST_ANY") / cyc)
        if "FETCH_SIZE" in v:
            line += " read %.1f MB" % (2 * per("FETCH_SIZE") * 1024 / 1e6)
        if "WRITE_SIZE" in v:
            line += " write %.1f MB" % (per("WRITE_SIZE") * 1024 / 1e6)
        print(line)
