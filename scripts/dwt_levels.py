"""Per-launch DWT kernel durations from a rocprofv3 --kernel-trace CSV run
(scripts/dwt_levels.sh): prints every k_dwt / k_dcshift launch in order with
its grid and duration, then the per-level minimum over repeats."""
import csv
import glob
import sys
from collections import defaultdict

rows = []
for p in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    with open(p) as f:
        rows += list(csv.DictReader(f))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
seq = [r for r in rows if "dwt" in r["Kernel_Name"] or "dcshift" in r["Kernel_Name"] or "mct_inv" in r["Kernel_Name"]]
best = defaultdict(lambda: 1e30)
for r in seq:
    name = r["Kernel_Name"].split("(")[0].replace("void grkgpu::", "")
    g = "%sx%s" % (r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("Grid_Size_Y", ""))
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    key = (name, g)
    best[key] = min(best[key], d)
for (name, g), d in best.items():
    print("%-50s grid %-14s best %8.2f us" % (name, g, d))
