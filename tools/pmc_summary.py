"""Average PMC counters per (kernel, grid size) over the passes written by gpu_pmc_cmd.sh.

python tools/pmc_summary.py OUTDIR [kernel-substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(os.path.join(out, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if flt not in name:
            continue
        key = (name[:60], int(r["Grid_Size"]), int(r["VGPR_Count"]), int(r["LDS_Block_Size"]))
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for key in sorted(vals):
    print("%s grid=%d vgpr=%d lds=%d  dur~%.1f us" % (key + (sum(dur[key]) / len(dur[key]),)))
    for cn, v in sorted(vals[key].items()):
        print("    %-24s %16.0f" % (cn, sum(v) / len(v)))
