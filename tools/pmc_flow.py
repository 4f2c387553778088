"""Summarise rocprofv3 --pmc passes of tools/flow_bench.py (tools/gpu_pmc_flow4.sh): per kernel
and grid size, the mean of each counter per dispatch (FETCH_SIZE / WRITE_SIZE in KiB as
reported: FETCH_SIZE under-counts 16-B/lane loads 2x on gfx950, MI355X_MICROARCH.md).

python tools/pmc_flow.py gpurun_out/pmc_flow4
"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    root = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(root, "*", "fb_counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("oflow::", "")
            if not any(k in name for k in ("corr", "warp", "det_", "fill")):
                continue
            key = (name, int(r["Grid_Size"]))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    cols = ["FETCH_SIZE", "WRITE_SIZE", "SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY",
            "SQ_WAIT_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_LDS",
            "SQ_LDS_BANK_CONFLICT"]
    print("kernel grid " + " ".join(cols))
    for (name, grid), d in sorted(acc.items(), key=lambda x: (x[0][0], -x[0][1])):
        vals = []
        for c in cols:
            v = d.get(c)
            vals.append("%.4g" % (sum(v) / len(v)) if v else "-")
        print(name[:40], grid, " ".join(vals))


if __name__ == "__main__":
    main()
