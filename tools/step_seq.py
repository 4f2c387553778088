"""One training step from a rocprofv3 kernel trace, kernel by kernel: start offset, duration,
stream, grid (workgroups), and how many other kernels overlap it -- to read the critical path.

python tools/step_seq.py <kernel_trace.csv> [--step K]   (K-th complete step from the end)
"""
import argparse
import csv
import re


def short(n):
    n = re.sub(r"\(.*", "", n).replace("void ", "").replace("oflow::", "")
    return n[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--step", type=int, default=1)
    args = ap.parse_args()
    rows = []
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r["Stream_Id"], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))))
    rows.sort()
    adam = [i for i, r in enumerate(rows) if re.search(r"adam_(dev_)?kernel", r[2])]
    k = len(adam) - args.step
    lo, hi = rows[adam[k - 1]][1], rows[adam[k]][1]
    ks = [r for r in rows if r[0] >= lo and r[1] <= hi]
    for s, e, n, st, g in ks:
        ov = sum(1 for s2, e2, *_ in ks if s2 < e and e2 > s) - 1
        print("%8.1f %7.1f  s%-2s wg%-6d ov%d  %s" % ((s - lo) / 1e3, (e - s) / 1e3, st, g, ov, short(n)))


if __name__ == "__main__":
    main()
