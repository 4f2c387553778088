"""Summarise a rocprofv3 SQ-counter pass (tools/gpu_r3r.sh) per conv kernel: the counters
averaged per dispatch, and the wave-cycle split of MI355X_MICROARCH.md's PMC table
(SQ_WAIT_ANY = parked at s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue stall, with its LDS
part SQ_WAIT_INST_LDS, SQ_ACTIVE_INST_ANY = issuing; the three add up to SQ_WAVE_CYCLES, all
in quad-cycles), MFMA busy per SIMD-cycle and the LDS bank-conflict share.

python tools/pmc_sq.py <counter_collection.csv> [kernel substring]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else "oflow::conv_"
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        if want not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"], r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        print("%s  (%d dispatches)" % (k[:100], n))
        wc = avg.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
                if c in avg:
                    print("    %-26s %6.1f %% of wave-cycles" % (c, 100.0 * avg[c] / wc))
        for c in sorted(avg):
            print("    %-26s %.4g" % (c, avg[c]))
        if "SQ_LDS_IDX_ACTIVE" in avg and avg["SQ_LDS_IDX_ACTIVE"]:
            print("    LDS bank-conflict cycles   %6.1f %% of LDS-active cycles" % (
                100.0 * avg.get("SQ_LDS_BANK_CONFLICT", 0.0) / avg["SQ_LDS_IDX_ACTIVE"]))


if __name__ == "__main__":
    main()
