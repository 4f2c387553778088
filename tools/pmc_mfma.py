"""MFMA utilisation per kernel from one rocprofv3 PMC pass of `python bench.py` with
SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE, merged into
profiles/pmc_traffic.json next to the HBM bytes of the same configuration.

Per dispatch (MI355X_MICROARCH.md, PMC notes): GRBM_GUI_ACTIVE is summed over the 8 XCDs, so
the kernel's cycles are GRBM_GUI_ACTIVE / 8; SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy cycles
summed over every SIMD (32 per v_mfma_f32_32x32x16_bf16, 16 per 16x16x32); the chip has
256 CUs x 4 SIMDs.  mfma_busy = MFMA_BUSY / (1024 * GRBM_GUI_ACTIVE / 8), averaged over the
kernel's dispatches (a dispatch shorter than ~0.3 ms reads its GRBM clock high, so short
kernels read low).  sq_busy = SQ_BUSY_CYCLES / (GRBM_GUI_ACTIVE) (the SQ's own busy share, per
XCD-summed cycle).

Usage: python tools/pmc_mfma.py <counter_collection.csv> H W B [precision]
"""
import csv
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4
XCDS = 8


def main():
    path, H, W, B = sys.argv[1:5]
    prec = sys.argv[5] if len(sys.argv) > 5 else "fp32"
    by = defaultdict(dict)          # (kernel, dispatch) -> counter -> value
    for r in csv.DictReader(open(path)):
        key = (r["Kernel_Name"], r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        by[key][r["Counter_Name"]] = by[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    acc = defaultdict(lambda: {"n": 0, "mfma": 0.0, "sq": 0.0, "grbm": 0.0, "busy": []})
    for (k, _), cs in by.items():
        g = cs.get("GRBM_GUI_ACTIVE", 0.0)
        if g <= 0 or "SQ_VALU_MFMA_BUSY_CYCLES" not in cs:
            continue
        a = acc[k]
        a["n"] += 1
        a["mfma"] += cs["SQ_VALU_MFMA_BUSY_CYCLES"]
        a["sq"] += cs.get("SQ_BUSY_CYCLES", 0.0)
        a["grbm"] += g
        a["busy"].append(cs["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * g / XCDS))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dbp = os.path.join(root, "profiles", "pmc_traffic.json")
    db = json.load(open(dbp)) if os.path.exists(dbp) else {"entries": {}}
    ent = db.setdefault("entries", {}).setdefault("%s:%sx%sx%s" % (prec, H, W, B), {
        "config": [int(H), int(W), int(B)], "precision": prec, "kernels": {}})
    ent["mfma_note"] = ("mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / "
                        "8 XCDs), mean over the kernel's dispatches of one bench run "
                        "(tools/pmc_mfma.py)")
    rows = []
    for k, a in acc.items():
        if a["n"] == 0:
            continue
        busy = sum(a["busy"]) / len(a["busy"])
        kc = a["grbm"] / XCDS / a["n"]
        e = ent["kernels"].setdefault(k, {})
        e["mfma_busy"] = round(busy, 4)
        e["sq_busy"] = round(a["sq"] / a["grbm"], 4) if a["grbm"] else None
        e["mfma_dispatches"] = a["n"]
        e["cycles_per_dispatch"] = round(kc)
        rows.append((a["grbm"], k, busy, a["n"], kc))
    with open(dbp, "w") as fh:
        json.dump(db, fh, indent=1)
    rows.sort(reverse=True)
    print("| kernel | dispatches | cycles / dispatch | MFMA busy |")
    print("|---|---|---|---|")
    for _, k, busy, n, kc in rows[:25]:
        print("| `%s` | %d | %.0f | %.1f %% |" % (k[:90], n, kc, 100 * busy))


if __name__ == "__main__":
    main()
