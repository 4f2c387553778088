"""Turn two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of `python bench.py` into HBM bytes
per launch for every liboflow kernel (template instance) -> profiles/pmc_traffic.json.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) counts 128-B requests of wide
coalesced reads as 64 B, i.e. half the bytes of 16-B/lane loads -> doubled here; WRITE_SIZE
(KiB) is exact for 16-B stores / dword atomics (the conv epilogue stores dwords: uncalibrated,
reported as-is).  Usage: python tools/pmc_traffic.py <fetch_csv> <write_csv> H W B [precision]
The entry is stored under "precision:HxWxB" in profiles/pmc_traffic.json (bench.py reads the
entry of its own configuration).
"""
import csv
import json
import os
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    fetch_csv, write_csv, H, W, B = sys.argv[1:6]
    prec = sys.argv[6] if len(sys.argv) > 6 else "fp32"
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    # the fp32 PMC passes of the round script run the default fp32 path (split kernels on)
    out = {"config": [int(H), int(W), int(B)], "precision": prec, "kernels": {},
           "f32_split": os.environ.get("OFLOW_F32_SPLIT", "1") == "1",
           "note": "bytes per launch = 2*FETCH_SIZE*1024 (gfx950 half-count correction for "
                   "16-B/lane loads) + WRITE_SIZE*1024; averaged over all launches of the "
                   "bench command (mixed layer shapes)"}
    for k in f:
        # (conv_b16i.hip's kernels live in an anonymous namespace: oflow::(anonymous namespace)::)
        if "oflow::" not in k or k not in w:        # every liboflow kernel
            continue
        fb = sum(f[k]) / len(f[k]) * 1024 * 2
        wb = sum(w[k]) / len(w[k]) * 1024
        out["kernels"][k] = {"launches": len(f[k]), "fetch_bytes": fb, "write_bytes": wb,
                             "hbm_bytes_per_launch": fb + wb}
    convs = [k for k in out["kernels"] if "conv_" in k]
    dom = max(convs, key=lambda k: out["kernels"][k]["launches"] *
              out["kernels"][k]["hbm_bytes_per_launch"]) if convs else None
    out["kernel"] = dom
    if dom:
        out["hbm_bytes_per_launch"] = out["kernels"][dom]["hbm_bytes_per_launch"]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "profiles", "pmc_traffic.json")
    db = {}
    if os.path.exists(path):
        with open(path) as fh:
            db = json.load(fh)
        if "entries" not in db:             # the round-2 single-entry file
            db = {"entries": {}}
    db.setdefault("entries", {})["%s:%sx%sx%s" % (prec, H, W, B)] = out
    with open(path, "w") as fh:
        json.dump(db, fh, indent=1)
    print(json.dumps({k: round(v["hbm_bytes_per_launch"] / 1e6, 2)
                      for k, v in out["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()
