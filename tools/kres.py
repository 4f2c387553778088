"""Per-kernel register / spill / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage
output on stdin:  hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kres.py"""
import re
import sys

rows, cur = {}, None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1).replace("_ZN5oflow", "")
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0] + ("S" if "Spill" in m.group(1) else "")] = m.group(2)
for k, v in rows.items():
    print("%-64s vgpr %4s agpr %4s spill %3s occ %2s lds %6s" % (
        k[:64], v.get("VGPRs"), v.get("AGPRs"), v.get("VGPRsS"), v.get("Occupancy"), v.get("LDS")))
