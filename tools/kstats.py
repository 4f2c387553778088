"""Summarise a rocprofv3 kernel_stats.csv (per-step ms assuming N steps)."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print("%-70s %6s %8.3f ms/step %6.2f%% avg %.3f ms" % (
        r['Name'][:70], r['Calls'], float(r['TotalDurationNs']) / 1e6 / steps,
        float(r['TotalDurationNs']) / tot * 100, float(r['AverageNs']) / 1e6))
print('total ms/step', tot / 1e6 / steps)
