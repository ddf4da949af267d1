"""Summarise a rocprofv3 kernel_stats.csv (dev tool): share, calls, average duration."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 16]:
    print(f"{float(r['TotalDurationNs']) / tot * 100:5.1f}% {int(r['Calls']):6d} "
          f"{float(r['AverageNs']) / 1e3:9.1f}us  {r['Name'][:96]}")
print(f"total {tot / 1e6:.2f} ms, per step {tot / 1e6 / steps:.2f} ms")
