"""Summarise a rocprofv3 kernel_stats.csv: per-step time per kernel (sorted)."""
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e6:8.3f} ms/step {float(r['Percentage']):6.2f}% "
          f"calls/step {int(r['Calls']) / steps:6.1f} avg {float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:90]}")
print(f"total {tot / steps / 1e6:.3f} ms/step")
