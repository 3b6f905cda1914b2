"""Summarize a rocprofv3 kernel_stats.csv: python tools/prof_summary.py <csv> <steps> [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
tot = sum(float(x["TotalDurationNs"]) for x in rows)
print(f"kernel time per step: {tot / steps / 1e6:.3f} ms")
for x in sorted(rows, key=lambda x: -float(x["TotalDurationNs"]))[:top]:
    print(f"{float(x['TotalDurationNs']) / steps / 1e6:8.3f} ms {int(x['Calls']) / steps:6.1f} calls "
          f"{float(x['AverageNs']) / 1e3:8.1f} us  {x['Name'][:80]}")
