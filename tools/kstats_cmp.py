"""Per-kernel totals per step of two rocprofv3 kernel traces (diagnostic):
    python tools/kstats_cmp.py A_kernel_trace.csv B_kernel_trace.csv STEPS"""
import csv
import sys
from collections import defaultdict


def load(f):
    d = defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ertd::unet::", "")[:70]
        d[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return d


a, b, n = load(sys.argv[1]), load(sys.argv[2]), float(sys.argv[3])
keys = sorted(set(a) | set(b), key=lambda k: -max(a.get(k, 0), b.get(k, 0)))
print(f"{'kernel':70s} {'A us/step':>10s} {'B us/step':>10s}")
for k in keys[:30]:
    print(f"{k:70s} {a.get(k, 0) / n:10.1f} {b.get(k, 0) / n:10.1f}")
print(f"{'TOTAL':70s} {sum(a.values()) / n:10.1f} {sum(b.values()) / n:10.1f}")
