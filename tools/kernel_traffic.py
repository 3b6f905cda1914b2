"""Per-kernel HBM bytes per launch from two rocprofv3 --pmc passes (diagnostic):
    python tools/kernel_traffic.py <fetch_dir> <write_dir> [name-substring ...]
bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count)."""
import collections
import csv
import glob
import os
import sys


def rows(d, counter):
    out = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                out[r["Kernel_Name"].split("(")[0][-70:]].append(float(r["Counter_Value"]))
    return out


fd, wd = sys.argv[1], sys.argv[2]
subs = sys.argv[3:]
fr, wr = rows(fd, "FETCH_SIZE"), rows(wd, "WRITE_SIZE")
for k in sorted(fr, key=lambda k: -sum(fr[k])):
    if subs and not any(s in k for s in subs):
        continue
    f = sorted(fr[k])[len(fr[k]) // 2]
    w = sorted(wr.get(k, [0]))[len(wr.get(k, [0])) // 2]
    print(f"{k:70s} n={len(fr[k]):4d} read {2 * f / 1024:9.1f} MB  write {w / 1024:9.1f} MB (median per launch)")
