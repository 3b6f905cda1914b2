"""Per-conv efficiency from a rocprofv3 kernel trace of bench.py (diagnostic).

    python tools/conv_trace.py gpurun_out/prof/run_kernel_trace.csv

Groups conv_kernel<KS,MODE,ACT,WCO,WO> dispatches by (template, grid) and
prints mean duration; FLOP per dispatch needs Cin, so it is reported for the
known U2 layer shapes via --cin lookups where unique."""
import collections
import csv
import re
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "conv_kernel<" in r["Kernel_Name"]]
g = collections.defaultdict(list)
for r in rows:
    m = re.search(r"conv_kernel<(\d+), (\d+), (\d+), (\d+), (\d+)>", r["Kernel_Name"])
    key = (m.groups(), int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]),
           int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]), r["LDS_Block_Size"], r["VGPR_Count"],
           r["Accum_VGPR_Count"])
    g[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
tot = sum(sum(v) for v in g.values())
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    (ks, mode, act, wco, wo), gx, gy, gz, lds, vg, ag = k
    print(f"ks{ks} mode{mode} act{act} wco{wco} wo{wo:>3s} grid {gx:4d}x{gy:2d}x{gz:3d} "
          f"lds {lds:>6s} vgpr {vg}+{ag}  n {len(v):4d}  mean {sum(v)/len(v):8.1f} us  "
          f"share {sum(v)/tot*100:5.1f}%")
