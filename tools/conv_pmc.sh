#!/bin/bash
# SQ counters of one conv layer (diagnostic): one rocprofv3 --pmc pass over
# tools/conv_probe.py, per-dispatch averages of the conv kernel.
#   PROBE_ARGS="--B 64" COUNTERS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES ..." tools/conv_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
d=gpurun_out/cpmc; rm -rf "$d"
timeout -s KILL 120 rocprofv3 --pmc ${COUNTERS:?} --output-format csv -d "$d" -o run \
  -- python3 tools/conv_probe.py ${PROBE_ARGS:-} > "$d.log" 2>&1
rc=$?; echo "[pmc] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$d.log"; exit $rc; }
f=$(find "$d" -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "conv_wino" in r["Kernel_Name"] or "conv_kernel<" in r["Kernel_Name"] or "conv_bf16_kernel<" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    v = v[3:] if len(v) > 3 else v
    print(f"{k:32s} {sum(v) / len(v):16.0f}")
PY
