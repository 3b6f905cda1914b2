#!/bin/bash
# rocprofv3 kernel traces of one U-Net probe per env value (diagnostic):
#   VAR=ERTD_UNET_GNFUSE VALUES="1 0" tools/gpu_trace_ab.sh -> gpurun_out/tr_<v>/ + per-kernel sums
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VALUES:?}; do
  d=gpurun_out/tr_$v; rm -rf "$d"
  env "${VAR:?}=$v" ERTD_UNET_SIDE=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run \
    -- python3 tools/unet_probe.py --config "${CFG:-U2}" --B "${B:-64}" --precision "${PREC:-fp32}" --steps 2 > "$d.log" 2>&1
  rc=$?; echo "[trace $v] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$d.log"; exit $rc; }
  f=$(find "$d" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'  {float(r["TotalDurationNs"])/1e3:10.1f} us  {int(r["Calls"]):5d} calls  {float(r["AverageNs"])/1e3:8.2f} us avg  {r["Name"][:90]}')
PY
done
exit 0
