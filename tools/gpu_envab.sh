#!/bin/bash
# Same-box A/B of environment knobs on the U-Net step (diagnostic): per
# setting (";"-separated list of space-separated VAR=value sets, "-" = none),
# the rocprofv3 kernel averages matching KPAT and the probe's step time.
#   SETS="-;ERTD_UNET_TPX1=1" KPAT="conv_kernel<1" tools/gpu_envab.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
IFS=';' read -ra S <<< "${SETS:?}"
i=0
for set in "${S[@]}"; do
  [ "$set" = "-" ] && set=""
  d=gpurun_out/eab_$i; rm -rf $d
  env $set timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
    -- python3 tools/unet_probe.py --config ${CFG:-U2} --B ${B:-64} --steps 4 > $d.log 2>&1 || { echo "[$set] failed"; tail -3 $d.log; exit 1; }
  python3 - $d/run_kernel_stats.csv "${set:--}" "${KPAT:?}" <<'PY'
import csv, re, sys
out = []
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], r["Name"]):
        nm = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1][:40]
        out.append(f"{nm} {float(r['AverageNs'])/1e3:7.2f} us x{r['Calls']}")
print(f"{sys.argv[2]:28s}", " | ".join(out))
PY
  echo -n "${set:--}: "; env $set timeout -k 10 60 python3 tools/unet_probe.py --config ${CFG:-U2} --B ${B:-64} --steps 20 2>&1 | tail -1
  i=$((i + 1))
done
