#!/bin/bash
# Same-box A/B of variant libraries on the reference train step (diagnostic):
# per variant (variants/<name>.so), TrainPlan timing + the kernel averages.
#   LIBS="cbwa3 cbwa6 cbwa10" tools/gpu_libab.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for n in ${LIBS:?}; do
  d=gpurun_out/lab_$n; rm -rf $d
  ERTD_LIB_PATH=$PWD/variants/$n.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
    -- python3 tools/train_ref_probe.py --steps 200 --plan-only > $d.log 2>&1 || { echo "[$n] failed"; tail -3 $d.log; exit 1; }
  grep "TrainPlan.run" $d.log | sed "s/^/$n rep$rep: /" | cut -c1-100
  python3 - $d/run_kernel_stats.csv $n <<'PY'
import csv, sys
out = []
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("conv_bwd", "enc_train", "final_kernel", "head_kernel<2>")) and int(r["Calls"]) > 10:
        out.append(f"{r['Name'].split('(')[0].split('::')[-1][:18]} {float(r['AverageNs'])/1e3:6.2f}")
print("   ", " | ".join(out))
PY
done
done
