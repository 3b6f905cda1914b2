#!/bin/bash
# conv_bwd_kernel ablations (diagnostic): per variant library (variants/cbw<N>.so,
# built on the CPU side with tools/build_variant.sh train "-DCBW_ABL=N"), the
# average conv_bwd_kernel duration over TrainPlan steps (rocprofv3 kernel trace).
#   CPU:  for n in 0 1 2 4 7; do tools/build_variant.sh train "-DCBW_ABL=$n" variants/cbw$n.so; done
#   GPU:  VARS="0 1 2 4 7" tools/cbw_abl.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for n in ${VARS:-0 1 2 4 7}; do
  d=gpurun_out/cbw$n; rm -rf $d
  ERTD_LIB_PATH=$PWD/variants/cbw$n.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
    -- python3 tools/train_ref_probe.py --steps 100 --plan-only > $d.log 2>&1 || { echo "[cbw$n] failed"; tail -3 $d.log; exit 1; }
  python3 - $d/run_kernel_stats.csv $n <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "conv_bwd" in r["Name"] or "enc_train" in r["Name"] or "final" in r["Name"] or "head_kernel<2>" in r["Name"]:
        print(f"ABL={sys.argv[2]:3s} {r['Name'].split('(')[0][-28:]:28s} {float(r['AverageNs'])/1e3:8.2f} us")
PY
done
