#!/bin/bash
# conv_in / conv_out weight gradients (wgt_kernel): op tests, then a kernel
# trace of the train step with the shipped library and each variants/<VARS>.so,
# per-kernel averages printed.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_unet_train.py -x -q --timeout 120 \
  --timeout-method thread -k "wgrad" > gpurun_out/wgt_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc $(tail -1 gpurun_out/wgt_tests.log)"; [ $rc -ne 0 ] && exit $rc
for v in base ${VARS:-}; do
  if [ $v != base ]; then export ERTD_LIB_PATH=$PWD/variants/$v.so; fi
  rm -rf gpurun_out/wgt_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wgt_$v -o run \
    -- python3 tools/train_probe.py --steps 10 > gpurun_out/wgt_$v.log 2>&1
  rc=$?; echo "[$v] rc=$rc $(tail -1 gpurun_out/wgt_$v.log | grep -o 'train: .*ms/step')"; [ $rc -ne 0 ] && exit $rc
  python3 - gpurun_out/wgt_$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "wgt_kernel" in r["Name"] or "gemm_small" in r["Name"]:
        print(f'  {r["Name"][:60]:60s} {int(r["Calls"]):4d} avg {float(r["AverageNs"]) / 1000:7.1f} us')
PY
done
