#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_unet.py tests/test_gpu_unet_ops.py tests/test_gpu_unet_train.py > gpurun_out/unet_tests.log 2>&1
rc=$?; tail -1 gpurun_out/unet_tests.log; [ $rc -ne 0 ] && { grep -m3 "Error\|assert" gpurun_out/unet_tests.log; exit $rc; }
for rep in 1 2; do for v in xcd0 xcd1; do
  echo -n "$v: "; ERTD_LIB_PATH=$PWD/variants/$v.so timeout -k 10 60 python3 tools/unet_probe.py --config U2 --B 64 --steps 20 2>&1 | tail -1
done; done
for rep in 1 2; do for k in 0 1; do
  echo -n "conv1x1g=$k: "; ERTD_CONV1X1G=$k ERTD_LIB_PATH=$PWD/variants/gdiag.so timeout -k 10 60 python3 tools/unet_probe.py --config U2 --B 64 --steps 20 2>&1 | tail -1
done; done
for k in 0 1; do
  d=gpurun_out/g1x1_$k; rm -rf $d
  ERTD_CONV1X1G=$k ERTD_LIB_PATH=$PWD/variants/gdiag.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
    -- python3 tools/unet_probe.py --config U2 --B 64 --steps 4 > $d.log 2>&1 || exit 1
  python3 - $d/run_kernel_stats.csv $k <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "conv1x1" in n or "conv_kernel<1," in n:
        print(sys.argv[2], n.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1][:40], r["Calls"], f"{float(r['AverageNs'])/1e3:.2f}")
PY
done
for k in 0 1; do
  d=gpurun_out/co_$k; rm -rf $d
  ERTD_CONV_OUT64=$k ERTD_LIB_PATH=$PWD/variants/codiag.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
    -- python3 tools/unet_probe.py --config U2 --B 64 --steps 4 > $d.log 2>&1 || exit 1
  python3 - $d/run_kernel_stats.csv $k <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "conv_out" in n:
        print("conv_out64 =", sys.argv[2], n.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1][:40], r["Calls"], f"{float(r['AverageNs'])/1e3:.2f}")
PY
done
