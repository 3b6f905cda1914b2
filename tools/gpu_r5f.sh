#!/bin/bash
# A/B: XCD-aware wino4s walk (x1) vs blockIdx order (x0); conv1x1g K chunk 16/32 vs the implicit GEMM
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_unet_ops.py > gpurun_out/unet_ops.log 2>&1
rc=$?; tail -1 gpurun_out/unet_ops.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do for v in x0 x1; do
  echo -n "$v: "; ERTD_LIB_PATH=$PWD/variants/$v.so timeout -k 10 60 python3 tools/unet_probe.py --config U2 --B 64 --steps 20 2>&1 | tail -1
done; done
for k in 0 1 2; do
  d=gpurun_out/g1x1_$k; rm -rf $d
  ERTD_CONV1X1G=$k ERTD_LIB_PATH=$PWD/variants/gdiag.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
    -- python3 tools/unet_probe.py --config U2 --B 64 --steps 4 > $d.log 2>&1 || exit 1
  python3 - $d/run_kernel_stats.csv $k <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "conv1x1g" in n or "conv_kernel<1," in n:
        print(sys.argv[2], n.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1][:40], r["Calls"], f"{float(r['AverageNs'])/1e3:.2f}")
PY
done
