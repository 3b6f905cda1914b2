#!/bin/bash
# wgw_gemm prefetch depth (WGW_SETS 3 / 4 = default / 5 via variant libraries
# in variants/): wgrad op tests, then the U2 B=32 train-step A/B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_unet_train.py -x -q --timeout 300 --timeout-method thread \
  -m gpu > gpurun_out/wgws_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/wgws_tests.log; [ $rc -ne 0 ] && exit $rc
for v in default wgw3 wgw5 default wgw3 wgw5; do
  if [ $v = default ]; then L=""; else L=$R/variants/$v.so; fi
  ERTD_LIB_PATH=$L timeout -k 10 300 python3 tools/train_probe.py --config U2 --B 32 --steps 30 > gpurun_out/wgws_$v.log 2>&1
  rc=$?; echo "[$v] rc=$rc $(tail -1 gpurun_out/wgws_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
