#!/bin/bash
# Winograd weight gradient: train tests, train-step A/B (ERTD_WGRAD_WINO), kernel profile
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_unet_train.py -x -q --timeout 300 --timeout-method thread -m gpu \
  > gpurun_out/wgw_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -4 gpurun_out/wgw_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 0 1; do
  ERTD_WGRAD_WINO=$v timeout -k 10 300 python3 tools/train_probe.py --steps 10 > gpurun_out/wgw_ab_$v.log 2>&1
  rc=$?; echo "[WGRAD_WINO=$v] rc=$rc $(tail -1 gpurun_out/wgw_ab_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
bash tools/gpu_train_prof.sh
