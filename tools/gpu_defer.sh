#!/bin/bash
# Deferred GN dgamma/dbeta reductions (ERTD_DEFER_REDUCE): train/op GPU tests,
# then the U2 B=32 train-step A/B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_unet_train.py tests/test_gpu_unet.py -x -q --timeout 300 \
  --timeout-method thread -m gpu > gpurun_out/defer_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/defer_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  ERTD_DEFER_REDUCE=$v timeout -k 10 300 python3 tools/train_probe.py --config U2 --B 32 --steps 30 > gpurun_out/defer_$v.log 2>&1
  rc=$?; echo "[DEFER=$v] rc=$rc $(tail -1 gpurun_out/defer_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
