#!/bin/bash
# Upsample-conv Winograd wgrad + the xi-split wino4s default: the train/op GPU
# tests, then the U2 B=32 train-step A/B (ERTD_WGRAD_WINO 1 = with the
# Upsample convs, 2 = stride-1 only) and a kernel trace of the step.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_unet_train.py tests/test_gpu_unet_ops.py -x -q --timeout 300 \
  --timeout-method thread -m gpu > gpurun_out/wgup_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -4 gpurun_out/wgup_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 1 2 1 2; do
  ERTD_WGRAD_WINO=$v timeout -k 10 300 python3 tools/train_probe.py --config U2 --B 32 --steps 30 > gpurun_out/wgup_$v.log 2>&1
  rc=$?; echo "[WGRAD_WINO=$v] rc=$rc $(tail -1 gpurun_out/wgup_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
