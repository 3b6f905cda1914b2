#!/bin/bash
# xi-split wino4s K split at 16x16 (ERTD_WINO4S_KSPLIT): op/train/U-Net GPU
# tests, then the U2 B=32 train-step A/B and the U2 B=64 sampler (unchanged path).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_unet_ops.py tests/test_gpu_unet_train.py tests/test_gpu_unet.py \
  -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/w4ks_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/w4ks_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  ERTD_WINO4S_KSPLIT=$v timeout -k 10 300 python3 tools/train_probe.py --config U2 --B 32 --steps 30 > gpurun_out/w4ks_$v.log 2>&1
  rc=$?; echo "[KSPLIT=$v] rc=$rc $(tail -1 gpurun_out/w4ks_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
VAR=ERTD_WINO4S_KSPLIT VALUES="1 0" STEPS=30 bash tools/ab.sh || exit $?
exit 0
