#!/bin/bash
# 1x1 conv kernel: op + model parity, U2 probe A/B (ERTD_CONV1X1), serialized layer trace
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_unet_ops.py tests/test_gpu_unet.py \
  -x -q --timeout 200 --timeout-method thread -m gpu -k "conv2d or forward or sampler or chain" > gpurun_out/c11_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -4 gpurun_out/c11_tests.log; [ $rc -ne 0 ] && exit $rc
VAR=ERTD_CONV1X1 VALUES="0 1 2" STEPS=40 bash tools/ab.sh || exit $?
bash tools/layer_trace.sh > gpurun_out/lt_U2.txt 2>&1; echo "[trace] rc=$?"
