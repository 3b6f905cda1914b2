#!/bin/bash
# conv_out channel groups (ERTD_CONV_OUT_NS 4 = default / 2 / 1): U-Net GPU
# tests, U2 fp32 and U3 bf16 probe A/B, and a U2 layer trace.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_unet.py tests/test_gpu_unet_ops.py -x -q --timeout 300 \
  --timeout-method thread -m gpu > gpurun_out/co_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/co_tests.log; [ $rc -ne 0 ] && exit $rc
VAR=ERTD_CONV_OUT_NS VALUES="4 1 4 1" STEPS=30 bash tools/ab.sh || exit $?
VAR=ERTD_CONV_OUT_NS VALUES="4 1" CFG=U3 B=256 PREC=bf16 STEPS=20 bash tools/ab.sh || exit $?
bash tools/layer_trace.sh > gpurun_out/lt_co.txt 2>&1; echo "[trace] rc=$?"; grep conv_out gpurun_out/lt_co.txt
exit 0
