#!/bin/bash
# F(4x4) register-weight variant (ERTD_WINO4S): parity under the variant, then
# a U2 B=64 probe A/B over its settings and a serialized layer trace.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
ERTD_WINO4S=${W4S_TEST:-2} timeout -k 10 600 python3 -u -m pytest tests/test_gpu_unet_ops.py tests/test_gpu_unet.py \
  -x -q --timeout 200 --timeout-method thread -m gpu -k "${W4S_K:-conv2d or forward or sampler or chain}" > gpurun_out/w4s_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -4 gpurun_out/w4s_tests.log; [ $rc -ne 0 ] && exit $rc
VAR=ERTD_WINO4S VALUES="${W4S_AB:-0 1 2 3}" STEPS=30 bash tools/ab.sh || exit $?
ERTD_WINO4S=${W4S_TRACE:-2} bash tools/layer_trace.sh > gpurun_out/lt_w4s.txt 2>&1; echo "[trace] rc=$?"
exit 0
