#!/bin/bash
# wino4s xi-split variant (ERTD_WINO4S_XS=2): parity under the variant, then a
# U2 B=64 A/B against the default and a serialized layer trace under it.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
ERTD_WINO4S_XS=2 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_unet_ops.py tests/test_gpu_unet.py \
  -x -q --timeout 200 --timeout-method thread -m gpu -k "${XS_K:-conv2d or forward or sampler or chain}" > gpurun_out/xs_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -4 gpurun_out/xs_tests.log; [ $rc -ne 0 ] && exit $rc
VAR=ERTD_WINO4S_XS VALUES="1 2 1 2" STEPS=30 bash tools/ab.sh || exit $?
ERTD_WINO4S_XS=2 bash tools/layer_trace.sh > gpurun_out/lt_xs2.txt 2>&1; echo "[trace] rc=$?"
exit 0
