#!/bin/bash
# fp32 sub-pixel Upsample conv: U-Net op + model GPU tests, U2 B=64 probe, kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_unet_ops.py tests/test_gpu_unet.py > gpurun_out/upp_tests.log 2>&1
rc=$?; tail -15 gpurun_out/upp_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 tools/unet_probe.py --config U2 --B 64 --steps 5 2>&1 | grep -v amdgpu.ids
rc=$?; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/uppt
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/uppt -o run \
  -- python3 tools/unet_probe.py --config U2 --B 64 --steps 2 > gpurun_out/uppt.log 2>&1
exit $?
