#!/bin/bash
# bf16 fused GN prologue: op + U-Net GPU tests, then U3 B=256 probe A/B
# (ERTD_UNET_BF16_FUSEGN=1 fused / 0 gn_stats + act pass) and a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_unet_ops.py tests/test_gpu_unet.py > gpurun_out/fg_tests.log 2>&1
rc=$?; tail -15 gpurun_out/fg_tests.log; [ $rc -ne 0 ] && exit $rc
for f in 1 0 1; do
  ERTD_UNET_BF16_FUSEGN=$f timeout -k 10 120 python3 tools/unet_probe.py --config U3 --B 256 --steps 3 --precision bf16 2>&1 | grep -v amdgpu.ids
  rc=$?; echo "[fuse=$f] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
rm -rf gpurun_out/fgp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fgp -o run \
  -- python3 tools/unet_probe.py --config U3 --B 256 --steps 2 --precision bf16 > gpurun_out/fgp.log 2>&1
exit $?
