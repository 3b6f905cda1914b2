#!/bin/bash
# skip-conv side branch of the step graph: U-Net GPU tests, then bench A/B
# (ERTD_UNET_SIDE=1 branch / 0 single chain), U2 fp32 and U3 bf16
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_unet.py tests/test_gpu_unet_ops.py > gpurun_out/side_tests.log 2>&1
rc=$?; tail -5 gpurun_out/side_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1; do
  ERTD_UNET_SIDE=$v timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-kde --no-reference \
    --no-cpu-baseline > gpurun_out/side_$v.log 2>&1
  rc=$?; echo "[side=$v] rc=$rc"; [ $rc -ne 0 ] && exit $rc
  grep '^{' gpurun_out/side_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['extra']['configs2_u3_bf16']['value'])"
done
exit 0
