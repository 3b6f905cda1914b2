#!/bin/bash
# round-5: U-Net tests, then U2 step time with the GroupNorm fold on / off
# (diagnostic library knob), then the production library's step timeline
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_unet.py tests/test_gpu_unet_ops.py tests/test_gpu_unet_train.py > gpurun_out/unet_tests.log 2>&1
rc=$?; tail -2 gpurun_out/unet_tests.log; echo "[unet tests] rc=$rc"; [ $rc -ne 0 ] && exit $rc
D=$PWD/ert-conditional-diffusion-model_amd/ertdiff/libertdiff_hip_diag.so
for rep in 1 2; do for k in 0 1; do
  echo -n "fold=$k: "; ERTD_LIB_PATH=$D ERTD_UNET_GNFOLD=$k timeout -k 10 60 python3 tools/unet_probe.py --config U2 --B 64 --steps 20 2>&1 | tail -1
done; done
echo -n "production: "; timeout -k 10 60 python3 tools/unet_probe.py --config U2 --B 64 --steps 20 2>&1 | tail -1
rm -rf gpurun_out/u2tl
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/u2tl -o run \
  -- python3 tools/unet_probe.py --config U2 --B 64 --steps 4 > gpurun_out/u2tl.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/u2tl.log; exit $rc; }
f=$(find gpurun_out/u2tl -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" --from-name conv_in_kernel --top 12
exit 0
