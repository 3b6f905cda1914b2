#!/bin/bash
# 1x1 weight-gradient GEMM (wg1_lds_kernel) check + same-box A/B (diagnostic):
# 1) the conv wgrad op tests; 2) the skip shapes timed (shipped plan), then
# every forced plan on the diag library; 3) the train step alternating the
# shipped library and variants/wg1off.so (-DWG1_LDS=0).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_unet_train.py -x -q --timeout 120 \
  --timeout-method thread -k "wgrad and not fused" > gpurun_out/wg1_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc $(tail -1 gpurun_out/wg1_tests.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 tools/wgrad_probe.py --skip > gpurun_out/wg1_probe.log 2>&1
rc=$?; cat gpurun_out/wg1_probe.log; [ $rc -ne 0 ] && exit $rc
for v in ${VARS:-wg1off}; do
  ERTD_LIB_PATH=$PWD/variants/$v.so timeout -k 10 120 python3 tools/wgrad_probe.py --skip \
    > gpurun_out/wg1_probe_$v.log 2>&1
  rc=$?; echo "[$v]"; cat gpurun_out/wg1_probe_$v.log; [ $rc -ne 0 ] && exit $rc
done
if [ "${SWEEP:-1}" = 1 ]; then
  ERTD_LIB_PATH=$PWD/ert-conditional-diffusion-model_amd/ertdiff/libertdiff_hip_diag.so \
    timeout -k 10 500 python3 -u tools/wgrad_probe.py --skip --sweep --reps 10 > gpurun_out/wg1_sweep.log 2>&1
  rc=$?; cat gpurun_out/wg1_sweep.log; [ $rc -ne 0 ] && exit $rc
fi
for k in 1 2; do
  for lib in base ${VARS:-wg1off}; do
    tag=$(basename $lib .so)
    if [ "$lib" = base ]; then unset ERTD_LIB_PATH; else export ERTD_LIB_PATH=$PWD/variants/$lib.so; fi
    timeout -k 10 200 python3 tools/train_probe.py --steps 100 > gpurun_out/wg1_$tag.log 2>&1
    rc=$?; echo "[$tag] rc=$rc $(tail -1 gpurun_out/wg1_$tag.log)"; [ $rc -ne 0 ] && exit $rc
  done
done
