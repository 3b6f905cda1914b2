#!/bin/bash
# GPU check of a change: selected -m gpu tests, then U2 probe A/B over env values
#   TESTS="tests/test_gpu_unet.py" VAR=ERTD_UNET_GNFUSE VALUES="1 0" tools/gpu_ab_probe.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
DIAG=$PWD/ert-conditional-diffusion-model_amd/ertdiff/libertdiff_hip_diag.so   # knobs: diagnostic build only
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu $TESTS > gpurun_out/gpu_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/gpu_tests.log; echo "[tests] rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
for v in ${VALUES:-1}; do
  env ERTD_LIB_PATH=$DIAG "${VAR:-ERTD_NONE}=$v" timeout -k 10 200 python3 tools/unet_probe.py --config "${CFG:-U2}" --B "${B:-64}" \
    --precision "${PREC:-fp32}" --steps "${STEPS:-30}" > gpurun_out/probe_$v.log 2>&1
  rc=$?; echo "[${VAR:-} = $v] rc=$rc $(tail -1 gpurun_out/probe_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
