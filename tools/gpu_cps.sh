#!/bin/bash
# Implicit-GEMM wgrad K split (diagnostic): the train step on the diag library
# under ERTD_WGRAD_WPC / ERTD_WGRAD_CPS values.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
export ERTD_LIB_PATH=$PWD/ert-conditional-diffusion-model_amd/ertdiff/libertdiff_hip_diag.so
for kv in "4 4" "4 2" "4 1" "8 1" "8 2"; do
  set -- $kv
  ERTD_WGRAD_WPC=$1 ERTD_WGRAD_CPS=$2 timeout -k 10 200 python3 tools/train_probe.py --steps 100 > gpurun_out/cps.log 2>&1
  rc=$?; echo "[wpc=$1 cps=$2] rc=$rc $(tail -1 gpurun_out/cps.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
