#!/bin/bash
# Environment A/B of the U-Net sampler on the GPU box (diagnostic).
#
#   VAR=ERTD_UNET_SIDE VALUES="1 0 1" CFG=U2 B=64 PREC=fp32 STEPS=50 tools/ab.sh
#
# Runs tools/unet_probe.py once per value of $VAR (each run under its own
# time limit; stops at the first failure) and prints the probe's summary line.
# The knobs (ERTD_UNET_SIDE, ERTD_WINO4S*, ERTD_UNET_TPX, ...: csrc/unet.h
# ERTD_KNOB) are read only by the diagnostic build, which this script loads:
# build it first on the CPU side (build.py --diag).  VAR=ERTD_LIB_PATH compares
# variant libraries (tools/build_variant.sh) instead.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
[ "${VAR:-}" != ERTD_LIB_PATH ] && export ERTD_LIB_PATH=$PWD/ert-conditional-diffusion-model_amd/ertdiff/libertdiff_hip_diag.so
VAR=${VAR:?set VAR to the environment variable to vary}
for v in ${VALUES:?set VALUES}; do
  env "$VAR=$v" timeout -k 10 300 python3 tools/unet_probe.py --config "${CFG:-U2}" --B "${B:-64}" \
    --precision "${PREC:-fp32}" --steps "${STEPS:-50}" > "gpurun_out/ab_${VAR}_${v//\//_}.log" 2>&1
  rc=$?
  echo "[$VAR=$v] rc=$rc $(tail -1 "gpurun_out/ab_${VAR}_${v//\//_}.log")"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
