#!/bin/bash
# Environment A/B of the U-Net sampler on the GPU box (diagnostic).
#
#   VAR=ERTD_UNET_SIDE VALUES="1 0 1" CFG=U2 B=64 PREC=fp32 STEPS=50 tools/ab.sh
#
# Runs tools/unet_probe.py once per value of $VAR (each run under its own
# time limit; stops at the first failure) and prints the probe's summary line.
# Knobs read by the library: ERTD_UNET_SIDE (skip-conv graph branch),
# ERTD_UNET_TPX / ERTD_UNET_WCO / ERTD_UNET_STAGE (fp32 conv tiling),
# ERTD_UNET_BF16_FUSEGN (fused bf16 GN prologue), ERTD_UNET_WINO (Winograd).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
VAR=${VAR:?set VAR to the environment variable to vary}
for v in ${VALUES:?set VALUES}; do
  env "$VAR=$v" timeout -k 10 300 python3 tools/unet_probe.py --config "${CFG:-U2}" --B "${B:-64}" \
    --precision "${PREC:-fp32}" --steps "${STEPS:-50}" > "gpurun_out/ab_${VAR}_${v//\//_}.log" 2>&1
  rc=$?
  echo "[$VAR=$v] rc=$rc $(tail -1 "gpurun_out/ab_${VAR}_${v//\//_}.log")"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
