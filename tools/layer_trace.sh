#!/bin/bash
# Serialized per-layer trace of one U-Net sampler config (diagnostic):
#   CFG=U2 B=64 PREC=fp32 tools/layer_trace.sh  -> gpurun_out/lt_<CFG>/, layer table on stdout
# ERTD_UNET_SIDE=0 (read by the diagnostic build, build.py --diag): one chain,
# so per-kernel durations are not inflated by overlap.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
d=gpurun_out/lt_${CFG:-U2}
rm -rf "$d"
ERTD_LIB_PATH=$PWD/ert-conditional-diffusion-model_amd/ertdiff/libertdiff_hip_diag.so ERTD_UNET_SIDE=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run \
  -- python3 tools/unet_probe.py --config "${CFG:-U2}" --B "${B:-64}" --precision "${PREC:-fp32}" --steps 2 > "$d.log" 2>&1
rc=$?; echo "[trace] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$d.log"; exit $rc; }
f=$(find "$d" -name '*kernel_trace.csv' | head -1)
python3 tools/unet_layers.py "$f" "${CFG:-U2}" "${B:-64}"
