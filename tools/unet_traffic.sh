#!/bin/bash
# HBM traffic of one U-Net sampler step from PMC counters (two separate passes,
# FETCH_SIZE and WRITE_SIZE; no trace domains), summed over every ertd::unet::
# dispatch of a short probe run:
#   CFG=U3 B=256 PREC=bf16 tools/unet_traffic.sh  -> gpurun_out/kernel_traffic.json
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
CFG=${CFG:-U3}; B=${B:-256}; PREC=${PREC:-bf16}; STEPS=${STEPS:-4}
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/upmc_$c
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/upmc_$c -o run \
    -- python3 tools/unet_probe.py --config $CFG --B $B --precision $PREC --steps $STEPS > gpurun_out/upmc_$c.log 2>&1
  rc=$?; echo "[pmc $c] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
# several passes in one call accumulate into one file
[ -f gpurun_out/kernel_traffic.json ] || cp -f profiles/kernel_traffic.json gpurun_out/kernel_traffic.json
# the probe runs 7 forwards and 2 x STEPS sampler steps; forward = one step's kernels
UNET_STEPS=$((7 + 2 * STEPS)) UNET_KEY=unet_${CFG}_B${B}_${PREC}_step \
  UNET_WORKLOAD="tools/unet_probe.py $CFG $PREC B=$B L=4693 (7 forwards + $((2 * STEPS)) sampler steps)" \
  python3 tools/pmc_summarize.py gpurun_out/upmc_FETCH_SIZE gpurun_out/upmc_WRITE_SIZE gpurun_out/kernel_traffic.json
