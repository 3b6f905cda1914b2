#!/bin/bash
# A/B of the fp32 conv schedule knobs on the U2 B=64 sampler step (diagnostic).
# Every GPU step has its own time limit; a fault/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/conv_ab.log; : > $out
for cfg in "1 0" "0 0" "1 1" "0 1"; do
  set -- $cfg
  echo "STAGE=$1 WCO=$2" >> $out
  ERTD_UNET_STAGE=$1 ERTD_UNET_WCO=$2 timeout -k 10 120 python tools/unet_probe.py --config ${CFG:-U2} --B ${B:-64} --steps 20 >> $out 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc" >> $out; exit $rc; }
done
cat $out
