#!/bin/bash
# bf16 stride-1 staging A/B: pre-transformed image (1) vs register staging (0), U3 B=256.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
out=gpurun_out/bf16_pre_ab.log; : > $out
for p in 1 0; do
  echo "BF16_PRE=$p" >> $out
  ERTD_UNET_BF16_PRE=$p timeout -k 10 150 python tools/unet_probe.py --config U3 --B 256 --steps 10 --precision bf16 >> $out 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc" >> $out; cat $out; exit $rc; }
done
cat $out
