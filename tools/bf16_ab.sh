#!/bin/bash
# bf16 conv tile A/B on U3 B=256 (diagnostic); each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
out=gpurun_out/bf16_ab.log; : > $out
for t in 0 1; do
  echo "BF16_TPX=$t" >> $out
  ERTD_UNET_BF16_TPX=$t timeout -k 10 150 python tools/unet_probe.py --config U3 --B 256 --steps 10 --precision bf16 >> $out 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc" >> $out; exit $rc; }
done
cat $out
