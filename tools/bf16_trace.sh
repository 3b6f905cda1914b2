#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for p in 1 0; do
  rm -rf gpurun_out/bft_$p
  ERTD_UNET_BF16_PRE=$p timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bft_$p -o run \
    -- python3 tools/unet_probe.py --config U3 --B 256 --steps 2 --precision bf16 > gpurun_out/bft_$p.log 2>&1
  rc=$?; echo "[p=$p] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
