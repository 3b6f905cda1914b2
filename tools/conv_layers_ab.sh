#!/bin/bash
# Kernel traces of the U2 B=64 probe for WCO automatic / forced 1 (diagnostic).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for w in 0 1; do
  rm -rf gpurun_out/lay_w$w
  ERTD_UNET_WCO=$w timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lay_w$w -o run \
    -- python3 tools/unet_probe.py --config U2 --B 64 --steps 2 > gpurun_out/lay_w$w.log 2>&1
  rc=$?; echo "[w=$w] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
