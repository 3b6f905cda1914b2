#!/bin/bash
# Winograd wgrad K-range split target (ERTD_WGW_TASKS) on the U2 B=32 train step.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 2048 1024 4096 2048 1024 4096; do
  ERTD_WGW_TASKS=$v timeout -k 10 300 python3 tools/train_probe.py --config U2 --B 32 --steps 30 > gpurun_out/wgwt_$v.log 2>&1
  rc=$?; echo "[WGW_TASKS=$v] rc=$rc $(tail -1 gpurun_out/wgwt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
