#!/bin/bash
# xi-split wino4s tuning (variant libraries in variants/: producer priority,
# V read-ahead): U2 B=64 probe per library, twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$(pwd)
for pass in 1 2; do
  for v in base pprio0 pprio3 pd3 pd4; do
    if [ $v = base ]; then L=""; else L=$R/variants/$v.so; fi
    ERTD_LIB_PATH=$L timeout -k 10 300 python3 tools/unet_probe.py --config U2 --B 64 --precision fp32 --steps 30 \
      > gpurun_out/w4t_$v.log 2>&1
    rc=$?; echo "[$v] rc=$rc $(tail -1 gpurun_out/w4t_$v.log)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
