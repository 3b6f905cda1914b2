#!/bin/bash
# Host-package A/B (diagnostic): the train tests, then tools/train_probe.py
# alternating this tree's ertdiff package and a copy under variants/oldpy
# (e.g. the package at an older commit: git show HEAD~1:... per file), both on
# this tree's library (ERTD_PKG_PATH / ERTD_LIB_PATH).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_unet_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tr_tests.log 2>&1
rc=$?; tail -2 gpurun_out/tr_tests.log; [ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export ERTD_PKG_PATH=$PWD/variants/oldpy ERTD_LIB_PATH=$PWD/ert-conditional-diffusion-model_amd/ertdiff/libertdiff_hip.so; else unset ERTD_PKG_PATH ERTD_LIB_PATH; fi
    timeout -k 10 200 python3 tools/train_probe.py --steps 100 > gpurun_out/ab_$v.log 2>&1
    rc=$?; echo "[$v] rc=$rc $(tail -1 gpurun_out/ab_$v.log)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
