#!/bin/bash
# GN backward channel parallelism: train/op GPU tests, U2 B=32 train probe,
# then the train-step kernel trace (tools/gpu_train_prof.sh).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_unet_train.py -x -q --timeout 300 \
  --timeout-method thread -m gpu > gpurun_out/gnb_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/gnb_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 tools/train_probe.py --config U2 --B 32 --steps 30 > gpurun_out/gnb_$i.log 2>&1
  rc=$?; echo "[train $i] rc=$rc $(tail -1 gpurun_out/gnb_$i.log)"; [ $rc -ne 0 ] && exit $rc
done
bash tools/gpu_train_prof.sh
