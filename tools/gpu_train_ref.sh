#!/bin/bash
# Reference-model train step on the GPU box: the train tests, then the
# reference train-step timing (eager train_step and TrainPlan) and a
# rocprofv3 kernel table of the plan's steps.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_train.py tests/test_gpu_unet_train.py > gpurun_out/train_tests.log 2>&1
rc=$?; tail -4 gpurun_out/train_tests.log; echo "[train tests] rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/train_ref_probe.py > gpurun_out/train_ref_probe.log 2>&1
rc=$?; cat gpurun_out/train_ref_probe.log | tail -20; echo "[probe] rc=$rc"; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/trprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trprof -o run \
  -- python3 tools/train_ref_probe.py --steps 200 --plan-only > gpurun_out/trprof.log 2>&1
echo "[train prof] rc=$?"
exit 0
