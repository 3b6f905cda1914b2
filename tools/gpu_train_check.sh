# U-Net op / model / train tests, then the per-kernel profile of UNetTrainPlan
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests/test_gpu_unet_ops.py tests/test_gpu_unet.py tests/test_gpu_unet_train.py} \
  -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/train_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -4 gpurun_out/train_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_train_prof.sh
