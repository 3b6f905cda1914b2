set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_unet_ops.py tests/test_gpu_unet.py ${TESTSEL:-} > gpurun_out/t_ops.log 2>&1; rc=$?; tail -2 gpurun_out/t_ops.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/t_ops.log | head -20; exit $rc; }
VAR=ERTD_UNET_WINO VALUES="1" CFG=U2 B=64 STEPS=50 bash tools/ab.sh || exit 1
VAR=ERTD_UNET_WINO VALUES="1" CFG=U3 B=256 PREC=bf16 STEPS=20 bash tools/ab.sh || exit 1
CFG=U2 B=64 bash tools/layer_trace.sh > gpurun_out/lt_U2.txt 2>&1; grep "conv_out\|conv_in\|total" gpurun_out/lt_U2.txt
