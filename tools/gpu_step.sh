set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_unet_ops.py tests/test_gpu_unet.py ${TESTSEL:-} > gpurun_out/t_ops.log 2>&1; rc=$?; tail -2 gpurun_out/t_ops.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/t_ops.log | head -20; exit $rc; }
VAR=ERTD_UNET_WINO VALUES="1" CFG=U3 B=256 PREC=bf16 STEPS=20 bash tools/ab.sh || exit 1
VAR=ERTD_UNET_WINO VALUES="1" CFG=U5 B=64 PREC=bf16 STEPS=10 bash tools/ab.sh || exit 1
DBGVAR=ERTD_BF16_DBG VALUES="0 1" PROBE_ARGS="--B 256 --precision bf16" bash tools/wino_dbg.sh
