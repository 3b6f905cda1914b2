# round-3 check: U-Net op/model/train tests, U2 probe A/B of the 1x1 wave tile, per-layer trace,
# bench (U2 headline + conv kernels + train plan)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_unet_ops.py tests/test_gpu_unet.py tests/test_gpu_unet_train.py \
  -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r3b_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -8 gpurun_out/r3b_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 1 2; do
  ERTD_UNET_TPX1=$v timeout -k 10 200 python3 tools/unet_probe.py --config U2 --B 64 --precision fp32 --steps 30 > gpurun_out/probe_tpx1_$v.log 2>&1
  rc=$?; echo "[TPX1=$v] rc=$rc $(tail -1 gpurun_out/probe_tpx1_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
bash tools/layer_trace.sh > gpurun_out/lt_U2_r3b.txt 2>&1; echo "[trace] rc=$?"
timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-u3 --no-u5 --no-ensemble --no-hbm-kernels --no-kde --no-reference > gpurun_out/r3b_bench.json 2> gpurun_out/r3b_bench.err
rc=$?; echo "[bench] rc=$rc"; exit $rc
