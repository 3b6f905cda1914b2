# split-bf16 + U5 chain checks (GPU box): op tests, U-Net tests, then a short bench of the bf16 legs
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_unet_ops.py tests/test_gpu_unet.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/split_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -15 gpurun_out/split_tests.log; [ $rc -ne 0 ] && exit $rc
cp gpurun_out/parity_errors.jsonl gpurun_out/parity_split.jsonl 2>/dev/null
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-ensemble --no-hbm-kernels --no-unet-train --no-kde --no-reference --no-conv-kernels > gpurun_out/split_bench.json 2> gpurun_out/split_bench.err
rc=$?; echo "[bench] rc=$rc"; exit $rc
