set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_unet.py tests/test_gpu_unet_ops.py tests/test_gpu_unet_train.py > gpurun_out/unet_tests.log 2>&1
rc=$?; tail -1 gpurun_out/unet_tests.log; [ $rc -ne 0 ] && { grep -m5 "Error\|assert\|FAILED" gpurun_out/unet_tests.log; exit $rc; }
for rep in 1 2 3; do echo -n "prod: "; timeout -k 10 60 python3 tools/unet_probe.py --config U2 --B 64 --steps 40 2>&1 | tail -1; done
rm -rf gpurun_out/dk
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dk -o run -- python3 tools/unet_probe.py --config U2 --B 64 --steps 8 > gpurun_out/dk.log 2>&1 || exit 1
python3 - gpurun_out/dk/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "dense_kernel" in r["Name"]: print(r["Name"].split("(")[0][-30:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
