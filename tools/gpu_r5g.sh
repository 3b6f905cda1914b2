set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_unet.py > gpurun_out/unet_tests.log 2>&1
rc=$?; tail -1 gpurun_out/unet_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do echo -n "prod: "; timeout -k 10 60 python3 tools/unet_probe.py --config U2 --B 64 --steps 20 2>&1 | tail -1; done
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/upmc_$c
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/upmc_$c -o run \
    -- python3 tools/unet_probe.py --config U2 --B 64 --steps 2 > gpurun_out/upmc_$c.log 2>&1 || exit 1
done
cp -f profiles/kernel_traffic.json gpurun_out/kernel_traffic.json
python3 tools/unet_layer_traffic.py gpurun_out/upmc_FETCH_SIZE gpurun_out/upmc_WRITE_SIZE U2 64 --json gpurun_out/kernel_traffic.json > gpurun_out/r05_u2_layer_traffic.txt 2>&1
grep "convs:\|step total\|top excess" gpurun_out/r05_u2_layer_traffic.txt
