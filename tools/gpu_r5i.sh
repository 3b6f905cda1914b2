set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
ERTD_LIB_PATH=$PWD/variants/epi0.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_unet.py -k "forward or chain" > gpurun_out/epi_tests.log 2>&1
rc=$?; tail -1 gpurun_out/epi_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do for v in head epi0 epi1 epi2; do
  echo -n "$v: "; ERTD_LIB_PATH=$PWD/variants/$v.so timeout -k 10 60 python3 tools/unet_probe.py --config U2 --B 64 --steps 20 2>&1 | tail -1
done; done
