set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_unet.py > gpurun_out/unet_tests.log 2>&1
rc=$?; tail -1 gpurun_out/unet_tests.log; [ $rc -ne 0 ] && exit $rc
D=$PWD/ert-conditional-diffusion-model_amd/ertdiff/libertdiff_hip_diag.so
for rep in 1 2 3; do for k in 0 1; do
  echo -n "side_emb=$k: "; ERTD_UNET_SIDE_EMB=$k ERTD_LIB_PATH=$D timeout -k 10 60 python3 tools/unet_probe.py --config U2 --B 64 --steps 40 2>&1 | tail -1
done; done
