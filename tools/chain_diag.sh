set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for B in 8 16 64; do
timeout -k 10 60 ./tools/diag_chain $B 1000 8 > gpurun_out/diag_chain_b$B.log 2>&1; rc=$?; grep -v "^   *[0-9]*[ :]" gpurun_out/diag_chain_b$B.log | grep -v "^step:\|^member" | head -20; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider -x -k "faithful or golden or plan" > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; exit $rc
