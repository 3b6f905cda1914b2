set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rf -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -30 gpurun_out/gpu_tests.log; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
bash tools/prof_probe.sh
