set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for a in 0 1 2 4 8 15; do timeout -k 10 60 ./tools/diag_enc_$a > gpurun_out/diag_enc_$a.log 2>&1 || exit 3; done
cat gpurun_out/diag_enc_*.log
bash tools/gpu_check.sh || exit $?
bash tools/pmc_traffic.sh
