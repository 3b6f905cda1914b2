# per-kernel breakdown of the U-Net train step (UNetTrainPlan, U2 B=32)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/tp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tp -o run \
  -- python3 tools/train_probe.py --steps 10 > gpurun_out/tp.log 2>&1
rc=$?; echo "[train prof] rc=$rc"; tail -2 gpurun_out/tp.log; exit $rc
