#!/bin/bash
# Round-end evidence at HEAD: pytest -m gpu, smoke, bench (default args), the
# serialized U2 per-layer trace, rocprofv3 --kernel-trace --stats of a short bench
# (U2 headline only), the U-Net and reference train-step kernel profiles, and with PMC=1 the U2 B=64
# fp32 PMC traffic pass.  SKIP_TESTS=1 / SKIP_BENCH=1 as in gpu_run.sh.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_run.sh || exit $?
bash tools/layer_trace.sh > gpurun_out/lt_U2.txt 2>&1; echo "[trace] rc=$?"
rm -rf gpurun_out/bprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bprof -o run \
  -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-u3 --no-u5 --no-ensemble --no-hbm-kernels \
  --no-kde --no-reference --no-unet-train --no-evaluation > gpurun_out/bprof.log 2>&1
echo "[bench prof] rc=$?"
bash tools/gpu_train_prof.sh
rm -rf gpurun_out/trprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trprof -o run \
  -- python3 tools/train_ref_probe.py --steps 200 --plan-only > gpurun_out/trprof.log 2>&1
echo "[ref train prof] rc=$?"; tail -2 gpurun_out/trprof.log
[ "${PMC:-0}" = 1 ] && { CFG=U2 B=64 PREC=fp32 bash tools/unet_traffic.sh; echo "[u2 pmc] rc=$?"; }
exit 0
