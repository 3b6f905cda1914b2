#!/bin/bash
# HBM traffic of the reference train step's kernels (TrainPlan, B=32, L=4693)
# from two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE); per-kernel
# medians and the step sum into gpurun_out/kernel_traffic.json (copy to profiles/).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/tpmc_$c
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/tpmc_$c -o run \
    -- python3 tools/train_ref_probe.py --steps 40 --plan-only > gpurun_out/tpmc_$c.log 2>&1
  rc=$?; echo "[pmc $c] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
[ -f gpurun_out/kernel_traffic.json ] || cp -f profiles/kernel_traffic.json gpurun_out/kernel_traffic.json
TRAIN=1 python3 tools/pmc_summarize.py gpurun_out/tpmc_FETCH_SIZE gpurun_out/tpmc_WRITE_SIZE gpurun_out/kernel_traffic.json
