#!/bin/bash
# HBM traffic of the hot kernels from PMC counters, two separate
# passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass), no trace domains.
# Writes gpurun_out/kernel_traffic.json; copy it to profiles/ (read by bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out profiles; export TMPDIR=/tmp
ARGS="--steps 20 --warmup 5 --ref-steps 1000 --ref-warmup 0 --no-cpu-baseline --no-hoisted --no-train --no-steps-schedule --roofline-reps 20 --no-u3 --no-u5 --no-kde --no-ensemble --no-evaluation --no-unet-train --no-hbm-kernels --no-conv-kernels ${BENCH_ARGS:-}"
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_$c
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$c -o run \
    -- python3 bench.py $ARGS > gpurun_out/pmc_$c.log 2>&1
  rc=$?; echo "[pmc $c] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
[ -f gpurun_out/kernel_traffic.json ] || cp -f profiles/kernel_traffic.json gpurun_out/kernel_traffic.json; UNET_STEPS=25 python3 tools/pmc_summarize.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/kernel_traffic.json
