#!/bin/bash
# round-3 check: full GPU tests + smoke + bench, Upsample-conv A/B, wino4s library
# variants A/B (ERTD_LIB_PATH), serialized U2 layer trace
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_run.sh || exit $?
VAR=ERTD_WINO4S_UP VALUES="0 1" STEPS=30 bash tools/ab.sh || exit $?
if ls variants/*.so > /dev/null 2>&1; then
  VAR=ERTD_LIB_PATH VALUES="$(ls $PWD/variants/*.so | tr '\n' ' ')" STEPS=30 bash tools/ab.sh || exit $?
fi
bash tools/layer_trace.sh > gpurun_out/lt_U2.txt 2>&1; echo "[trace] rc=$?"
