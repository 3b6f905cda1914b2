#!/bin/bash
# Full GPU check + per-layer trace (diagnostic): gpu_run.sh (pytest -m gpu, smoke, bench),
# then the serialized U2 layer table into gpurun_out/lt_U2.txt
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash tools/gpu_run.sh || exit $?
bash tools/layer_trace.sh > gpurun_out/lt_U2.txt 2>&1; echo "[trace] rc=$?"
