#!/bin/bash
# Round-end evidence (tools/gpu_final.sh) plus the U2 B=64 fp32 PMC traffic pass.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_final.sh || exit $?
CFG=U2 B=64 PREC=fp32 bash tools/unet_traffic.sh; echo "[u2 pmc] rc=$?"
exit 0
