#!/bin/bash
# PMC traffic of the U5 bf16 and U2 fp32 steps at HEAD, then the train-step kernel profile
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
CFG=U5 B=64 PREC=bf16 STEPS=2 bash tools/unet_traffic.sh || exit $?
cp gpurun_out/kernel_traffic.json profiles/kernel_traffic.json
CFG=U2 B=64 PREC=fp32 STEPS=4 bash tools/unet_traffic.sh || exit $?
bash tools/gpu_train_prof.sh
