#!/bin/bash
# SQ counters of the U-Net convs (diagnostic): one --pmc pass, short probe run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/upmc
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
  --output-format csv -d gpurun_out/upmc -o run -- python3 tools/unet_probe.py --config ${CFG:-U2} --B 64 --steps 1 > gpurun_out/upmc.log 2>&1
echo "[pmc] rc=$?"
