#!/bin/bash
# rocprofv3 kernel trace of one U3 B=256 bf16 probe run (diagnostic; per-layer table locally).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/bfl
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bfl -o run \
  -- python3 tools/unet_probe.py --config U3 --B 256 --steps 2 --precision bf16 > gpurun_out/bfl.log 2>&1
rc=$?; tail -4 gpurun_out/bfl.log; exit $rc
