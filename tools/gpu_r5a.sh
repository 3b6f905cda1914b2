#!/bin/bash
# round-5 check: reference train bench leg + U2 step timeline (production library)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python3 -u -c "
import sys, json, torch; sys.argv=['bench.py']
import bench
print(json.dumps(bench.train_bench(torch.device('cuda', 0))))" > gpurun_out/train_bench.log 2>&1
rc=$?; tail -2 gpurun_out/train_bench.log; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/u2tl
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/u2tl -o run \
  -- python3 tools/unet_probe.py --config U2 --B 64 --steps 4 > gpurun_out/u2tl.log 2>&1
rc=$?; tail -1 gpurun_out/u2tl.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 60 python3 tools/unet_probe.py --config U2 --B 64 --steps 20 2>&1 | tail -1
f=$(find gpurun_out/u2tl -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" --from-name conv_in_kernel --top 16
