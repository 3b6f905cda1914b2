#!/bin/bash
# per-layer conv times of U2 B=64 fp32: default tiles vs overrides (diagnostic)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "ERTD_NONE=0" "ERTD_UNET_WCO=1" "ERTD_UNET_STAGE=0"; do
  tag=${v//=/_}
  rm -rf gpurun_out/ab_$tag
  env $v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_$tag -o run \
    -- python3 tools/unet_probe.py --config U2 --B 64 --steps 2 > gpurun_out/ab_$tag.log 2>&1
  rc=$?; echo "[$v] rc=$rc"; grep steps/s gpurun_out/ab_$tag.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
