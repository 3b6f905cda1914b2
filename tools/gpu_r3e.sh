#!/bin/bash
# With the xi-split default: 16x16 F(4x4) selection A/B (ERTD_WINO4S 4 = only
# where items fill the CUs, 2 = every 16x16 conv) on the U2 B=64 sampler and
# the U2 B=32 train step, then a U3 bf16 B=256 serialized layer trace.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
VAR=ERTD_WINO4S VALUES="4 2 4 2" STEPS=30 bash tools/ab.sh || exit $?
for v in 4 2 4 2; do
  ERTD_WINO4S=$v timeout -k 10 300 python3 tools/train_probe.py --config U2 --B 32 --steps 30 > gpurun_out/tr_w4s_$v.log 2>&1
  rc=$?; echo "[train WINO4S=$v] rc=$rc $(tail -1 gpurun_out/tr_w4s_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
CFG=U3 B=256 PREC=bf16 bash tools/layer_trace.sh > gpurun_out/lt_u3.txt 2>&1; echo "[u3 trace] rc=$?"
exit 0
