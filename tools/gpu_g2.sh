#!/bin/bash
# round-3 diagnostics: F(4x4) stamps, per-layer trace, A/B of library variants
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "--Cin 64 --Cout 64 --H 64" "--Cin 384 --Cout 128 --H 32"; do
  n=$(echo $cfg | tr -d ' -')
  ERTD_LIB_PATH=ab/stamp.so timeout -k 10 120 python3 tools/wino4_stamps.py $cfg > gpurun_out/st_$n.log 2>&1
  rc=$?; echo "[stamps $cfg] rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/st_$n.log; exit $rc; }
done
for v in ert-conditional-diffusion-model_amd/ertdiff/libertdiff_hip.so ab/dmai0.so; do
  ERTD_LIB_PATH=$v timeout -k 10 200 python3 tools/unet_probe.py --config U2 --B 64 --steps 30 > gpurun_out/probe.log 2>&1
  rc=$?; echo "[probe $v] rc=$rc $(tail -1 gpurun_out/probe.log)"; [ $rc -ne 0 ] && exit $rc
done
bash tools/layer_trace.sh > gpurun_out/lt_U2_new.txt 2>&1; echo "[trace] rc=$?"
exit 0
