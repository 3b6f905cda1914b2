#!/bin/bash
# round-5 profiles: U2 B=64 per-layer PMC traffic (two passes), serialized layer
# tables for U2 B=64 / B=128 (configs[3] rank shape) and U5 B=64 bf16
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/upmc_$c
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/upmc_$c -o run \
    -- python3 tools/unet_probe.py --config U2 --B 64 --steps 2 > gpurun_out/upmc_$c.log 2>&1
  rc=$?; echo "[pmc $c] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cp -f profiles/kernel_traffic.json gpurun_out/kernel_traffic.json
python3 tools/unet_layer_traffic.py gpurun_out/upmc_FETCH_SIZE gpurun_out/upmc_WRITE_SIZE U2 64 \
  --json gpurun_out/kernel_traffic.json > gpurun_out/r05_u2_layer_traffic.txt 2>&1
echo "[traffic] rc=$?"; tail -12 gpurun_out/r05_u2_layer_traffic.txt
CFG=U2 B=64 bash tools/layer_trace.sh > gpurun_out/r05_unet_layers.txt 2>&1; echo "[lt U2 64] rc=$?"; tail -6 gpurun_out/r05_unet_layers.txt
CFG=U2 B=128 bash tools/layer_trace.sh > gpurun_out/r05_unet_layers_B128.txt 2>&1; echo "[lt U2 128] rc=$?"; tail -6 gpurun_out/r05_unet_layers_B128.txt
CFG=U5 B=64 PREC=bf16 bash tools/layer_trace.sh > gpurun_out/r05_unet_layers_U5_B64.txt 2>&1; echo "[lt U5 64] rc=$?"; tail -4 gpurun_out/r05_unet_layers_U5_B64.txt
exit 0
