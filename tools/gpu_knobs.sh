#!/bin/bash
# Knob sweep (diagnostic): tools/train_probe.py (or PROBE="tools/unet_probe.py
# --config U2 --B 64 --steps 50", the sampler step) on the diag library with one
# ERTD_<knob>=<value> per run; KNOBS="NAME=V NAME=V ..." (base first).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
export ERTD_LIB_PATH=$PWD/ert-conditional-diffusion-model_amd/ertdiff/libertdiff_hip_diag.so
for kv in base ${KNOBS}; do
  if [ $kv = base ]; then env_kv=""; else env_kv="ERTD_$kv"; fi
  env $env_kv timeout -k 10 200 python3 ${PROBE:-tools/train_probe.py --steps 100} > gpurun_out/knob.log 2>&1
  rc=$?; echo "[$kv] rc=$rc $(tail -1 gpurun_out/knob.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
