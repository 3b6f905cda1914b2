#!/bin/bash
# Winograd conv chunk-time breakdown (diagnostic): ERTD_WINO_DBG variants of one
# 64->64 64x64 B=64 GN+SiLU layer under rocprofv3 --kernel-trace; prints the
# conv_wino_kernel average per variant.  The variants exist only in the
# diagnostic build (build.py --diag), which this script loads.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VALUES:-0 1 2 4 8 6 7}; do
  d=gpurun_out/wdbg_$v; rm -rf "$d"
  env ERTD_LIB_PATH=$PWD/ert-conditional-diffusion-model_amd/ertdiff/libertdiff_hip_diag.so "${DBGVAR:-ERTD_WINO_DBG}=$v" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run \
    -- python3 tools/conv_probe.py ${PROBE_ARGS:-} > "$d.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "[dbg=$v] rc=$rc"; tail -3 "$d.log"; exit $rc; }
  f=$(find "$d" -name '*kernel_trace.csv' | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
r = [int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in csv.DictReader(open(sys.argv[1]))
     if "conv_wino" in x["Kernel_Name"] or "conv_kernel<" in x["Kernel_Name"] or "conv_bf16_kernel<" in x["Kernel_Name"]]
r = r[3:] if len(r) > 3 else r
print(f"[dbg={sys.argv[2]}] conv kernel {sum(r) / len(r) / 1000:.1f} us avg over {len(r)}")
PY
done
exit 0
