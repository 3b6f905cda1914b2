#!/bin/bash
# SQ counters of one conv layer (tools/conv_probe.py) per --pmc pass (diagnostic).
#   PROBE_ARGS="--Cin 64 ..." KERNEL=conv_wino_kernel tools/wino_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
for pass in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
            "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT"; do
  d=gpurun_out/wpmc_$i; rm -rf "$d"
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$d" -o run \
    -- python3 tools/conv_probe.py --reps 3 ${PROBE_ARGS:-} > "$d.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "[pass $i] rc=$rc"; tail -3 "$d.log"; exit $rc; }
  f=$(find "$d" -name '*counter_collection.csv' | head -1)
  python3 - "$f" "${KERNEL:-conv_wino_kernel}" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(f"{k:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
PY
  i=$((i+1))
done
exit 0
