set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_unet.py ${TESTSEL:-} > gpurun_out/t_ops.log 2>&1; rc=$?; tail -2 gpurun_out/t_ops.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/t_ops.log | head -20; exit $rc; }
VAR=ERTD_UNET_WINO VALUES="1" CFG=U2 B=64 STEPS=50 bash tools/ab.sh || exit 1
CFG=U2 B=64 bash tools/layer_trace.sh > gpurun_out/lt_U2.txt 2>&1
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/lt_U2/run_kernel_trace.csv')))
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows if 'dense_kernel' in r['Kernel_Name']]
print('dense', d[-6:])
PY
