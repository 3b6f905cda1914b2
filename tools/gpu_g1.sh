set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "--Cin 64 --Cout 64 --H 64" "--Cin 64 --Cout 64 --H 64 --res" "--Cin 128 --Cout 128 --H 32" "--Cin 384 --Cout 128 --H 32"; do
  n=$(echo $cfg | tr -d ' -')
  ERTD_LIB_PATH=ab/stamp.so timeout -k 10 120 python3 tools/wino4_stamps.py $cfg > gpurun_out/st_$n.log 2>&1
  rc=$?; echo "[stamps $cfg] rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/st_$n.log; exit $rc; }
done
ERTD_WINO4_W16=1 ERTD_LIB_PATH=ab/stamp.so timeout -k 10 120 python3 tools/wino4_stamps.py --Cin 256 --Cout 256 --H 16 > gpurun_out/st_w16.log 2>&1; echo "[w16] rc=$?"
bash tools/layer_trace.sh > gpurun_out/lt_U2_head.txt 2>&1; echo "[trace] rc=$?"
exit 0
