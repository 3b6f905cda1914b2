#!/bin/bash
# Same-box A/B of variant libraries (variants/<name>.so) on the U-Net step:
# per variant, the rocprofv3 kernel averages of the kernels matching KPAT
# (a Python regex) over a U2 B=64 probe run, and the probe's step time.
#   LIBS="co1 co2" KPAT="conv_out" tools/gpu_kab.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for n in ${LIBS:?}; do
  d=gpurun_out/kab_$n; rm -rf $d
  ERTD_LIB_PATH=$PWD/variants/$n.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
    -- python3 tools/unet_probe.py --config ${CFG:-U2} --B ${B:-64} --steps 4 > $d.log 2>&1 || { echo "[$n] failed"; tail -3 $d.log; exit 1; }
  python3 - $d/run_kernel_stats.csv $n "${KPAT:?}" <<'PY'
import csv, re, sys
out = []
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], r["Name"]):
        nm = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1][:40]
        out.append(f"{nm} {float(r['AverageNs'])/1e3:7.2f} us x{r['Calls']}")
print(f"{sys.argv[2]:8s}", " | ".join(out))
PY
done
done
for n in ${LIBS}; do echo -n "$n: "; ERTD_LIB_PATH=$PWD/variants/$n.so timeout -k 10 60 python3 tools/unet_probe.py --config ${CFG:-U2} --B ${B:-64} --steps 20 2>&1 | tail -1; done
