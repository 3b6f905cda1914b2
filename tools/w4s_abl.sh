#!/bin/bash
# conv_wino4s_kernel chunk-cost breakdown (diagnostic): the ablation builds
# variants/*.so (e.g. tools/build_variant.sh unet_conv_wino4s -DWINO4S_ABL=<n> variants/abl<n>.so)
# of one layer under rocprofv3 --kernel-trace, per layer shape; prints the conv
# kernel's average per variant ("base" = the shipped library).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for shape in ${SHAPES:-"64 64 64" "256 256 16" "512 256 16" "128 128 32"}; do
  set -- $shape
  for lib in base $(ls variants/*.so 2>/dev/null); do
    tag=$(basename $lib .so); d=gpurun_out/abl_${tag}_$1_$2_$3; rm -rf "$d"
    if [ "$lib" = base ]; then unset ERTD_LIB_PATH; else export ERTD_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run \
      -- python3 tools/conv_probe.py --Cin $1 --Cout $2 --H $3 --B 64 --reps 10 > "$d.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "[$tag $shape] rc=$rc"; tail -3 "$d.log"; exit $rc; }
    f=$(find "$d" -name '*kernel_trace.csv' | head -1)
    python3 - "$f" "$tag" "$shape" <<'PY'
import csv, sys
r = [int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in csv.DictReader(open(sys.argv[1]))
     if "conv_wino" in x["Kernel_Name"]]
r = r[3:] if len(r) > 3 else r
print(f"[{sys.argv[3]}] {sys.argv[2]:6s} conv_wino4s {sum(r) / len(r) / 1000:7.1f} us avg over {len(r)}")
PY
  done
done
unset ERTD_LIB_PATH
exit 0
