#!/bin/bash
# Same-box A/B of variant libraries (diagnostic; build them on the CPU side with
# tools/build_variant.sh ... variants/<name>.so):
#   LIBS="variants/a.so variants/b.so" SHAPES="64 64 64;256 256 16" tools/gpu_ab.sh
# 1) per shape, the conv_wino4s kernel average under rocprofv3 --kernel-trace for
#    the shipped library ("base") and each variant (tools/w4s_abl.sh's loop);
# 2) the U2 B=64 sampler step (tools/unet_probe.py) alternating base / variants
#    ROUNDS times.  Every GPU step has its own time limit; stops at a failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
LIBS=${LIBS:-$(ls variants/*.so 2>/dev/null)}
IFS=';' read -ra SH <<< "${SHAPES:-64 64 64;128 128 32;256 256 16;512 256 16}"
if [ "${SKIP_LAYERS:-0}" != 1 ]; then
for shape in "${SH[@]}"; do
  set -- $shape
  for lib in base $LIBS; do
    tag=$(basename $lib .so); d=gpurun_out/ab_${tag}_$1_$2_$3; rm -rf "$d"
    if [ "$lib" = base ]; then unset ERTD_LIB_PATH; else export ERTD_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run \
      -- python3 tools/conv_probe.py --Cin $1 --Cout $2 --H $3 --B ${B:-64} --reps 10 > "$d.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "[$tag $shape] rc=$rc"; tail -3 "$d.log"; exit $rc; }
    f=$(find "$d" -name '*kernel_trace.csv' | head -1)
    python3 - "$f" "$tag" "$shape" <<'PY'
import csv, sys
r = [int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in csv.DictReader(open(sys.argv[1]))
     if "conv_wino" in x["Kernel_Name"]]
r = r[3:] if len(r) > 3 else r
print(f"[{sys.argv[3]}] {sys.argv[2]:10s} conv {sum(r) / len(r) / 1000:7.1f} us avg over {len(r)}")
PY
  done
done
fi
unset ERTD_LIB_PATH
for k in $(seq ${ROUNDS:-2}); do
  for lib in base $LIBS; do
    tag=$(basename $lib .so)
    if [ "$lib" = base ]; then unset ERTD_LIB_PATH; else export ERTD_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 200 python3 tools/unet_probe.py --config ${CFG:-U2} --B ${B:-64} --precision ${PREC:-fp32} \
      --steps ${STEPS:-50} > gpurun_out/abp_$tag.log 2>&1
    rc=$?; echo "[$tag] rc=$rc $(tail -1 gpurun_out/abp_$tag.log)"; [ $rc -ne 0 ] && exit $rc
  done
done
unset ERTD_LIB_PATH
exit 0
