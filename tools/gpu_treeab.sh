#!/bin/bash
# Same-box A/B of whole source trees and variant libraries on the U2 sampler
# step (diagnostic).  A tree is a git worktree of an older commit with its own
# libraries built in place (git worktree add variants/r4 <sha>; build.py and
# build.py --diag inside it): it runs its OWN tools/unet_probe.py and package,
# so C-ABI changes between the commits do not matter.  LIBS are variant
# libraries of HEAD (tools/build_variant.sh), loaded through ERTD_LIB_PATH.
#   TREES="variants/r4" LIBS="variants/r5.so" ROUNDS=3 LAYERS=1 tools/gpu_treeab.sh
# LAYERS=1 also writes the serialized per-layer table of HEAD and of each tree
# (gpurun_out/treeab_layers_<tag>.txt).  Every GPU step has its own time limit;
# the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; ROOT=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
probe() {   # $1 tag, $2 tree root; ERTD_LIB_PATH as set by the caller
  timeout -k 10 200 python3 "$2/tools/unet_probe.py" --config ${CFG:-U2} --B ${B:-64} --precision ${PREC:-fp32} \
    --steps ${STEPS:-100} > gpurun_out/treeab_$1.log 2>&1
  rc=$?; echo "[$1] rc=$rc $(tail -1 gpurun_out/treeab_$1.log)"; return $rc
}
layers() {  # $1 tag, $2 tree root (its diagnostic library: one chain, no side stream)
  d=$ROOT/gpurun_out/treeab_lt_$1; rm -rf "$d"
  (cd "$2" && ERTD_LIB_PATH=$PWD/ert-conditional-diffusion-model_amd/ertdiff/libertdiff_hip_diag.so ERTD_UNET_SIDE=0 \
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run \
    -- python3 tools/unet_probe.py --config ${CFG:-U2} --B ${B:-64} --precision ${PREC:-fp32} --steps 2) > "$d.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "[layers $1] rc=$rc"; tail -3 "$d.log"; return $rc; }
  f=$(find "$d" -name '*kernel_trace.csv' | head -1)
  python3 tools/unet_layers.py "$f" ${CFG:-U2} ${B:-64} > gpurun_out/treeab_layers_$1.txt
  echo "[layers $1] $(grep conv_wino4s_kernel gpurun_out/treeab_layers_$1.txt)"
}
if [ "${LAYERS:-0}" = 1 ]; then
  layers head "$ROOT" || exit $?
  for t in ${TREES:-}; do layers "$(basename $t)" "$ROOT/$t" || exit $?; done
fi
for k in $(seq ${ROUNDS:-2}); do
  unset ERTD_LIB_PATH; probe head "$ROOT" || exit $?
  for t in ${TREES:-}; do probe "$(basename $t)" "$ROOT/$t" || exit $?; done
  for l in ${LIBS:-}; do ERTD_LIB_PATH=$ROOT/$l probe "$(basename $l .so)" "$ROOT" || exit $?; done
done
exit 0
