#!/bin/bash
# Build an alternative libertdiff_hip.so with one source (or a comma-separated
# list) recompiled under extra flags (same-box kernel A/B through ERTD_LIB_PATH;
# run on the CPU side):
#   tools/build_variant.sh unet_conv_wino4 "-DWINO4_PD=4" ab/pd4.so
#   tools/build_variant.sh chain,capi "-DCHAIN_SPI=1 -DERTD_CHAIN_RING=8" variants/spi1.so
set -eu
cd "$(dirname "$0")/.."
src=$1; flags=$2; out=$3
# DIAG=1: start from the diagnostic build (build.py --diag: reads the ERTD_* knobs)
if [ "${DIAG:-0}" = 1 ]; then
  python3 ert-conditional-diffusion-model_amd/build.py --diag > /dev/null
  B=ert-conditional-diffusion-model_amd/build/diag; flags="$flags -DERTD_DIAG"
else
  python3 ert-conditional-diffusion-model_amd/build.py > /dev/null
  B=ert-conditional-diffusion-model_amd/build
fi
mkdir -p "$(dirname "$out")" ab/obj
IFS=',' read -ra SRCS <<< "$src"
objs=$(ls $B/*.o); new=""
for s in "${SRCS[@]}"; do
  objs=$(echo "$objs" | grep -v "/$s\.o$")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $flags \
    -I include -I ert-conditional-diffusion-model_amd/csrc -c ert-conditional-diffusion-model_amd/csrc/$s.hip \
    -o ab/obj/$s.$$.o
  new="$new ab/obj/$s.$$.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $new -o "$out"
rm -f $new
echo "$out"
