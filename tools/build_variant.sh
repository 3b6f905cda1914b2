#!/bin/bash
# Build an alternative libertdiff_hip.so with one source recompiled under extra
# flags (same-box kernel A/B through ERTD_LIB_PATH; run on the CPU side):
#   tools/build_variant.sh unet_conv_wino4 "-DWINO4_PD=4" ab/pd4.so
set -eu
cd "$(dirname "$0")/.."
src=$1; flags=$2; out=$3
python3 ert-conditional-diffusion-model_amd/build.py > /dev/null
B=ert-conditional-diffusion-model_amd/build; mkdir -p "$(dirname "$out")" ab/obj
objs=$(ls $B/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $flags \
  -I include -I ert-conditional-diffusion-model_amd/csrc -c ert-conditional-diffusion-model_amd/csrc/$src.hip \
  -o ab/obj/$src.$$.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs ab/obj/$src.$$.o -o "$out"
rm -f ab/obj/$src.$$.o
echo "$out"
