set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
D=$PWD/ert-conditional-diffusion-model_amd/ertdiff/libertdiff_hip_diag.so
for cfg in "U2 2"; do set -- $cfg
ERTD_LIB_PATH=$D ERTD_UNET_GNFOLD=0 timeout -k 10 120 python3 tools/fold_dbg.py --config $1 --B $2 --tag off || exit 1
for k in 1 2; do
ERTD_LIB_PATH=$D ERTD_UNET_GNFOLD=$k timeout -k 10 120 python3 tools/fold_dbg.py --config $1 --B $2 --tag on$k || exit 1
python3 tools/fold_dbg.py --compare off on$k
done
done
