set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
LIBS="r8p2 r8p3 r4p3 r16p2 r8p1" KPAT="conv_out64" bash tools/gpu_kab.sh 2>&1 | grep -v "U2 fp32"
cp variants/r8p2.so variants/cbwa6.so
LIBS="cbwa6 cbwa4 cbwa8 cbwa10" bash tools/gpu_libab.sh
