set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export ERTD_BENCH_DEBUG=1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-train --no-steps-schedule --no-hoisted --roofline-reps 1 2>&1 | grep -v amdgpu.ids | cut -c1-250
