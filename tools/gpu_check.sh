#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench, rocprof kernel trace of the
# same bench command, PMC traffic passes.  Every GPU step has its own time
# limit; a fault/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
stop_if_fatal() {  # pytest returns 1 on failed tests: keep going; anything else: stop
  local rc=$1 what=$2
  echo "[$what] rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal rc in $what; stopping"; exit "$rc"; fi
}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > gpurun_out/gpu_tests.log 2>&1
  rc=$?; tail -40 gpurun_out/gpu_tests.log; stop_if_fatal $rc pytest
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -5 gpurun_out/smoke.log; stop_if_fatal $rc smoke
fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; tail -5 gpurun_out/bench.log; stop_if_fatal $rc bench
if [ "${PROFILE:-1}" = "1" ]; then
  export TMPDIR=/tmp
  rm -rf gpurun_out/prof
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
    -- python3 bench.py ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
  rc=$?; tail -3 gpurun_out/prof.log; stop_if_fatal $rc rocprof
fi
if [ "${PMC:-1}" = "1" ]; then
  bash tools/pmc_traffic.sh; stop_if_fatal $? pmc
fi
