#!/bin/bash
# GPU-box check (diagnostic): the -m gpu tests, smoke(), then a short bench.
#   STEPS=... BENCH_ARGS="..." TESTS="tests/..." tools/gpu_run.sh
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
rm -f gpurun_out/parity_errors.jsonl
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
    ${TESTS:-tests} > gpurun_out/gpu_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/gpu_tests.log; echo "[tests] rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -2 gpurun_out/smoke.log; echo "[smoke] rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; echo "[bench] rc=$rc"; grep '^{' gpurun_out/bench.log | cut -c1-600; [ $rc -ne 0 ] && tail -20 gpurun_out/bench.log
  exit $rc
fi
exit 0
