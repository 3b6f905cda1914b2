#!/bin/bash
# Compare faithful-chain schedules under rocprofv3 kernel traces (diagnostic).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for sch in seq pipe; do
  ERTD_FAITHFUL_SCHEDULE=$sch timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sched_$sch -o run \
    -- python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-hoisted --no-train > gpurun_out/sched_$sch.log 2>&1
  rc=$?; echo "$sch rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/sched_$sch.log
  [ $rc -eq 0 ] || exit $rc
done
