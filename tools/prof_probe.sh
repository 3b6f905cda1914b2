#!/bin/bash
# rocprofv3 kernel stats of tools/launch_probe.py (diagnostic); prints a summary.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/probe
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/probe -o run \
  -- python3 tools/launch_probe.py > gpurun_out/probe.log 2>&1
rc=$?; grep -E "graph|eager" gpurun_out/probe.log
python3 - <<'PY'
import csv
r = list(csv.DictReader(open('gpurun_out/probe/run_kernel_stats.csv')))
for x in r[:8]:
    print(f"{x['Name'][:48]:48s} calls {x['Calls']:>6s} avg {float(x['AverageNs'])/1000:7.2f} us  min {float(x['MinNs'])/1000:7.2f}  {float(x['Percentage']):5.1f}%")
PY
exit $rc
