#!/bin/bash
# U-Net train-step time vs the wgrad range partition (diagnostic):
#   tools/wgrad_sweep.sh  -> one line per (workgroups per CU, min chunks per range)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for cfg in "2 8" "4 4" "4 8" "3 4" "8 2"; do
  set -- $cfg
  echo -n "wpc=$1 cps=$2: "
  ERTD_WGRAD_WPC=$1 ERTD_WGRAD_CPS=$2 timeout -k 10 120 python -u tools/train_prof.py U2 32 5 2>/dev/null | tail -1 || exit 1
done
