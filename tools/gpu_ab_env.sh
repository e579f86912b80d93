#!/bin/bash
# A/B of table-kernel library variants x AIRICE_TABLE_RPL values on one grid, alternating order.
#   tools/gpu_ab_env.sh "<grid>" "<rpl values>" lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
G=$1; RPLS=$2; shift 2
for round in 1 2 3; do
  for lib in "$@"; do
    for r in $RPLS; do
      AIRICE_TABLE_RPL=$r timeout -k 10 120 python tools/ab_table.py --one $lib --reps 300 --grid=$G 2>/dev/null | sed "s/^/R=$r /" || exit 1
    done
  done
done
