#!/bin/bash
# A/B of the table kernel's rays-per-lane choice (AIRICE_TABLE_RPL=1|2) on one library:
# cfg2 and the reference default grid, alternating order; sha1 of the float tables must agree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for g in "-20000,300000,20,92,180,0.5" "-20000,300000,10,90.1,180,0.1"; do
  for r in 1 2 1 2 1 2; do
    AIRICE_TABLE_RPL=$r timeout -k 10 120 python tools/ab_table.py --one airiceraytracing_amd/libairice.so --reps 300 --grid=$g | sed "s/^/R=$r grid=$g /" || exit 1
  done
done
