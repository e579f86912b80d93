#!/bin/bash
# A/B of one environment switch on the cfg2 table launch, alternating order over 3 rounds:
#   tools/gpu_ab_var.sh VAR "v1 v2 ..." [lib.so] [grid]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
VAR=$1; VALS=$2; LIB=${3:-airiceraytracing_amd/libairice.so}; G=${4:--20000,300000,20,92,180,0.5}
for round in 1 2 3; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 120 python tools/ab_table.py --one $LIB --reps 300 --grid=$G 2>/dev/null | sed "s/^/$VAR=$v /" || exit 1
  done
done
