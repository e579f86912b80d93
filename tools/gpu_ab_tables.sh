#!/bin/bash
# A/B of table-kernel library builds on the cfg2 grid, alternating order over 3 rounds (tools/ab_table.py).
#   tools/gpu_ab_tables.sh lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for round in 1 2 3; do
  for lib in "$@"; do
    timeout -k 10 120 python tools/ab_table.py --one $lib --reps 300 2>/dev/null || exit 1
  done
done
