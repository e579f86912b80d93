#!/bin/bash
# A/B of minimizer library builds on cfg3 (1e6 solves, tools/solve_stats.py --child: whole
# solve call time and the sha1 of outputs + status), alternating order over 3 rounds.
#   tools/gpu_ab_solve.sh lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for round in 1 2 3; do
  for lib in "$@"; do
    AB_LIB=$lib timeout -k 10 120 python tools/solve_stats.py --child $(basename $lib .so) 1000000 2>/dev/null || exit 1
  done
done
