#!/bin/bash
# A/B of minimizer builds: cfg3 1e6 solves, alternating libraries (tools/solve_stats.py child).
#   tools/gpu_ab_solve.sh lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for round in 1 2 3; do
  for lib in "$@"; do
    AB_LIB=$lib timeout -k 10 120 python tools/solve_stats.py --child fast 1000000 2>/dev/null | sed "s|^|$lib |" || exit 1
  done
done
