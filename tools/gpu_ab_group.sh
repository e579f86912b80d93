#!/bin/bash
# A/B of the batch-wide minimizer grouping: each library with AIRICE_GROUP_MIN=0 (block-local
# roots_kernel) and its built-in threshold, cfg3 1e6 solves, alternating order.
#   tools/gpu_ab_group.sh lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for round in 1 2 3; do
  for lib in "$@"; do
    for g in 0 default; do
      if [ $g = 0 ]; then export AIRICE_GROUP_MIN=0; else unset AIRICE_GROUP_MIN; fi
      AB_LIB=$lib timeout -k 10 120 python tools/solve_stats.py --child fast 1000000 2>/dev/null | sed "s|^|$lib G=$g |" || exit 1
    done
  done
done
