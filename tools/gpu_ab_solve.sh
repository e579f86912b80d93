#!/bin/bash
# A/B of minimizer builds on cfg3 (1e6 solves, tools/solve_stats.py --child: whole solve call
# time and the sha1 of outputs + status), alternating order over 3 rounds.  An argument is a
# libairice.so run with this tree's Python package, optionally with an environment
# (lib.so:VAR=val,VAR=val), or a directory holding another tree's package, tests/ and tools/.
#   tools/gpu_ab_solve.sh lib1.so lib2.so:AIRICE_BISECT_EXACT=1 dir3 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
N=${AB_N:-1000000}
for round in 1 2 3; do
  for spec in "$@"; do
    lib=${spec%%:*}
    envs=""
    [ "$spec" != "$lib" ] && envs=$(echo ${spec#*:} | tr ',' ' ')
    name=$(basename $lib .so)${envs:+[$envs]}
    if [ -d "$lib" ]; then
      (cd $lib && env $envs timeout -k 10 120 python tools/solve_stats.py --child "$name" $N 2>/dev/null) || exit 1
    else
      env $envs AB_LIB=$lib timeout -k 10 120 python tools/solve_stats.py --child "$name" $N 2>/dev/null || exit 1
    fi
  done
done
