#!/bin/bash
# round 3: inverse quadratic interpolation in the secant search -- A/B + evaluation counts
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu_ab_solve.sh ab/base.so ab/iqi1.so ab/iqi2.so > gpurun_out/ab_iqi.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab_iqi.log
[ $rc -eq 0 ] || exit 1
for v in iqi1 iqi2; do AB_LIB=ab/$v.so timeout -k 10 300 python tools/solve_stats.py 2>&1 | grep -v amdgpu.ids | head -4 > gpurun_out/stats_$v.log; echo "$v rc=$?"; cat gpurun_out/stats_$v.log; done
