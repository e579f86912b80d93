#!/bin/bash
# round 3: wave-uniform phase dispatch in the root finder (with / without paired guards) -- A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu_ab_solve.sh ab/base.so ab/uni.so ab/unipg.so > gpurun_out/ab_uni.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab_uni.log
exit $rc
