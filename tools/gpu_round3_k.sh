#!/bin/bash
# round 3: IQI search + ice 1/C from the kernel arguments -- A/B against the previous build, then
# the bit-exactness tests of the root finder and the GPU parity suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu_ab_solve.sh ab/base.so ab/new.so > gpurun_out/ab_new.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab_new.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
exit $rc
