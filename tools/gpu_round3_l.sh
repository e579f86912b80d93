#!/bin/bash
# round 3: the lookup's two rows searched side by side -- order probe A/B, lookup + compat tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for round in 1 2; do for v in lk0 lk1; do AB_LIB=ab/$v.so timeout -k 10 300 python tools/lookup_order_probe.py 2>&1 | grep -v amdgpu.ids > gpurun_out/lkp_${v}_$round.log; rc=$?; echo "$v rc=$rc"; head -3 gpurun_out/lkp_${v}_$round.log; [ $rc -eq 0 ] || exit 1; done; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_lookup.py tests/test_gpu_compat.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_l.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_l.log
exit $rc
