#!/bin/bash
# round 3: the lookup's fallback pass fused into one 256-lane kernel -- lookup tests, then A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lookup.py tests/test_gpu_compat.py tests/test_gpu_scalar_wave.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_n.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_n.log
[ $rc -eq 0 ] || exit 1
for round in 1 2; do for v in fb0 fb1; do AB_LIB=ab/$v.so timeout -k 10 300 python tools/lookup_order_probe.py --random-only 2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/$v /"; done; done
