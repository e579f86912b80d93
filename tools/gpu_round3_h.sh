#!/bin/bash
# round 3 evidence: PMC passes of the current kernels, then the bench line (roofline from the new
# PMC summary), the rocprofv3 kernel-trace summary of the same workload, and the GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash $R/tools/gpu_pmc.sh > gpurun_out/pmc_run.log 2>&1; rc=$?; echo "pmc rc=$rc"; tail -3 gpurun_out/pmc_run.log
[ $rc -eq 0 ] || exit 1
cp gpurun_out/pmc/pmc_summary.json profiles/pmc_summary.json || exit 1
bash $R/tools/gpu_bench_profile.sh > gpurun_out/bench_profile.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench_profile.log
[ $rc -eq 0 ] || exit 1
cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
exit $rc
