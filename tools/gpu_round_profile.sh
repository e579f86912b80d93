#!/bin/bash
# Round evidence in one GPU session: the default bench line (with the CPU baseline), the
# rocprofv3 --kernel-trace --stats summary of the same workload, and the PMC passes.
# Outputs under gpurun_out/; copy into profiles/ with tools/collect_profiles.py <round>.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_bench_profile.sh && bash $R/tools/gpu_pmc.sh
