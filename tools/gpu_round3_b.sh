#!/bin/bash
# round 3: PMC passes of the current build, then the table micro-option A/B (with oracle parity)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu_pmc.sh > gpurun_out/pmc_run.log 2>&1; echo "pmc rc=$?"
AB_PARITY=1 bash tools/gpu_ab_tables.sh ab/t_base.so ab/t_s.so ab/t_sq.so ab/t_sqi.so ab/t_sqic.so > gpurun_out/ab_tables.log 2>&1; echo "ab rc=$?"
