#!/bin/bash
# round 3: kernel durations of the scalar calls (latency driver under rocprofv3), the root
# finder's guard-skip / overshoot variants, and the evaluation-count statistics
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
mkdir -p /tmp/lat && python -c "import gzip,shutil;shutil.copyfileobj(gzip.open('airiceraytracing_amd/data/Atmosphere.dat.gz'),open('/tmp/lat/Atmosphere.dat','wb'))" || exit 1
(cd /tmp/lat && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/lat_prof -o lat --output-format csv -- $R/tests/cpp/latency_driver) > gpurun_out/lat_prof.log 2>&1; rc=$?; echo "latprof rc=$rc"
[ $rc -eq 0 ] || exit 1
bash tools/gpu_ab_solve.sh ab/base.so ab/gskip.so ab/oshoot.so ab/both.so > gpurun_out/ab_guard.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab_guard.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python tools/solve_stats.py > gpurun_out/solve_stats.log 2>&1; echo "stats rc=$?"; cat gpurun_out/solve_stats.log
