#!/bin/bash
# round 3: grouping by path span A/B; RTF two-lane ends (latency + bit-exact tests)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu_ab_solve.sh ab/base.so ab/span.so ab/span16.so ab/a16.so > gpurun_out/ab_span.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab_span.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_rtf.py tests/test_gpu_compat.py tests/test_gpu_pywrapper_cpp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_g.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_g.log
[ $rc -eq 0 ] || exit 1
mkdir -p /tmp/lat && python -c "import gzip,shutil;shutil.copyfileobj(gzip.open('airiceraytracing_amd/data/Atmosphere.dat.gz'),open('/tmp/lat/Atmosphere.dat','wb'))" && (cd /tmp/lat && timeout -k 10 120 $R/tests/cpp/latency_driver) > gpurun_out/latency.json 2>gpurun_out/latency.err; echo "lat rc=$?"; tail -1 gpurun_out/latency.json
