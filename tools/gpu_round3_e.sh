#!/bin/bash
# round 3: scalar latencies, minimizer A/B (paired evaluations), bisect replay + parity tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
mkdir -p /tmp/lat && python -c "import gzip,shutil;shutil.copyfileobj(gzip.open('airiceraytracing_amd/data/Atmosphere.dat.gz'),open('/tmp/lat/Atmosphere.dat','wb'))" && (cd /tmp/lat && timeout -k 10 120 $R/tests/cpp/latency_driver) > gpurun_out/latency.json 2>gpurun_out/latency.err; echo "lat rc=$?"; tail -1 gpurun_out/latency.json
bash tools/gpu_ab_solve.sh ab/pair0.so ab/pair1.so ab/pair2.so > gpurun_out/ab_pair.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab_pair.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_bisect_replay.py tests/test_gpu_parity.py tests/test_gpu_scalar_wave.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_e.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_e.log
exit $rc
