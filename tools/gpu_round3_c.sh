#!/bin/bash
# round 3: GPU tests, scalar latencies, a short bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit 1
mkdir -p /tmp/lat && python -c "import gzip,shutil;shutil.copyfileobj(gzip.open('airiceraytracing_amd/data/Atmosphere.dat.gz'),open('/tmp/lat/Atmosphere.dat','wb'))" && (cd /tmp/lat && timeout -k 10 120 $R/tests/cpp/latency_driver) > gpurun_out/latency.json 2>gpurun_out/latency.err; echo "lat rc=$?"; tail -1 gpurun_out/latency.json
timeout -k 10 300 python bench.py --no-cpu --no-cfg4 --no-scalar > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err; echo "bench rc=$?"
