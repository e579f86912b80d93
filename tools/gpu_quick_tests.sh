#!/bin/bash
# GPU session: the whole -m gpu suite (one process, per-test timeout) and the scalar-latency driver.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -rf ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1; rc=$?
tail -15 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit 1
mkdir -p /tmp/lat && python -c "import gzip,shutil; shutil.copyfileobj(gzip.open('$R/airiceraytracing_amd/data/Atmosphere.dat.gz'), open('/tmp/lat/Atmosphere.dat','wb'))" && cd /tmp/lat && timeout -k 10 120 $R/tests/cpp/latency_driver > $OUT/latency.json 2> $OUT/latency.err && cat $OUT/latency.json
