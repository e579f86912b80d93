#!/bin/bash
# round 3: scalar latencies after the sync change, then the PMC passes of the current kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
mkdir -p /tmp/lat && python -c "import gzip,shutil;shutil.copyfileobj(gzip.open('airiceraytracing_amd/data/Atmosphere.dat.gz'),open('/tmp/lat/Atmosphere.dat','wb'))" && (cd /tmp/lat && timeout -k 10 120 $R/tests/cpp/latency_driver) > gpurun_out/latency.json 2>gpurun_out/latency.err; echo "lat rc=$?"; tail -1 gpurun_out/latency.json
bash $R/tools/gpu_pmc.sh > gpurun_out/pmc_run.log 2>&1; rc=$?; echo "pmc rc=$rc"; tail -5 gpurun_out/pmc_run.log
exit $rc
