#!/bin/bash
# one-wave kernels: argument-block prefetch on/off (one-ray stamps), then the scalar latencies
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in rs_nopf rs_pf; do echo "== $v"; AB_LIB=ab/$v.so timeout -k 10 200 python tools/ray_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1; done
mkdir -p /tmp/lat && python -c "import gzip,shutil;shutil.copyfileobj(gzip.open('airiceraytracing_amd/data/Atmosphere.dat.gz'),open('/tmp/lat/Atmosphere.dat','wb'))" || exit 1
echo "== latency (in-tree build)"; (cd /tmp/lat && timeout -k 10 120 $R/tests/cpp/latency_driver) | tail -1
