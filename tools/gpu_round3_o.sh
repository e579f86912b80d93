#!/bin/bash
# round 3: lookup_kernel occupancy (6 / 7 / 8 waves per SIMD) -- order-probe A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for round in 1 2; do for v in lw0 lw7 lw8; do AB_LIB=ab/$v.so timeout -k 10 300 python tools/lookup_order_probe.py 2>&1 | grep -v amdgpu.ids | head -2 | tr '\n' ' ' | sed "s/^/$v /"; echo; done; done
