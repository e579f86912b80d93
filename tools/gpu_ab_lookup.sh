#!/bin/bash
# A/B of table-lookup builds: 1e6 cfg3 queries on the cfg2 table (tools/lookup_order_probe.py,
# random order line), alternating libraries.
#   tools/gpu_ab_lookup.sh lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for round in 1 2 3; do
  for lib in "$@"; do
    AB_LIB=$lib timeout -k 10 120 python tools/lookup_order_probe.py --random-only 2>/dev/null | sed "s|^|$lib |" || exit 1
  done
done
