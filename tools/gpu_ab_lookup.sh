#!/bin/bash
# A/B of table-lookup builds: 1e6 cfg3 queries on the cfg2 table (tools/lookup_order_probe.py,
# random order line), alternating builds over 3 rounds.  An argument is a libairice.so (run with
# this tree's Python package) or a directory holding another tree's package, tests/ and tools/
# (a build whose Python binding differs, e.g. another pack format).
#   tools/gpu_ab_lookup.sh lib1.so dir2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for round in 1 2 3; do
  for b in "$@"; do
    if [ -d "$b" ]; then
      (cd $b && timeout -k 10 120 python tools/lookup_order_probe.py --random-only 2>/dev/null) | sed "s|^|$b |" || exit 1
    else
      AB_LIB=$b timeout -k 10 120 python tools/lookup_order_probe.py --random-only 2>/dev/null | sed "s|^|$b |" || exit 1
    fi
  done
done
