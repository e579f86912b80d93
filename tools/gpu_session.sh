#!/bin/bash
# One GPU session: the -m gpu suite, a table A/B of library builds (tools/ab_table.py) and a
# default bench.py run.  Usage: tools/gpu_session.sh TAG [ab_lib.so ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 \
  --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
grep -E "passed|failed|error" $OUT/gpu_tests.log | tail -3
[ $rc -eq 0 ] || exit 1
if [ $# -gt 0 ]; then
  for round in 1 2 3; do
    for lib in "$@"; do
      timeout -k 10 120 python tools/ab_table.py --one $lib --reps 300 >> $OUT/ab.log 2>/dev/null || exit 1
    done
  done
  cat $OUT/ab.log
fi
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
head -c 600 $OUT/bench.json; echo
