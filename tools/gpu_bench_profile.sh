#!/bin/bash
# One GPU session: bench line, kernel-trace stats of the same command, counter list.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp
# --no-multi: the several-antenna item runs table_kernel on concurrent streams, which would skew
# the per-launch table_kernel average that collect_profiles.py checks against the headline.
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python $R/bench.py --no-cpu --no-multi --no-scalar > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof.err; exit 1; }
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
find $OUT/prof -name "*stats*" | head
