#!/bin/bash
# FETCH_SIZE calibration on the GPU box: tools/fetch_calib (built in-tree
# with hipcc, see its header) timed with HIP events, then one rocprofv3 --pmc pass per counter
# group over the same binary; tools/fetch_calib.py writes gpurun_out/fcal/fetch_calib.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/fcal
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 $R/tools/fetch_calib $OUT/timings.json > $OUT/run.log 2>&1 || { echo "fetch_calib failed"; cat $OUT/run.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/p1 -o p1 --output-format csv -- \
  $R/tools/fetch_calib > $OUT/p1.log 2>&1 || { echo "pass 1 failed"; tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_MISS_sum TCC_REQ_sum -d $OUT/p2 -o p2 --output-format csv -- \
  $R/tools/fetch_calib > $OUT/p2.log 2>&1 || { echo "pass 2 failed (counter names?)"; tail -5 $OUT/p2.log; }
python $R/tools/fetch_calib.py $OUT/fetch_calib.json $OUT/timings.json $OUT/p1 $OUT/p2
