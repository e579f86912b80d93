#!/bin/bash
# Cache counters of the table lookup (bench.py --only lookup: 1e6 random cfg3 queries on the cfg2
# table), one rocprofv3 --pmc pass per counter group: L1->L2 read requests and L1 accesses (TCP),
# L2 requests, hits, misses and fabric reads (TCC).  Writes gpurun_out/lkpmc/lookup_cache.json.
# With a library argument (tools/gpu_lookup_pmc.sh lib.so) the 1e6 queries of
# tools/lookup_order_probe.py --random-only on that build: gpurun_out/lkpmc/<lib>.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/lkpmc
LIB=$1
NAME=lookup_cache
[ -n "$LIB" ] && NAME=$(basename $LIB .so)
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
P1="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum"
P2="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM_RD SQ_WAVES"
for p in 1 2; do
  [ $p = 1 ] && ctr="$P1" || ctr="$P2"
  if [ -n "$LIB" ]; then
    AB_LIB=$R/$LIB timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/${NAME}_p$p -o p$p --output-format csv -- \
      python $R/tools/lookup_order_probe.py --random-only > $OUT/${NAME}_p$p.log 2>&1 || { echo "pass $p failed"; tail -5 $OUT/${NAME}_p$p.log; exit 1; }
  else
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/${NAME}_p$p -o p$p --output-format csv -- \
      python $R/bench.py --only lookup --no-cpu > $OUT/${NAME}_p$p.log 2>&1 || { echo "pass $p failed"; tail -5 $OUT/${NAME}_p$p.log; exit 1; }
  fi
done
python $R/tools/pmc_summarize.py $OUT/$NAME.json $OUT/${NAME}_p1 $OUT/${NAME}_p2 | grep -i "lookup"
