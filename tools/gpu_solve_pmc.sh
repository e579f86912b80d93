#!/bin/bash
# PMC instruction mix of the root finder, guarded vs every-midpoint bisection (cfg3, 1e6).
# Writes gpurun_out/spmc/*.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/spmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES"
C2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F64"
for mode in ${SPMC_MODES:-fast exact}; do
  for p in a b; do
    [ $p = a ] && ctr="$C" || ctr="$C2"
    if [ $mode = exact ]; then export AIRICE_BISECT_EXACT=1; else unset AIRICE_BISECT_EXACT; fi
    timeout -k 10 200 rocprofv3 --pmc $ctr -d $OUT/${mode}_$p -o ${mode}_$p --output-format csv -- \
      python $R/tools/solve_stats.py --child $mode 1000000 > $OUT/${mode}_$p.log 2>&1 \
      || { echo "pass ${mode}_$p failed"; tail -5 $OUT/${mode}_$p.log; exit 1; }
  done
  python $R/tools/pmc_summarize.py $OUT/$mode.json $OUT/${mode}_a $OUT/${mode}_b | grep roots
done
