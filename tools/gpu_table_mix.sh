#!/bin/bash
# PMC instruction mix and wait profile of the cfg2 table kernel (three separate --pmc passes over
# a short bench run).  Writes gpurun_out/tmix/*.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/tmix
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
A="SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVES"
B="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU SQ_INSTS_SMEM"
for p in a b c; do
  [ $p = a ] && ctr="$A"; [ $p = b ] && ctr="$B"; [ $p = c ] && ctr="$C"
  timeout -k 10 200 rocprofv3 --pmc $ctr -d $OUT/$p -o $p --output-format csv -- \
    python $R/bench.py --no-cpu --no-multi --no-scalar --no-cfg4 --no-default-grid --no-solve --no-lookup --no-trace --no-pcie --steps 3 --warmup 1 > $OUT/$p.log 2>&1 \
    || { echo "pass $p failed"; tail -5 $OUT/$p.log; exit 1; }
done
python $R/tools/pmc_summarize.py $OUT/mix.json $OUT/a $OUT/b $OUT/c | grep table_kernel
