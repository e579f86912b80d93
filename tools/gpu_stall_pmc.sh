#!/bin/bash
# Stall attribution for the table kernel: PMC passes (each --pmc pass alone, no tracing domains)
# over tools/ab_table.py --one (cfg2, the repo's libairice.so).  Writes gpurun_out/stall/*.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stall
LIB=${1:-$R/airiceraytracing_amd/libairice.so}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
run() { # name, counters
  timeout -k 10 200 rocprofv3 --pmc $2 -d $OUT/$1 -o $1 --output-format csv -- \
    python $R/tools/ab_table.py --one $LIB --reps 20 > $OUT/$1.log 2>&1 \
    || { echo "pass $1 failed rc=$?"; tail -5 $OUT/$1.log; return 1; }
}
run s1 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" && \
run s2 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES" && \
run s3 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM" && \
run s4 "SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH SQ_IFETCH" && \
run s5 "SQ_INST_CYCLES_SMEM SQ_INSTS_VSKIPPED SQ_LEVEL_WAVES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_INSTS_VALU_TRANS_F64" && \
python $R/tools/pmc_summarize.py $OUT/stall_pmc.json $OUT/s1 $OUT/s2 $OUT/s3 $OUT/s4 $OUT/s5
