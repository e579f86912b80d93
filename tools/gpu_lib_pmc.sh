#!/bin/bash
# PMC passes of the cfg3 solve (tools/solve_stats.py --child, 1e6 queries) for library builds:
# wave-cycle decomposition and instruction mix.  tools/gpu_lib_pmc.sh OUTDIR lib1.so [lib2.so ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
PA="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
PB="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES"
for lib in "$@"; do
  name=$(basename $lib .so)
  for p in a b; do
    [ $p = a ] && ctr="$PA" || ctr="$PB"
    (cd /tmp && AB_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/${name}_$p -o ${name}_$p --output-format csv -- \
      python $R/tools/solve_stats.py --child $name 1000000 > $OUT/${name}_$p.log 2>&1) \
      || { echo "pass ${name}_$p failed"; tail -5 $OUT/${name}_$p.log; exit 1; }
  done
  python $R/tools/pmc_summarize.py $OUT/$name.json $OUT/${name}_a $OUT/${name}_b | grep "roots_sorted"
done
