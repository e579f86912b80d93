#!/bin/bash
# PMC passes (separate runs, --pmc only with --kernel-trace/--stats-free collection) for the
# bench kernels and the ocml op-weight micro-kernels.  Writes gpurun_out/pmc/*.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o /tmp/opweights_bench $R/tools/opweights_bench.hip || exit 1
cd /tmp
P1="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES"
P2="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
run() { # name, counters, cmd...
  local name=$1; shift; local ctr=$1; shift
  timeout -k 10 300 rocprofv3 --pmc $ctr -d $OUT/$name -o $name --output-format csv -- "$@" > $OUT/$name.log 2>&1 || { echo "pass $name failed rc=$?"; tail -5 $OUT/$name.log; return 1; }
}
run ow_a "$P1" /tmp/opweights_bench && \
run bench_a "$P1" python $R/bench.py --no-cpu --no-multi --no-scalar --no-cfg4 --no-default-grid --steps 3 --warmup 1 --solve-steps 1 && \
run bench_b "$P2" python $R/bench.py --no-cpu --no-multi --no-scalar --no-cfg4 --no-default-grid --steps 3 --warmup 1 --solve-steps 1 && \
run bench_w "WRITE_SIZE" python $R/bench.py --no-cpu --no-multi --no-scalar --no-cfg4 --no-default-grid --steps 3 --warmup 1 --solve-steps 1 && \
run bench_f "FETCH_SIZE" python $R/bench.py --no-cpu --no-multi --no-scalar --no-cfg4 --no-default-grid --steps 3 --warmup 1 --solve-steps 1 && \
run cfg4_a "$P1" python $R/bench.py --cfg4-only --cfg4-reps 1 --cfg4-host none --no-cpu && \
run cfg4_b "$P2" python $R/bench.py --cfg4-only --cfg4-reps 1 --cfg4-host none --no-cpu && \
run cfg4_w "WRITE_SIZE" python $R/bench.py --cfg4-only --cfg4-reps 1 --cfg4-host none --no-cpu && \
run cfg4_f "FETCH_SIZE" python $R/bench.py --cfg4-only --cfg4-reps 1 --cfg4-host none --no-cpu && \
python $R/tools/pmc_summarize.py $OUT/opweights_pmc.json $OUT/ow_a && \
python $R/tools/pmc_summarize.py $OUT/cfg4_pmc.json $OUT/cfg4_a $OUT/cfg4_b $OUT/cfg4_w $OUT/cfg4_f && \
python $R/tools/pmc_summarize.py $OUT/bench_pmc.json $OUT/bench_a $OUT/bench_b $OUT/bench_w $OUT/bench_f && \
python $R/tools/make_pmc_summary.py $OUT/bench_pmc.json $OUT/pmc_summary.json $OUT/cfg4_pmc.json > /dev/null
