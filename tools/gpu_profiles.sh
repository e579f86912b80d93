#!/bin/bash
# Round evidence, one GPU session: the default bench line, then rocprofv3 --kernel-trace --stats
# of each workload on its own (bench.py --only ITEM: the headline table steps + that item;
# --cfg4-only; the scalar latency driver), so that every line item's kernel time can be read
# from its own stats file.  tools/collect_profiles.py ROUND copies them into profiles/.
#   tools/gpu_profiles.sh [OUTDIR]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/prof}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench.err; exit 1; }
head -c 300 $OUT/bench.json; echo
cd /tmp
for item in table solve trace lookup; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$item -o $item --output-format csv -- \
    python $R/bench.py --only $item > $OUT/prof_$item.json 2> $OUT/prof_$item.err \
    || { echo "rocprof $item failed rc=$?"; tail -5 $OUT/prof_$item.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_cfg4 -o cfg4 --output-format csv -- \
  python $R/bench.py --cfg4-only --cfg4-reps 9 --no-cpu > $OUT/prof_cfg4.json 2> $OUT/prof_cfg4.err \
  || { echo "rocprof cfg4 failed rc=$?"; tail -5 $OUT/prof_cfg4.err; exit 1; }
mkdir -p /tmp/scalar_prof && gunzip -c $R/airiceraytracing_amd/data/Atmosphere.dat.gz > /tmp/scalar_prof/Atmosphere.dat
cd /tmp/scalar_prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_scalar -o scalar --output-format csv -- \
  $R/tests/cpp/latency_driver > $OUT/prof_scalar.json 2> $OUT/prof_scalar.err \
  || { echo "rocprof scalar failed rc=$?"; tail -5 $OUT/prof_scalar.err; exit 1; }
find $OUT -name "*kernel_stats.csv" | sort
