set -o pipefail
O=gpurun_out/r04j; mkdir -p $O
bash tools/gpu_ab_tables.sh ab/base.so ab/s_ilp.so ab/s_memc.so > $O/ab_table.log 2>&1 || { cat $O/ab_table.log; exit 1; }
bash tools/gpu_ab_solve.sh ab/base.so ab/s_ilp.so ab/s_memc.so > $O/ab_solve.log 2>&1 || { cat $O/ab_solve.log; exit 1; }
bash tools/gpu_ab_lookup.sh ab/base.so ab/s_ilp.so ab/s_memc.so > $O/ab_lookup.log 2>&1 || { cat $O/ab_lookup.log; exit 1; }
cat $O/ab_table.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['lib'], round(d['ms']*1e3,2), d['sha1'][:10])"
cat $O/ab_solve.log $O/ab_lookup.log
