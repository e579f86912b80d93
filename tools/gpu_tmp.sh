set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
bash tools/gpu_ab_solve.sh ab/lean1.so ab/bs128.so ab/bs64.so ab/lib_r03.so ab/r03_bs64.so > $O/ab_solve.log 2>&1 || { cat $O/ab_solve.log; exit 1; }
cat $O/ab_solve.log
bash tools/gpu_ab_tables.sh ab/lean1.so ab/a1.so > $O/ab_table.log 2>&1 || { cat $O/ab_table.log; exit 1; }
cat $O/ab_table.log
bash tools/gpu_ab_lookup.sh ab/lean1.so ab/fb_exit.so > $O/ab_lookup.log 2>&1 || { cat $O/ab_lookup.log; exit 1; }
cat $O/ab_lookup.log
