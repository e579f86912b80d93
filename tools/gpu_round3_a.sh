mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?" >> gpurun_out/gpu_tests.log; tail -2 gpurun_out/gpu_tests.log
bash tools/gpu_ab_solve.sh ab/base.so ab/sorted.so > gpurun_out/ab_solve.log 2>&1; cat gpurun_out/ab_solve.log
timeout -k 10 300 python bench.py --cfg4-only > gpurun_out/cfg4_only.json 2> gpurun_out/cfg4_only.err; echo "cfg4 rc=$?"
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err; echo "bench rc=$?"
