set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pythonwrapper.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pw.log 2>&1 && tail -3 gpurun_out/pw.log &&
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --cpu-seconds 4 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 50 --warmup 5 --no-cpu --no-trace --no-lookup --no-pcie --solve-n 100000 > gpurun_out/tr1.json 2> gpurun_out/tr1.err && cat gpurun_out/tr1.json
