#!/bin/bash
# GPU session: full -m gpu suite, smoke, torchrun bench rehearsal (1 rank nccl, 2 ranks gloo).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider -rA > $OUT/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
grep -E "passed|failed" $OUT/gpu_tests.log | tail -3
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu --solve-n 100000 > $OUT/torchrun1.json 2> $OUT/torchrun1.err || { echo torchrun1 failed; tail $OUT/torchrun1.err; exit 1; }
head -c 400 $OUT/torchrun1.json; echo
AIRICE_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --solve-n 100000 > $OUT/torchrun2.json 2> $OUT/torchrun2.err || { echo torchrun2 failed; tail $OUT/torchrun2.err; exit 1; }
head -c 400 $OUT/torchrun2.json; echo
