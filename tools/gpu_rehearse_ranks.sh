#!/bin/bash
# Multi-rank rehearsal of the driver's scaling bench on one GPU: N ranks share cuda:0 over gloo
# (RCCL refuses two ranks on one device); every line item runs, cfg4 host assembly included, with
# the CPU parity legs (shortened CPU baselines).
#   tools/gpu_rehearse_ranks.sh N TAG [bench.py args...]     (e.g. 4 cfg4 --workload cfg4)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-4}
TAG=${2:-cfg2}
shift 2
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/rehearse${N}_${TAG}
AIRICE_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus $N --steps 5 --warmup 2 --cpu-seconds 2 "$@" \
  > $OUT.json 2> $OUT.err || { echo "rehearsal N=$N $TAG failed"; grep -v Warn $OUT.err | tail -30; exit 1; }
python - <<PY
import json
d = json.load(open("$OUT.json"))
print({k: d.get(k) for k in ("value", "n_gpus", "ms_per_step", "scaling", "rccl_world_size",
                             "dist_backend", "kernel_ms_per_rank", "data")})
print("sharded:", {k: v for k, v in (d.get("sharded") or {}).items() if not isinstance(v, (dict, list))})
t = d.get("table_cfg4") or {}
print("cfg4:", {k: t.get(k) for k in ("value", "assemble", "assemble_ms", "assemble_GBps",
                                       "host_assembly_error", "kernel_ms_per_rank", "parity_vs_cpu")})
PY
