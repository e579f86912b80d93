#!/bin/bash
# Multi-rank rehearsal of the driver's scaling bench on one GPU: N ranks share cuda:0 over gloo
# (RCCL refuses two ranks on one device); every line item runs, cfg4 host assembly included.
#   tools/gpu_rehearse_ranks.sh N
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-4}
cd $R && mkdir -p gpurun_out
AIRICE_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus $N --steps 5 --warmup 2 --no-cpu \
  > gpurun_out/rehearse$N.json 2> gpurun_out/rehearse$N.err || { echo "rehearsal N=$N failed"; grep -v Warn gpurun_out/rehearse$N.err | tail -30; exit 1; }
python - <<PY
import json
d = json.load(open("gpurun_out/rehearse$N.json"))
print({k: d[k] for k in ("value", "n_gpus", "ms_per_step", "scaling")})
print("sharded:", {k: v for k, v in (d.get("sharded") or {}).items() if not isinstance(v, (dict, list))})
t = d.get("table_cfg4") or {}
print("cfg4:", {k: t.get(k) for k in ("value", "assemble", "assemble_ms", "assemble_GBps", "host_assembly_error", "parity_vs_cpu")})
PY
