set -o pipefail
mkdir -p gpurun_out
AB_PARITY=1 bash tools/gpu_ab_env.sh "-20000,300000,20,92,180,0.5" "1" "$@" > gpurun_out/ab5.log 2>&1; rc=$?
grep -o '"lib": "[^"]*", "ms": [0-9.]*\|max_ulps": [0-9]*\|full_max_rel": [0-9.e-]*' gpurun_out/ab5.log | paste - - -
exit $rc
