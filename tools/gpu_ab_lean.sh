set -o pipefail
mkdir -p gpurun_out
AB_PARITY=1 bash tools/gpu_ab_env.sh "-20000,300000,20,92,180,0.5" "1" ab/c0.so ab/c2.so ab/d1.so ab/d2.so ab/d3.so > gpurun_out/ab4.log 2>&1; rc=$?
grep -o '"lib": "[^"]*", "ms": [0-9.]*\|max_ulps": [0-9]*\|full_max_rel": [0-9.e-]*' gpurun_out/ab4.log | paste - - - 
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; grep -h "max_rel" gpurun_out/gpu_tests.log | head -20; exit $rc
