#!/bin/bash
# GPU check after a kernel change: primitive + parity + replay tests, then a short bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/gpu_tests.log | head -80; exit 1; }
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --cpu-seconds 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
wc -l gpurun_out/bench.json
python -c "
import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['minimizer']['value'], d['pywrapper_trace'], d['table_lookup']['value'])"
