#!/bin/bash
# GPU session: parity tests + bench line (+ kernel stats) for an iteration.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider -rA -s > $OUT/gpu_tests.log 2>&1; rc=$?
grep -E "^\.*\[|passed|failed" $OUT/gpu_tests.log | sed 's/^\.*//' | tail -15
[ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/gpu_tests.log | head -20; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench.json'))
print('value %.4g rays/s  kernel_ms %.4f  frac %.3f  minimizer %.4g solves/s (%.3f ms)' % (d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['minimizer']['value'], d['minimizer']['kernel_ms']))
print('parity', d['parity_vs_cpu'], 'cpu', d['cpu_baseline']['value'])"
