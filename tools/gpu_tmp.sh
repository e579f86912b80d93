set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_cfg4.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --only cfg4 > $O/cfg4.json 2>$O/cfg4.err || { tail $O/cfg4.err; exit 1; }
python -c "import json;d=json.loads(open('$O/cfg4.json').read());c=d['table_cfg4'];print(c['first_build_ms'],c['ms_per_build'],c['kernel_ms'])"
