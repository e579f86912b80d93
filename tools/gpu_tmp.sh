set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 300 python bench.py --only cfg4 > $O/cfg4.json 2>$O/cfg4.err || { tail $O/cfg4.err; exit 1; }
python -c "import json;d=json.loads(open('$O/cfg4.json').read());c=d['table_cfg4'];print(c['first_build_ms'],c['new_key_build_ms'],c['ms_per_build'],c['kernel_ms'])"
bash tools/gpu_pmc.sh || exit 1
