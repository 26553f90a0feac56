set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
python -c "
import json;d=json.load(open('gpurun_out/bench.json'));x=d['detail'];print(d['value'], d['ms_per_step'], d['roofline'], x['full_candidates']['value'], x['decode']['value'], x['cdc_mode']['value'], x['lz77'])"
