set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lz77 or adversarial or multiblock or full_size or edge or smoke or container_golden or cdc" > gpurun_out/t_lz.log 2>&1 || { tail -30 gpurun_out/t_lz.log; exit 1; }
tail -2 gpurun_out/t_lz.log
for v in 1 0 1 0; do KOLM_LZ_LOCAL=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 > gpurun_out/b_$v.json 2>/dev/null || exit 1; python -c "
import json;d=json.load(open('gpurun_out/b_$v.json'));x=d['detail'];print('local=$v', d['value'], d['ms_per_step'], x['lz77'], x['device_ms'], list(x['kernels_ms_per_step'].items())[:6])"; done
