# LZ77 checks + A/B: the LZ-related GPU tests, then bench lines under env settings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lz77 or adversarial or multiblock or edge or smoke or cdc_vs or variable" > gpurun_out/t_lz.log 2>&1 || { tail -30 gpurun_out/t_lz.log; exit 1; }
tail -1 gpurun_out/t_lz.log
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 > gpurun_out/b_$n.json 2>gpurun_out/b_$n.err || return 1
  python -c "
import json;d=json.load(open('gpurun_out/b_$n.json'));x=d['detail'];print('$n', d['value'], d['ms_per_step'], x['lz77'], x['device_ms']['ms_lz'], list(x['kernels_ms_per_step'].items())[:4])"
  grep "k_lz_local us" gpurun_out/b_$n.err | tail -1
}
run serial KOLM_SERIAL=1 KOLM_LZ_PROF=1 || exit 1
run overl KOLM_LZ_PROF=1 || exit 1
run overl2 || exit 1
