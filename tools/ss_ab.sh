# serial kernel times of two builds (small-sort experiment)
set -o pipefail
for L in ab/A.so ab/B.so; do
  KOLM_SERIAL=1 KOLM_LIB=$L timeout -k 10 200 python bench.py --steps 4 --warmup 2 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 > gpurun_out/ss.json 2>/dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/ss.json'));k=d['detail']['kernels_ms_per_step'];f=d['detail']['families_ms_per_step'];print('$L', d['value'], d['ms_per_step'], f.get('small_sort'), {x:v for x,v in k.items() if 'small' in x})"
done
