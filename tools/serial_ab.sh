mkdir -p gpurun_out/lz3
for L in ab/A.so ab/B.so; do
  KOLM_SERIAL=1 KOLM_LIB=$L timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 > gpurun_out/lz3/b.json 2> gpurun_out/lz3/b.err || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/lz3/b.json'));k=d['detail']['kernels_ms_per_step'];print('$L', d['value'], d['ms_per_step'], {x:v for x,v in k.items() if 'lz' in x})"
done
