# step time vs batch size (per-GPU MiB): does a smaller working set (L2 / MALL) help?
set -o pipefail
for m in 256 128 64 32 16; do
  timeout -k 10 200 python bench.py --mib $m --steps 6 --warmup 2 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 > gpurun_out/sz_$m.json 2>/dev/null || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/sz_$m.json'));x=d['detail'];print($m, d['value'], d['ms_per_step'], x['device_ms'], list(x['families_ms_per_step'].items())[:6])"
done
