# overlap placement of the LZ77 parse (KOLM_OVERLAP 0 = at once, 1 = after Lyndon, 2 = after
# round 0, default) and stream priorities (KOLM_PRIO=0: equal)
set -o pipefail
for r in 1 2; do for cfg in "KOLM_OVERLAP=0" "KOLM_OVERLAP=1" "KOLM_OVERLAP=2" "KOLM_OVERLAP=0 KOLM_PRIO=0" "KOLM_OVERLAP=2 KOLM_PRIO=0"; do
  env $cfg timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 > gpurun_out/ov.json 2>/dev/null || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/ov.json'));print('$cfg', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done
