# A/B of environment settings in one GPU call: bash tools/env_ab.sh "ENV1=a ENV2=b" "ENV1=c" ...
# (each setting twice, alternating; 256 MiB bench, hot path only)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 --no-serial-pass > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));print('[$cfg]', d['value'], d['ms_per_step'], d['detail']['families_ms_per_step'])"
  done
done
