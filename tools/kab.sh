# A/B of environment settings in one GPU call, printing step time and chosen kernels' ms/step:
#   KERNELS="k_r0_final k_lsd" bash tools/kab.sh "ENV1=a" "ENV1=b" ...
# (each setting twice, alternating; 256 MiB bench, hot path only)
set -o pipefail
export KOLM_BENCH_ALLK=1
mkdir -p gpurun_out
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 --no-serial-pass > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || exit 1
    python -c "
import json,os;d=json.load(open('gpurun_out/ab_$i.json'));k=d['detail'].get('kernels_all_ms_per_step') or d['detail']['kernels_ms_per_step']
ks=os.environ.get('KERNELS','').split()
print('[$cfg]', d['value'], d['ms_per_step'], {n:v for n,v in k.items() if any(n.startswith(x) for x in ks)})"
  done
done
