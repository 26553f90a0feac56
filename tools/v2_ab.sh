# v2_new leg (ids 0..10 on 32 MiB) under environment settings: bash tools/v2_ab.sh "ENV=a" "ENV=b" ...
set -o pipefail
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 2 > gpurun_out/v2ab.json 2> gpurun_out/v2ab.err || { tail -5 gpurun_out/v2ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/v2ab.json'));print('[$cfg]', d['detail']['v2_new'])"
done
