#!/bin/bash
# parity of the LZ77 parse + A/B of two library builds + SQ counters and solo time of the current one
OUT=${1:-gpurun_out/r6f}
mkdir -p "$OUT"
bash tools/gpu_call.sh "$OUT" "tests:lz77+bench_stream+config_shapes+switches+edge_cases+adversarial" || exit 1
bash tools/ab.sh "$OUT" ab/r6_head.so ab/r6_c16.so 2 || exit 1
bash tools/ab.sh "$OUT" ab/r6_lead1.so ab/r6_c16.so 2 || exit 1
bash tools/gpu_call.sh "$OUT" "run:solo:KOLM_SERIAL=0:--steps,2,--warmup,1,--no-cpu-baseline,--full-steps,0,--decode-steps,0,--cdc-steps,0,--v2-steps,0,--config-steps,0,--host-steps,0,--c4-steps,0" || exit 1
python3 -c "import json;d=json.load(open('$OUT/run_solo.json'));print('solo', d['detail']['lz77_parse'])"
bash tools/sq_lz.sh "$OUT/sq" k_lz_local || exit 1
for r in 1 2; do
  for v in 0 1; do
    bash tools/gpu_call.sh "$OUT" "run:cls${v}_$r:KOLM_CLS_STREAMS=$v:--steps,5,--warmup,2,--no-cpu-baseline,--full-steps,0,--decode-steps,0,--cdc-steps,0,--v2-steps,0,--host-steps,0,--no-serial-pass" || exit 1
  done
done
