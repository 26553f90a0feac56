#!/bin/bash
# Round-6 LZ77 parse forms on the GPU box: parity of every form on the LZ77 / bench-stream tests,
# then alternating quick benches of each form (KOLM_LZ_LANES: 0 = 16-lane chains, 1 = a chain
# per lane 16 KiB homes 11 hash bits, 2 = 10 bits, 3 = 8 KiB homes), SQ counters and phase clocks.
#   bash tools/ab_lz.sh OUT
OUT=${1:-gpurun_out/ablz}
mkdir -p "$OUT"
set -o pipefail
bash tools/gpu_call.sh "$OUT" "tests:lz77+bench_stream+config_shapes+switches+round0+toc_cases+multi" || exit 1
for m in 2 3; do
  KOLM_LZ_LANES=$m timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "lz77_local or bench_stream_lz77 or config_shapes" > "$OUT/tests_lanes$m.log" 2>&1 || { tail -30 "$OUT/tests_lanes$m.log"; exit 1; }
  tail -1 "$OUT/tests_lanes$m.log"
done
for r in 1 2; do
  for m in 0 1 2 3; do bash tools/gpu_call.sh "$OUT" "ab:KOLM_LZ_LANES=$m" || exit 1; done
done
for m in 0 1 3; do
  bash tools/gpu_call.sh "$OUT" "run:solo$m:KOLM_LZ_LANES=$m:--steps,2,--warmup,1,--no-cpu-baseline,--full-steps,0,--decode-steps,0,--cdc-steps,0,--v2-steps,0,--config-steps,0,--host-steps,0,--c4-steps,0" || exit 1
  python3 -c "import json;d=json.load(open('$OUT/run_solo$m.json'));print('solo', $m, d['detail']['lz77_parse'], d['detail']['serialised_step_ms'])"
done
for m in 1 3; do
  KOLM_LZ_LANES=$m bash tools/sq_lz.sh "$OUT/sq$m" k_lz_lanes || exit 1
  KOLM_LZ_LANES=$m KOLM_LZ_PROF=1 timeout -k 10 200 python bench.py --mib 256 --steps 1 --warmup 1 --kt-steps 1 \
    --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 \
    --c4-steps 0 > "$OUT/lzprof$m.json" 2> "$OUT/lzprof$m.err" || { tail -20 "$OUT/lzprof$m.err"; exit 1; }
  grep "k_lz" "$OUT/lzprof$m.err" | head -4
done
