#!/bin/bash
# Hot-path A/B step on the GPU box: BBWT/LZ77 parity subset, per-phase Duval profile, bench line.
OUT=${1:-gpurun_out/hot}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "bbwt or adversarial or large_known or lyndon or multiblock or full_size" -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
KOLM_DUVAL_PROF=1 KOLM_SERIAL=1 timeout -k 10 120 python3 tools/profile_run.py --iters 3 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
grep -E "duval|iter" $OUT/prof.log | tail -2
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench.json'));print('hot', d['value'],d['ms_per_step']);print(d['detail']['kernels_ms_per_step'])"
