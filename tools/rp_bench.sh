#!/bin/bash
# Re-Pair A/B on the GPU box: parity tests of candidate 9, 256-block trace, full bench line.
OUT=${1:-gpurun_out/rp}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_decode.py -k "repair" -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
( timeout -k 10 120 python tools/rp_trace.py run $OUT 1 enwik && timeout -k 10 120 python tools/rp_trace.py run $OUT 256 enwik ) > $OUT/trace.log 2>&1 || { tail -30 $OUT/trace.log; exit 1; }
grep -E "ms_repair" $OUT/trace.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --cdc-steps 0 --v2-steps 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench.json'));print('hot', d['value'],d['ms_per_step']);f=d['detail']['full_candidates'];print('full', f['value'], 'repair ms', f['ms_repair'], 'step ms', f['ms_per_step'], 'decode', f['decode']['value'])"
