#!/bin/bash
# Re-Pair A/B step on the GPU box: parity tests of candidate 9, then traces (tools/rp_trace.py).
OUT=${1:-gpurun_out/rp}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_decode.py -k "repair" -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
( timeout -k 10 120 python tools/rp_trace.py run $OUT 1 enwik && timeout -k 10 120 python tools/rp_trace.py run $OUT 64 enwik && timeout -k 10 120 python tools/rp_trace.py run $OUT 256 enwik && timeout -k 10 120 python tools/rp_trace.py run $OUT 1 gradient ) > $OUT/trace.log 2>&1 || { tail -30 $OUT/trace.log; exit 1; }
grep -E "ms_repair|section ms" $OUT/trace.log
