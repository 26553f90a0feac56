#!/bin/bash
# Round-end evidence on one GPU box: GPU tests, the default bench line, rocprofv3 kernel
# stats (overlapped and serialised streams) and the PMC traffic passes (one counter set per
# rocprofv3 run, kernel-trace domain only).  OUT defaults to gpurun_out/final.
OUT=${1:-gpurun_out/final}
ARGS="--mib 256 --steps 1 --warmup 1 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0"
mkdir -p $OUT
export TMPDIR=/tmp
( for i in $(seq 1 90); do sleep 20; echo "tick $i" >> $OUT/ticks.txt; done ) &
TICK=$!
trap "kill $TICK 2>/dev/null" EXIT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py $ARGS > $OUT/kt.log 2>&1 || exit 1
KOLM_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kts -o kt --output-format csv -- python3 bench.py $ARGS > $OUT/kts.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/hit -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/hit.log 2>&1 || exit 1
python3 tools/pmc_traffic.py $OUT > $OUT/pmc_summary.json
echo final done
