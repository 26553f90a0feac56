#!/bin/bash
# Round profiling recipe (run on the GPU box from the repo root):
#   kernel-trace stats of the overlapped and of the serialised pipeline + separate PMC passes
#   (FETCH_SIZE / WRITE_SIZE / TCC hit-miss), each its own rocprofv3 invocation, kernel-trace
#   domain only.  The bench runs 3 encode batches (warmup, timed step, kernel-timed step).
OUT=${1:-gpurun_out/prof}
ARGS=${2:-"--mib 256 --steps 1 --warmup 1 --kt-steps 1 --no-serial-pass --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 --c4-steps 0"}
mkdir -p $OUT
export TMPDIR=/tmp
( for i in $(seq 1 60); do sleep 20; echo "tick $i" >> $OUT/ticks.txt; done ) &
TICK=$!
trap "kill $TICK 2>/dev/null" EXIT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py $ARGS > $OUT/kt.log 2>&1 || exit 1
if [ "$3" = "stats" ]; then echo profile done; exit 0; fi  # kernel stats of the overlapped run only
KOLM_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kts -o kts --output-format csv -- python3 bench.py $ARGS > $OUT/kts.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/hit -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/hit.log 2>&1 || exit 1
python3 tools/pmc_traffic.py $OUT 3 > $OUT/pmc_summary.json
echo profile done
