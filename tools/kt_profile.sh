#!/bin/bash
# Kernel-trace profile of the bench workload (rocprofv3 --kernel-trace --stats only) + per-stream timeline.
OUT=${1:-gpurun_out/kt}
ARGS=${2:-"--steps 2 --warmup 1 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0"}
mkdir -p $OUT
export TMPDIR=/tmp
( for i in $(seq 1 40); do sleep 20; echo "tick $i" >> $OUT/ticks.txt; done ) &
TICK=$!
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py $ARGS > $OUT/kt.log 2>&1
RC=$?
kill $TICK 2>/dev/null
[ $RC -eq 0 ] || { tail -20 $OUT/kt.log; exit $RC; }
F=$(find $OUT/kt -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py $F > $OUT/timeline.txt 2>&1
S=$(find $OUT/kt -name "*kernel_stats.csv" | head -1)
cp $S $OUT/kernel_stats.csv
echo profile done
